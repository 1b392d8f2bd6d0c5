/* A recording stand-in for librccl's entry points used by librt_amd (ncclCommInitAll,
 * ncclCommDestroy, ncclGather, ncclScatter, ncclGroupStart/End, ncclGetErrorString).  Test
 * infrastructure only: tests/test_rccl_sequence.py builds it with gcc, points RT_RCCL_LIB at it and
 * reads back every call in order (stub_count / stub_get) to check a multi-device frame's collective
 * sequence on a CPU.  No data moves. */
#include <stdint.h>
#include <stdlib.h>

enum { OP_INIT = 1, OP_DESTROY, OP_GROUP_START, OP_GROUP_END, OP_GATHER, OP_SCATTER, OP_MARK };

typedef struct stub_rec {
    int32_t op, init, rank, dtype, root, pad;
    uint64_t send, recv, count, stream;
} stub_rec;

typedef struct stub_comm {
    int32_t init, rank, ndev;
} stub_comm;

static stub_rec *g_log;
static int g_n, g_cap, g_inits;

static stub_rec *push(int op)
{
    if (g_n == g_cap) {
        g_cap = g_cap ? 2 * g_cap : 1024;
        g_log = (stub_rec *)realloc(g_log, sizeof(stub_rec) * (size_t)g_cap);
    }
    stub_rec *r = &g_log[g_n++];
    *r = (stub_rec){0};
    r->op = op;
    return r;
}

int ncclCommInitAll(void **comms, int ndev, const int *devlist)
{
    const int id = g_inits++;
    for (int k = 0; k < ndev; k++) {
        stub_comm *c = (stub_comm *)malloc(sizeof *c);
        c->init = id;
        c->rank = k;
        c->ndev = ndev;
        comms[k] = c;
        stub_rec *r = push(OP_INIT);
        r->init = id;
        r->rank = k;
        r->count = (uint64_t)ndev;
        r->root = devlist[k];
    }
    return 0;
}

int ncclCommDestroy(void *comm)
{
    stub_comm *c = (stub_comm *)comm;
    stub_rec *r = push(OP_DESTROY);
    r->init = c->init;
    r->rank = c->rank;
    free(c);
    return 0;
}

static int coll(int op, const void *send, void *recv, size_t count, int dtype, int root, void *comm, void *stream)
{
    const stub_comm *c = (const stub_comm *)comm;
    stub_rec *r = push(op);
    r->init = c->init;
    r->rank = c->rank;
    r->dtype = dtype;
    r->root = root;
    r->send = (uint64_t)(uintptr_t)send;
    r->recv = (uint64_t)(uintptr_t)recv;
    r->count = (uint64_t)count;
    r->stream = (uint64_t)(uintptr_t)stream;
    return 0;
}

int ncclGather(const void *send, void *recv, size_t count, int dtype, int root, void *comm, void *stream)
{
    return coll(OP_GATHER, send, recv, count, dtype, root, comm, stream);
}

int ncclScatter(const void *send, void *recv, size_t count, int dtype, int root, void *comm, void *stream)
{
    return coll(OP_SCATTER, send, recv, count, dtype, root, comm, stream);
}

int ncclGroupStart(void) { push(OP_GROUP_START); return 0; }
int ncclGroupEnd(void) { push(OP_GROUP_END); return 0; }
const char *ncclGetErrorString(int rc) { (void)rc; return "stub"; }

/* the test's own hooks: a trace marker (where the caller launched a device's kernels) and the log */
void stub_mark(int32_t ctx, int32_t device)
{
    stub_rec *r = push(OP_MARK);
    r->init = ctx;
    r->rank = device;
}
int stub_count(void) { return g_n; }
void stub_get(int i, stub_rec *out) { *out = g_log[i]; }
void stub_reset(void) { g_n = 0; g_inits = 0; }
