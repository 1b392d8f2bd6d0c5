// rt_multi.hip — frame assembly of a multi-device context:
//
//   * the row-stripe permutation between a frame and the stacked per-device parts, one kernel in
//     either direction (parts -> frame after the gather; frame -> parts before a blend's scatter);
//   * RCCL, loaded on first use with dlopen: a process that already holds librccl (torch) shares
//     that copy, and a single-GPU host never maps the 570 MB library.
//
// Frame row y lies in stripe s = y / stripe, owned by part p = s % n_parts, at local row
// (s / n_parts) * stripe + y % stripe of that part (rt_part_rows order).  The stacked buffer holds
// n_parts parts of max_rows rows each (part 0 owns the most rows; the others are padded).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>

#include <mutex>

#include "rt_internal.h"

static_assert(RT_NCCL_UINT8 == ncclUint8 && RT_NCCL_INT32 == ncclInt32 && RT_NCCL_FLOAT32 == ncclFloat32,
              "RCCL datatype constants");
static_assert(sizeof(ncclComm_t) == sizeof(void *) && sizeof(ncclResult_t) == sizeof(int), "RCCL handle types");

namespace {

// One block per frame row: the row's bytes move between the frame and its part, as 16-, 4- or
// 1-byte words (whichever the row length and both addresses admit).  HBM-bound: one read, one write.
template <typename T>
__global__ void __launch_bounds__(256) k_stripes(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                 int n_parts, int stripe, int max_rows, size_t row_bytes,
                                                 int to_frame)
{
    const int y = blockIdx.x;
    const int s = y / stripe;
    const size_t part_row = (size_t)(s % n_parts) * (size_t)max_rows + (size_t)(s / n_parts) * stripe + y % stripe;
    const size_t f_off = (size_t)y * row_bytes, p_off = part_row * row_bytes;
    const T *a = reinterpret_cast<const T *>(src + (to_frame ? p_off : f_off));
    T *b = reinterpret_cast<T *>(dst + (to_frame ? f_off : p_off));
    const size_t n = row_bytes / sizeof(T);
    for (size_t i = threadIdx.x; i < n; i += 256) b[i] = a[i];
}

}  // namespace

int rt_launch_stripes(const void *src, void *dst, int H, int n_parts, int stripe, int max_rows, size_t row_bytes,
                      int to_frame, void *stream)
{
    if (H <= 0 || row_bytes == 0) return RT_OK;
    const uintptr_t al = (uintptr_t)src | (uintptr_t)dst | (uintptr_t)row_bytes;
    hipStream_t st = (hipStream_t)stream;
    const uint8_t *s8 = (const uint8_t *)src;
    uint8_t *d8 = (uint8_t *)dst;
    if ((al & 15) == 0)
        hipLaunchKernelGGL(k_stripes<uint4>, dim3(H), dim3(256), 0, st, s8, d8, n_parts, stripe, max_rows, row_bytes, to_frame);
    else if ((al & 3) == 0)
        hipLaunchKernelGGL(k_stripes<uint32_t>, dim3(H), dim3(256), 0, st, s8, d8, n_parts, stripe, max_rows, row_bytes, to_frame);
    else
        hipLaunchKernelGGL(k_stripes<uint8_t>, dim3(H), dim3(256), 0, st, s8, d8, n_parts, stripe, max_rows, row_bytes, to_frame);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_set_error(RT_E_HIP, "k_stripes: %s", hipGetErrorString(e));
    return RT_OK;
}

// ---- RCCL ------------------------------------------------------------------------------------------
static RtRccl g_rccl;
static std::once_flag g_rccl_once;
static char g_rccl_err[256] = "";

const RtRccl *rt_rccl(void)
{
    std::call_once(g_rccl_once, [] {
        // RT_RCCL_LIB: another library with RCCL's entry points (tests/test_rccl_sequence.py loads a
        // recording stub through it to check a frame's call sequence without GPUs)
        const char *lib = getenv("RT_RCCL_LIB");
        void *h = lib && lib[0] ? dlopen(lib, RTLD_NOW | RTLD_LOCAL) : dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h && !(lib && lib[0])) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char *e = dlerror();
            snprintf(g_rccl_err, sizeof g_rccl_err, "dlopen librccl: %s", e ? e : "?");
            return;
        }
        RtRccl r{};
        r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.gather = (decltype(r.gather))dlsym(h, "ncclGather");
        r.scatter = (decltype(r.scatter))dlsym(h, "ncclScatter");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        if (!r.comm_init_all || !r.comm_destroy || !r.gather || !r.scatter || !r.group_start || !r.group_end ||
            !r.error_string) {
            snprintf(g_rccl_err, sizeof g_rccl_err, "librccl lacks ncclGather / ncclScatter / ncclCommInitAll");
            return;
        }
        r.ok = true;
        g_rccl = r;
    });
    return g_rccl.ok ? &g_rccl : nullptr;
}

const char *rt_rccl_error(void) { return g_rccl_err; }

int rt_rccl_try(int rc, const char *what)
{
    if (rc == 0) return RT_OK;
    const RtRccl *R = rt_rccl();
    return rt_set_error(RT_E_HIP, "%s: RCCL error %d (%s)", what, rc, R ? R->error_string(rc) : "?");
}
