// rt_api.hip — the C ABI of include/rt.h: context, scene upload, frame orchestration.
//
// rt_trace_frame replaces the body of Raytracer.trace_frame (src/raytracer.ts:308-330): the camera
// state and RaytracerConfig arrive as plain structs, the scene was flattened once by
// rt_upload_scene, the kernels run on this context's GPU, and the ExposureBuffer pixels come back
// in the caller's Float32Array.  A ray that reaches a state where the reference throws a JS Error
// makes the call return RT_E_FAULT (outputs still written, status[] = 2 for those pixels).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <new>
#include <vector>

#include "rt.h"
#include "rt_internal.h"
#include "rt_jsnum.h"

static thread_local char g_err[512] = "";

int rt_set_error(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

extern "C" const char *rt_last_error(void) { return g_err; }
extern "C" int rt_abi_version(void) { return RT_ABI_VERSION; }

#define HIP_TRY(x)                                                                                \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) return rt_set_error(RT_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes)
    {
        if (bytes <= cap) return RT_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (bytes == 0) return RT_OK;
        HIP_TRY(hipMalloc(&p, bytes));
        cap = bytes;
        return RT_OK;
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

struct rt_ctx {
    int device = 0;
    int flags = 0;
    bool bvh_sah = true;             // SAH splits (RT_BVH_SAH=0: median split)
    bool split = true;               // walk pass + test pass (RT_SPLIT=0: fused k_trace)
    int cand_cap = 64;               // candidate nodes per pixel in the split path (RT_CAND_CAP)
    int split_levels = RT_MAX_LEVELS + 1;   // split-path bounce levels (RT_SPLIT_LEVELS)
    int claim_chunk = 1;             // items per queue claim in the short passes (RT_CLAIM_CHUNK)
    int xcd_mask = 0;                // passes claiming per-XCD bands (RT_XCD: 1 walk, 2 first, 4 shade)
    int shade_occ = 3;               // k_shade occupancy variant (RT_SHADE_OCC)
    int cont_group = 8;              // continuation rays per wave (RT_CONT_GROUP): their passes are
                                     // latency-bound, fewer lanes per wave shorten the slowest wave
    int seg = 8;                     // segments per bounce ray, levels >= 1 (RT_SEG: 0/1 off, 2..64)
    int occ = 0;
    int diag = 0;
    hipStream_t stream = nullptr;
    bool has_scene = false;
    bool scatter = false;            // a mirror shade with roughness > 0 is reachable
    RtDevScene scene{};
    RtSceneStore *store = nullptr;   // the resident scene (rt_scene.hip)
    DevBuf b_stat, b_cand, b_cand_n, b_first, b_queue, b_ctr, b_setup, b_dirs, b_rgb, b_hit_e, b_hit_n, b_status, b_counters, b_fault;
    DevBuf b_walk;
    static constexpr int NEV = 256;
    hipEvent_t ev[NEV][2] = {};
    int ev_next = 0, ev_count = 0;
};

static int use_device(rt_ctx *c)
{
    HIP_TRY(hipSetDevice(c->device));
    return RT_OK;
}

extern "C" int rt_create(const rt_create_desc *desc, rt_ctx **out)
{
    if (!out) return rt_set_error(RT_E_INVALID, "rt_create: out is null");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return rt_set_error(RT_E_NODEVICE, "rt_create: no HIP device");
    const int dev = desc ? desc->device : 0;
    if (dev < 0 || dev >= n) return rt_set_error(RT_E_INVALID, "rt_create: device %d of %d", dev, n);
    rt_ctx *c = new (std::nothrow) rt_ctx();
    if (!c) return rt_set_error(RT_E_INVALID, "rt_create: out of memory");
    c->device = dev;
    c->flags = desc ? desc->flags : 0;
    if (const char *e = getenv("RT_NO_CULL"))
        if (e[0] == '1') c->flags |= RT_CREATE_NO_CULL;
    if (const char *e = getenv("RT_BVH_SAH")) c->bvh_sah = atoi(e) != 0;
    if (const char *e = getenv("RT_SPLIT")) c->split = atoi(e) != 0;
    if (c->flags & RT_CREATE_NO_SPLIT) c->split = false;
    if (const char *e = getenv("RT_CAND_CAP")) c->cand_cap = atoi(e) < 1 ? 1 : atoi(e);
    if (const char *e = getenv("RT_XCD")) c->xcd_mask = atoi(e) & 7;
    if (const char *e = getenv("RT_SHADE_OCC")) c->shade_occ = atoi(e);
    if (const char *e = getenv("RT_CLAIM_CHUNK")) c->claim_chunk = atoi(e) < 1 ? 1 : (atoi(e) > 64 ? 64 : atoi(e));
    if (const char *e = getenv("RT_SPLIT_LEVELS")) c->split_levels = atoi(e) < 1 ? 1 : atoi(e);
    if (const char *e = getenv("RT_CONT_GROUP")) c->cont_group = atoi(e) < 1 ? 1 : (atoi(e) > 64 ? 64 : atoi(e));
    if (const char *e = getenv("RT_SEG")) {
        int k = 1;
        while (k < 64 && 2 * k <= atoi(e)) k *= 2;                  // a power of two, at most 64
        c->seg = atoi(e) > 1 ? k : 0;
    }
    if (const char *e = getenv("RT_OCC")) c->occ = atoi(e);
    if (const char *e = getenv("RT_DIAG")) c->diag = atoi(e);     // timing experiments only
    int r = use_device(c);
    if (r == RT_OK && hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        r = rt_set_error(RT_E_HIP, "rt_create: hipStreamCreate failed");
    for (int i = 0; r == RT_OK && i < rt_ctx::NEV; i++)
        if (hipEventCreate(&c->ev[i][0]) != hipSuccess || hipEventCreate(&c->ev[i][1]) != hipSuccess)
            r = rt_set_error(RT_E_HIP, "rt_create: hipEventCreate failed");
    if (r == RT_OK && !(c->store = rt_store_new(c->bvh_sah))) r = rt_set_error(RT_E_INVALID, "rt_create: out of memory");
    if (r == RT_OK) r = c->b_setup.ensure(sizeof(RtFrameSetup));
    if (r == RT_OK) r = c->b_counters.ensure(sizeof(unsigned long long) * CT_N);
    if (r == RT_OK) r = c->b_fault.ensure(sizeof(int));   // ray fault flag
    if (r == RT_OK) r = c->b_ctr.ensure(sizeof(int32_t) * RT_CTR_INTS);
    if (r != RT_OK) {
        rt_destroy(c);
        return r;
    }
    *out = c;
    return RT_OK;
}

extern "C" void rt_destroy(rt_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    rt_store_free(c->store);
    c->store = nullptr;
    DevBuf *bufs[] = {&c->b_stat, &c->b_cand, &c->b_cand_n, &c->b_first, &c->b_queue, &c->b_ctr, &c->b_setup, &c->b_dirs,
                      &c->b_rgb, &c->b_hit_e, &c->b_hit_n, &c->b_status, &c->b_counters, &c->b_fault,
                      &c->b_walk};
    for (DevBuf *b : bufs) b->release();
    for (int i = 0; i < rt_ctx::NEV; i++)
        for (int k = 0; k < 2; k++)
            if (c->ev[i][k]) (void)hipEventDestroy(c->ev[i][k]);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" int rt_upload_scene(rt_ctx *c, const rt_scene_desc *s)
{
    if (!c || !s) return rt_set_error(RT_E_INVALID, "rt_upload_scene: null argument");
    int r = use_device(c);
    if (r != RT_OK) return r;
    c->has_scene = false;
    if ((r = rt_store_upload(c->store, s, false, c->stream, &c->scene, &c->scatter, nullptr)) != RT_OK) return r;
    c->has_scene = true;
    return RT_OK;
}

extern "C" int rt_update_scene(rt_ctx *c, const rt_scene_desc *s, rt_update_stats *stats)
{
    if (!c || !s) return rt_set_error(RT_E_INVALID, "rt_update_scene: null argument");
    int r = use_device(c);
    if (r != RT_OK) return r;
    c->has_scene = false;
    if ((r = rt_store_upload(c->store, s, true, c->stream, &c->scene, &c->scatter, stats)) != RT_OK) return r;
    c->has_scene = true;
    return RT_OK;
}

static int check_frame_args(rt_ctx *c, const rt_camera_desc *cam, const rt_config_desc *cfg)
{
    if (!c || !cam || !cfg) return rt_set_error(RT_E_INVALID, "null argument");
    if (!c->has_scene) return rt_set_error(RT_E_NOSCENE, "no scene uploaded");
    if (cam->width <= 0 || cam->height <= 0 || (long long)cam->width * cam->height > (1ll << 31) / 3)
        return rt_set_error(RT_E_INVALID, "bad screen size %dx%d", cam->width, cam->height);
    if (cfg->default_substance < -1 || cfg->default_substance >= c->scene.n_subs)
        return rt_set_error(RT_E_INVALID, "bad default_substance %d", cfg->default_substance);
    if (cfg->sky_image < 0 || cfg->sky_image > c->scene.n_images)
        return rt_set_error(RT_E_INVALID, "bad sky_image %d (%d images)", cfg->sky_image, c->scene.n_images);
    if (cfg->scatter_mode != RT_SCATTER_REJECT && cfg->scatter_mode != RT_SCATTER_COUNTER)
        return rt_set_error(RT_E_INVALID, "bad scatter_mode %d", cfg->scatter_mode);
    if (c->scatter && cfg->scatter_mode != RT_SCATTER_COUNTER)
        return rt_set_error(RT_E_UNSUPPORTED,
                            "roughness_index > 0 on a mirror: scatter_ray draws from one sequential PRNG "
                            "(src/raytracer.ts:121-133); pass scatter_mode RT_SCATTER_COUNTER for the "
                            "per-pixel counter stream");
    return RT_OK;
}

// Prepare per-frame buffers and the launch description for one part.
static int prepare(rt_ctx *c, const rt_camera_desc *cam, const rt_config_desc *cfg, int part, int n_parts,
                   int stripe, bool want_ids, RtLaunch &L)
{
    const int rows = rt_part_rows(cam->height, part, n_parts, stripe);
    const size_t P = (size_t)rows * (size_t)cam->width;
    int r;
    if ((r = c->b_dirs.ensure(sizeof(double) * 3 * (P ? P : 1))) != RT_OK) return r;
    if (want_ids) {
        if ((r = c->b_hit_e.ensure(sizeof(int32_t) * (P ? P : 1))) != RT_OK) return r;
        if ((r = c->b_hit_n.ensure(sizeof(int32_t) * (P ? P : 1))) != RT_OK) return r;
        if ((r = c->b_status.ensure(P ? P : 1)) != RT_OK) return r;
    }
    memset(&L, 0, sizeof L);
    L.scene = c->scene;
    L.cam = *cam;
    L.cfg = *cfg;
    L.part = part;
    L.n_parts = n_parts;
    L.stripe_rows = stripe;
    L.rows = rows;
    L.setup = (RtFrameSetup *)c->b_setup.p;
    L.dirs = (double *)c->b_dirs.p;
    L.hit_entity = want_ids ? (int32_t *)c->b_hit_e.p : nullptr;
    L.hit_node = want_ids ? (int32_t *)c->b_hit_n.p : nullptr;
    L.status = want_ids ? (uint8_t *)c->b_status.p : nullptr;
    L.fault = (int32_t *)c->b_fault.p;
    L.cull = (c->flags & RT_CREATE_NO_CULL) ? 0 : 1;
    L.ctr = (int32_t *)c->b_ctr.p;
    L.occ = c->occ;
    L.diag = c->diag;
    L.cont_group = c->cont_group;
    L.split_levels = c->split_levels;
    L.claim_chunk = c->claim_chunk;
    L.xcd_mask = c->xcd_mask;
    L.shade_occ = c->shade_occ;
    L.seg = c->seg;
    if (c->split && P > 0) {
        // split path buffers: cand_cap node ids per pixel, k-major.  If they cannot
        // be allocated the frame runs the fused kernel instead (same results).
        L.cand_cap = c->cand_cap;
        if (c->b_cand.ensure(sizeof(int32_t) * (size_t)L.cand_cap * P) == RT_OK &&
            c->b_cand_n.ensure(2 * sizeof(int32_t) * P) == RT_OK && c->b_first.ensure(2 * sizeof(int32_t) * P) == RT_OK &&
            c->b_queue.ensure(3 * sizeof(RtCont) * P) == RT_OK) {
            L.cand = (int32_t *)c->b_cand.p;
            L.cand_n = (int32_t *)c->b_cand_n.p;
            L.ray_cn = L.cand_n + P;
            L.first = (int32_t *)c->b_first.p;
            L.queue[0] = (RtCont *)c->b_queue.p;
            L.queue[1] = L.queue[0] + P;
            L.ovf = L.queue[1] + P;
        } else {
            (void)hipGetLastError();
            L.cand = nullptr;
            L.cand_n = nullptr;
            L.first = nullptr;
        }
    }
    return RT_OK;
}

static void fill_stats(rt_stats *st, const unsigned long long *h)
{
    st->segments = (int64_t)h[CT_SEG]; st->n_ret = (int64_t)h[CT_RET]; st->n_slot = (int64_t)h[CT_SLOT];
    st->n_loc = (int64_t)h[CT_LOC]; st->n_sph = (int64_t)h[CT_SPH]; st->n_box = (int64_t)h[CT_BOX];
    st->n_tri = (int64_t)h[CT_TRI]; st->n_hit = (int64_t)h[CT_HIT]; st->primary = (int64_t)h[CT_PRIM];
    st->n_warn = (int64_t)h[CT_WARN]; st->n_fault = (int64_t)h[CT_FAULT];
    st->n_cull = (int64_t)h[CT_CULL]; st->n_exact = (int64_t)h[CT_EXACT];
}

extern "C" int rt_trace_frame(rt_ctx *c, const rt_camera_desc *cam, const rt_config_desc *cfg, float *rgb_inout,
                              int32_t *hit_entity, int32_t *hit_node, uint8_t *status, rt_stats *stats)
{
    const auto t0 = std::chrono::steady_clock::now();
    int r = check_frame_args(c, cam, cfg);
    if (r != RT_OK) return r;
    if (!rgb_inout) return rt_set_error(RT_E_INVALID, "rt_trace_frame: rgb_inout is null");
    if ((r = use_device(c)) != RT_OK) return r;
    const int H = cam->height;
    const bool ids = hit_entity || hit_node || status;
    RtLaunch L;
    if ((r = prepare(c, cam, cfg, 0, 1, H, ids, L)) != RT_OK) return r;
    const size_t P = (size_t)cam->width * (size_t)H;
    if ((r = c->b_rgb.ensure(sizeof(float) * 3 * P)) != RT_OK) return r;
    L.rgb = (float *)c->b_rgb.p;
    L.blend = cfg->col_weight != 1.0;
    if (L.blend) HIP_TRY(hipMemcpyAsync(L.rgb, rgb_inout, sizeof(float) * 3 * P, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(c->b_fault.p, 0, sizeof(int), c->stream));
    if (stats) {
        HIP_TRY(hipMemsetAsync(c->b_counters.p, 0, sizeof(unsigned long long) * CT_N, c->stream));
        L.counters = (unsigned long long *)c->b_counters.p;
    }
    hipEvent_t *ev = c->ev[c->ev_next];
    if ((r = rt_launch_frame(L, c->stream, ev[0], ev[1])) != RT_OK) return r;
    HIP_TRY(hipMemcpyAsync(rgb_inout, L.rgb, sizeof(float) * 3 * P, hipMemcpyDeviceToHost, c->stream));
    if (hit_entity) HIP_TRY(hipMemcpyAsync(hit_entity, L.hit_entity, sizeof(int32_t) * P, hipMemcpyDeviceToHost, c->stream));
    if (hit_node) HIP_TRY(hipMemcpyAsync(hit_node, L.hit_node, sizeof(int32_t) * P, hipMemcpyDeviceToHost, c->stream));
    if (status) HIP_TRY(hipMemcpyAsync(status, L.status, P, hipMemcpyDeviceToHost, c->stream));
    int fault = 0;
    HIP_TRY(hipMemcpyAsync(&fault, c->b_fault.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    unsigned long long h[CT_N] = {};
    if (stats) HIP_TRY(hipMemcpyAsync(h, c->b_counters.p, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (stats) {
        memset(stats, 0, sizeof *stats);
        fill_stats(stats, h);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
        stats->kernel_ms = ms;
        stats->frame_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    if (fault) return rt_set_error(RT_E_FAULT, "a ray reached a state where the reference throws (status 2/3 pixels)");
    return RT_OK;
}

extern "C" int rt_trace_rows_device(rt_ctx *c, const rt_camera_desc *cam, const rt_config_desc *cfg, int32_t part,
                                    int32_t n_parts, int32_t stripe_rows, void *d_rgb, void *stream,
                                    int32_t *rows_out, rt_stats *stats)
{
    const auto t0 = std::chrono::steady_clock::now();
    int r = check_frame_args(c, cam, cfg);
    if (r != RT_OK) return r;
    if (n_parts < 1 || part < 0 || part >= n_parts || stripe_rows < 1)
        return rt_set_error(RT_E_INVALID, "rt_trace_rows_device: bad partition %d/%d stripe %d", part, n_parts, stripe_rows);
    if ((r = use_device(c)) != RT_OK) return r;
    RtLaunch L;
    if ((r = prepare(c, cam, cfg, part, n_parts, stripe_rows, false, L)) != RT_OK) return r;
    if (rows_out) *rows_out = L.rows;
    if (!d_rgb && L.rows > 0) return rt_set_error(RT_E_INVALID, "rt_trace_rows_device: d_rgb is null");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    L.rgb = (float *)d_rgb;
    L.blend = cfg->col_weight != 1.0;
    if (stats) {
        HIP_TRY(hipMemsetAsync(c->b_counters.p, 0, sizeof(unsigned long long) * CT_N, st));
        L.counters = (unsigned long long *)c->b_counters.p;
    }
    hipEvent_t *ev = c->ev[c->ev_next];
    c->ev_next = (c->ev_next + 1) % rt_ctx::NEV;
    c->ev_count = c->ev_count < rt_ctx::NEV ? c->ev_count + 1 : rt_ctx::NEV;
    if ((r = rt_launch_frame(L, st, ev[0], ev[1])) != RT_OK) return r;
    if (stats) {
        unsigned long long h[CT_N] = {};
        HIP_TRY(hipMemcpyAsync(h, c->b_counters.p, sizeof h, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        memset(stats, 0, sizeof *stats);
        fill_stats(stats, h);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
        stats->kernel_ms = ms;
        stats->frame_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return RT_OK;
}

// ---- device-resident exposure buffer (rt_exposure.hip) ---------------------------------
extern "C" int rt_exposure_stats_device(rt_ctx *c, const float *d_rgb, int64_t n_pixels, void *stream,
                                        rt_exposure_stats *out)
{
    if (!c || !out || n_pixels < 0 || (n_pixels > 0 && !d_rgb))
        return rt_set_error(RT_E_INVALID, "rt_exposure_stats_device: bad argument");
    int r = use_device(c);
    if (r != RT_OK) return r;
    const int n_blocks = (int)(n_pixels / 256 + 1 < 1024 ? n_pixels / 256 + 1 : 1024);
    if ((r = c->b_stat.ensure(sizeof(double) * (2 * (size_t)n_blocks + 4))) != RT_OK) return r;
    double *d_out = (double *)c->b_stat.p;
    double *d_part = d_out + 4;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if ((r = rt_launch_exposure_stats(d_rgb, (long long)n_pixels, d_part, n_blocks, d_out, st)) != RT_OK) return r;
    double h[3];
    HIP_TRY(hipMemcpyAsync(h, d_out, sizeof h, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    out->mean = h[0];
    out->variance = h[1];
    out->absdev = h[2];
    return RT_OK;
}

extern "C" int rt_tonemap_device(rt_ctx *c, const float *d_rgb, int64_t n_pixels, double drange_low,
                                 double drange_high, uint8_t *d_rgba, void *stream)
{
    if (!c || n_pixels < 0 || (n_pixels > 0 && (!d_rgb || !d_rgba)))
        return rt_set_error(RT_E_INVALID, "rt_tonemap_device: bad argument");
    int r = use_device(c);
    if (r != RT_OK) return r;
    return rt_launch_tonemap(d_rgb, (long long)n_pixels, drange_low, drange_high, d_rgba,
                             stream ? (hipStream_t)stream : c->stream);
}

// ToneMapper_DRLimited / _StdDevAroundMean / _AbsDevAroundMean / _Identity (src/view/tone_mapping.ts:22-80)
extern "C" int rt_tonemap_range(int32_t mode, const rt_exposure_stats *st, int32_t dynamic_range, double min_dynamic,
                                double max_dynamic, double range_out[2])
{
    if (!range_out || (mode != RT_TONEMAP_IDENTITY && !st))
        return rt_set_error(RT_E_INVALID, "rt_tonemap_range: null argument");
    if (mode == RT_TONEMAP_IDENTITY) {
        range_out[0] = 0;
        range_out[1] = 1;
        return RT_OK;
    }
    if (mode != RT_TONEMAP_STDDEV && mode != RT_TONEMAP_ABSDEV)
        return rt_set_error(RT_E_INVALID, "rt_tonemap_range: mode %d", mode);
    const double coef = (double)(int32_t)(1u << ((uint32_t)dynamic_range & 31));   // 1 << dynamic_range
    const double dev = mode == RT_TONEMAP_STDDEV ? sqrt(st->variance) : st->absdev;
    double hi = rtjs::jmin(st->mean + dev, max_dynamic);
    double lo = hi / coef;
    if (lo < min_dynamic) {
        lo = min_dynamic;
        hi = lo * coef;
    }
    range_out[0] = lo;
    range_out[1] = hi;
    return RT_OK;
}

extern "C" int rt_kernel_times(rt_ctx *c, double *ms_out, int32_t n)
{
    if (!c || (!ms_out && n > 0)) return rt_set_error(RT_E_INVALID, "rt_kernel_times: null argument");
    int k = n < c->ev_count ? n : c->ev_count;
    for (int i = 0; i < k; i++) {
        const int idx = ((c->ev_next - k + i) % rt_ctx::NEV + rt_ctx::NEV) % rt_ctx::NEV;
        HIP_TRY(hipEventSynchronize(c->ev[idx][1]));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[idx][0], c->ev[idx][1]));
        ms_out[i] = ms;
    }
    return k;
}

extern "C" int rt_debug_walk(rt_ctx *c, const double origin[3], const double dir[3], int32_t include_undefined,
                             int32_t max_out, int32_t *out_tree, int32_t *out_octant, int32_t *n_out)
{
    if (!c || !origin || !dir || !out_tree || !out_octant || !n_out || max_out < 0)
        return rt_set_error(RT_E_INVALID, "rt_debug_walk: bad argument");
    if (!c->has_scene) return rt_set_error(RT_E_NOSCENE, "no scene uploaded");
    int r;
    if ((r = use_device(c)) != RT_OK) return r;
    if ((r = c->b_walk.ensure(sizeof(int32_t) * (2 * (size_t)max_out + 1))) != RT_OK) return r;
    int32_t *d_tree = (int32_t *)c->b_walk.p, *d_oct = d_tree + max_out, *d_n = d_oct + max_out;
    if ((r = rt_launch_debug_walk(c->scene, origin, dir, include_undefined, max_out, d_tree, d_oct, d_n, c->stream)) != RT_OK)
        return r;
    int32_t n = 0;
    HIP_TRY(hipMemcpyAsync(&n, d_n, sizeof n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (n < 0) return rt_set_error(RT_E_FAULT, "rt_debug_walk: the walker threw");
    HIP_TRY(hipMemcpy(out_tree, d_tree, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(out_octant, d_oct, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    *n_out = n;
    return RT_OK;
}

extern "C" int rt_debug_camera_dirs(rt_ctx *c, const rt_camera_desc *cam, double *dirs_out)
{
    if (!c || !cam || !dirs_out) return rt_set_error(RT_E_INVALID, "rt_debug_camera_dirs: null argument");
    if (!c->has_scene) return rt_set_error(RT_E_NOSCENE, "no scene uploaded");
    if (cam->width <= 0 || cam->height <= 0) return rt_set_error(RT_E_INVALID, "bad screen size");
    int r;
    if ((r = use_device(c)) != RT_OK) return r;
    rt_config_desc cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.refmax = 1;
    cfg.default_substance = -1;
    cfg.col_weight = 1;
    RtLaunch L;
    if ((r = prepare(c, cam, &cfg, 0, 1, cam->height, false, L)) != RT_OK) return r;
    const size_t P = (size_t)cam->width * (size_t)cam->height;
    if ((r = c->b_rgb.ensure(sizeof(float) * 3 * P)) != RT_OK) return r;
    L.rgb = (float *)c->b_rgb.p;
    L.skip_trace = 1;
    if ((r = rt_launch_frame(L, c->stream, nullptr, nullptr)) != RT_OK) return r;
    std::vector<double> soa(3 * P);
    HIP_TRY(hipMemcpyAsync(soa.data(), L.dirs, sizeof(double) * 3 * P, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (size_t p = 0; p < P; p++)
        for (int i = 0; i < 3; i++) {
            const size_t x = p % (size_t)cam->width, y = p / (size_t)cam->width;
            dirs_out[3 * p + i] = soa[i * P + x * (size_t)cam->height + y];   // x-major on the device
        }
    return RT_OK;
}
