// rt_exposure.hip — the device-resident ExposureBuffer consumers:
// luminance statistics (src/view/exposure_buffer.ts:90-136) and the tone-mapped RGBA8 image a
// canvas receives (discretize_to_screen :145-158 + CanvasScreen.set_pixel_i / convert_color,
// src/view/screen_canvas.ts:45-55,92-94).  Both read the f32 buffer once per pass: HBM-bound.
#include <hip/hip_runtime.h>

#include "rt_internal.h"
#include "rt_jsnum.h"

namespace {

constexpr double W_R = 0.299, W_G = 0.587, W_B = 0.114;   // rgb_to_y, src/view/exposure_buffer.ts:161-172
constexpr double JS_EPSILON = 2.220446049250313e-16;      // Number.EPSILON

// rgb_to_y in the reference's evaluation order (left to right)
__device__ __forceinline__ double luma(const float *px)
{
    return W_R * (double)px[0] + W_G * (double)px[1] + W_B * (double)px[2];
}

// clamp (src/math/mathutils.ts:18-20): Math.max(Math.min(x, hi), lo), NaN-propagating
__device__ __forceinline__ double js_clamp(double x, double lo, double hi) { return rtjs::jmax(rtjs::jmin(x, hi), lo); }

// (x << 0) for x in [0, 255] or NaN (ToInt32: NaN -> 0, truncation toward zero)
__device__ __forceinline__ int js_to_int32_small(double x) { return x == x ? (int)x : 0; }

constexpr int STAT_THREADS = 256;

__device__ __forceinline__ double block_sum(double v, double *lds)
{
    // fixed-order tree: lanes by xor shuffles, then the four waves in index order
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) lds[wave] = v;
    __syncthreads();
    double s = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < STAT_THREADS / 64; w++) s += lds[w];
    __syncthreads();
    return s;
}

// PASS 0: partial sums of Y; PASS 1: partial sums of (Y - mean)^2 and |Y - mean|, mean = out[0].
template <int PASS>
__global__ void __launch_bounds__(STAT_THREADS) k_luma_partial(const float *__restrict__ rgb, long long n,
                                                              double *__restrict__ partials,
                                                              const double *__restrict__ out)
{
    __shared__ double lds[STAT_THREADS / 64];
    const long long stride = (long long)gridDim.x * STAT_THREADS;
    const double mean = PASS ? out[0] : 0.0;
    double a = 0, b = 0;
    for (long long i = (long long)blockIdx.x * STAT_THREADS + threadIdx.x; i < n; i += stride) {
        const double y = luma(rgb + 3 * i);
        if (PASS == 0) {
            a += y;
        } else {
            const double delta = y - mean;
            a += delta * delta;
            b += fabs(delta);
        }
    }
    a = block_sum(a, lds);
    if (PASS) b = block_sum(b, lds);
    if (threadIdx.x == 0) {
        partials[2 * blockIdx.x] = a;
        partials[2 * blockIdx.x + 1] = b;
    }
}

// One block: the block partials in fixed order; PASS 0 writes mean, PASS 1 variance and absdev
// (each sum divided by n_pixels, as the reference does).
template <int PASS>
__global__ void __launch_bounds__(STAT_THREADS) k_luma_final(const double *__restrict__ partials, int n_parts,
                                                            long long n, double *__restrict__ out)
{
    __shared__ double lds[STAT_THREADS / 64];
    double a = 0, b = 0;
    for (int k = threadIdx.x; k < n_parts; k += STAT_THREADS) {
        a += partials[2 * k];
        b += partials[2 * k + 1];
    }
    a = block_sum(a, lds);
    b = block_sum(b, lds);
    if (threadIdx.x == 0) {
        if (PASS == 0) {
            out[0] = a / (double)n;
        } else {
            out[1] = a / (double)n;
            out[2] = b / (double)n;
        }
    }
}

// discretize_to_screen + set_pixel_i for one pixel per thread.  The reference maps
// `pixels.slice(i, i+2)` (two channels) through Float32Array.map (values rounded to f32), so the
// canvas gets R and G, blue = undefined (stored as 0) and alpha 0xff.
__global__ void __launch_bounds__(256) k_tonemap(const float *__restrict__ rgb, long long n, double low, double high,
                                                 uchar4 *__restrict__ rgba)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float *px = rgb + 3 * i;
    const double drange = high - low;
    const double y = luma(px);
    const double cmpr = (y - low) / drange;
    const double scale = cmpr / (y + JS_EPSILON);
    const float c0 = (float)js_clamp((double)px[0] * scale, 0.0, 1.0);
    const float c1 = (float)js_clamp((double)px[1] * scale, 0.0, 1.0);
    uchar4 o;
    o.x = (unsigned char)js_to_int32_small(js_clamp((double)c0, 0.0, 1.0) * 255);
    o.y = (unsigned char)js_to_int32_small(js_clamp((double)c1, 0.0, 1.0) * 255);
    o.z = 0;
    o.w = 0xff;
    rgba[i] = o;
}

}  // namespace

#define HIP_TRY(x)                                                                           \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) return rt_set_error(RT_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

int rt_launch_exposure_stats(const float *d_rgb, long long n, double *d_partials, int n_blocks, double *d_out3,
                             void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_luma_partial<0>, dim3(n_blocks), dim3(STAT_THREADS), 0, st, d_rgb, n, d_partials,
                       (const double *)d_out3);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_luma_final<0>, dim3(1), dim3(STAT_THREADS), 0, st, (const double *)d_partials, n_blocks, n,
                       d_out3);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_luma_partial<1>, dim3(n_blocks), dim3(STAT_THREADS), 0, st, d_rgb, n, d_partials,
                       (const double *)d_out3);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_luma_final<1>, dim3(1), dim3(STAT_THREADS), 0, st, (const double *)d_partials, n_blocks, n,
                       d_out3);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_launch_tonemap(const float *d_rgb, long long n, double low, double high, uint8_t *d_rgba, void *stream)
{
    if (n <= 0) return RT_OK;
    hipLaunchKernelGGL(k_tonemap, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_rgb, n, low,
                       high, reinterpret_cast<uchar4 *>(d_rgba));
    HIP_TRY(hipGetLastError());
    return RT_OK;
}
