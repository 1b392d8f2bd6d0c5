// Per-step cost of k_frame_start's rotation chain: one rotate_vectors component
// step is x' = x c + y s, y' = -x s + y c in binary64 without contraction; a row's scan is a
// dependent chain of such steps.  Variants: the chain alone, with a store per step (k_frame_start's
// pattern), with stores of register copies, and two independent chains per lane (ILP 2).
//
//     hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/probe/chain_latency tools/probe/chain_latency.hip
//     ./tools/probe/chain_latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ void rot(double &x, double &y, double c, double s)
{
    const double nx = x * c + y * s, ny = x * -s + y * c;
    x = nx;
    y = ny;
}

template <int V>
__global__ void __launch_bounds__(256) k_chain(double *out, long long *cyc, int n, int rows, double c, double s)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rows) return;
    double x = 0.3 + 1e-6 * t, y = 0.7 - 1e-6 * t;
    double x2 = 0.5 + 1e-6 * t, y2 = 0.1 - 1e-6 * t;
    const long long t0 = clock64();
    double *p = out + t;
    if (V == 0) {
#pragma unroll 4
        for (int k = 0; k < n; k++) rot(x, y, c, s);
        *p = x + y;
    } else if (V == 1) {
#pragma unroll 4
        for (int k = 0; k < n; k++) { *p = x; p += rows; rot(x, y, c, s); }
    } else if (V == 2) {                       // 4 steps in registers, then 4 stores
        for (int k = 0; k + 4 <= n; k += 4) {
            const double a0 = x; rot(x, y, c, s);
            const double a1 = x; rot(x, y, c, s);
            const double a2 = x; rot(x, y, c, s);
            const double a3 = x; rot(x, y, c, s);
            p[0] = a0; p[rows] = a1; p[2 * rows] = a2; p[3 * rows] = a3;
            p += 4 * rows;
        }
    } else if (V == 5) {                       // (x, x+1) pairs adjacent: one 16-byte store per 2 steps
        double2 *q = reinterpret_cast<double2 *>(out) + t;
        for (int k = 0; k + 2 <= n; k += 2) {
            const double a0 = x; rot(x, y, c, s);
            const double a1 = x; rot(x, y, c, s);
            *q = make_double2(a0, a1);
            q += rows;
        }
    } else if (V == 6) {                       // buffer store: lane offset in a VGPR, column in an SGPR
        typedef unsigned int u2 __attribute__((ext_vector_type(2)));
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
        int so = 0;
#pragma unroll 4
        for (int k = 0; k < n; k++) {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, x), r, t * 8, so, 0);
            so += rows * 8;
            rot(x, y, c, s);
        }
    } else if (V == 7) {                       // wave-uniform base stepped in scalar registers, 32-bit lane offset
        const char *b0 = reinterpret_cast<const char *>(out) + (size_t)blockIdx.x * blockDim.x * 8;
        char *b = const_cast<char *>(b0);
        const unsigned lo = threadIdx.x * 8u;
#pragma unroll 4
        for (int k = 0; k < n; k++) {
            *reinterpret_cast<double *>(b + lo) = x;
            b += (size_t)rows * 8;
            rot(x, y, c, s);
        }
    } else if (V == 8) {                       // buffer store of a copy taken before the rotation
        typedef unsigned int u2 __attribute__((ext_vector_type(2)));
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
        int so = 0;
#pragma unroll 4
        for (int k = 0; k < n; k++) {
            const double keep = x;
            rot(x, y, c, s);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, keep), r, t * 8, so, 0);
            so += rows * 8;
        }
    } else if (V == 3) {                       // two chains per lane, no stores
#pragma unroll 4
        for (int k = 0; k < n; k++) { rot(x, y, c, s); rot(x2, y2, c, s); }
        *p = x + y + x2 + y2;
    } else if (V == 4) {                       // two chains per lane, a store each per step
        double *q = p + (size_t)n * rows;
#pragma unroll 4
        for (int k = 0; k < n; k++) { *p = x; *q = x2; p += rows; q += rows; rot(x, y, c, s); rot(x2, y2, c, s); }
    }
    const long long t1 = clock64();
    if ((threadIdx.x & 63) == 0) cyc[t >> 6] = t1 - t0;
}

template <int V>
static void run(const char *name, int rows, int n, double *out, long long *cyc, int bs = 256)
{
    const int blocks = (rows + bs - 1) / bs;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; i++) k_chain<V><<<blocks, bs>>>(out, cyc, n, rows, 0.99999, 0.0044);
    hipEventRecord(a);
    const int reps = 20;
    for (int i = 0; i < reps; i++) k_chain<V><<<blocks, bs>>>(out, cyc, n, rows, 0.99999, 0.0044);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    std::vector<long long> h((rows + 63) / 64);
    hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    long long mx = 0;
    for (long long v : h) mx = v > mx ? v : mx;
    printf("{\"variant\": \"%s\", \"block\": %d, \"lanes\": %d, \"steps\": %d, \"us\": %.2f, \"ns_per_step\": %.2f, "
           "\"clk_per_step\": %.1f}\n", name, bs, rows, n, 1e3 * ms / reps, 1e6 * ms / reps / n, (double)mx / n);
}

int main()
{
    double *out;
    long long *cyc;
    const int n = 1500, max_rows = 6480;
    hipMalloc(&out, sizeof(double) * (size_t)max_rows * n * 2);
    hipMalloc(&cyc, sizeof(long long) * 1024);
    for (int rows : {64, 6480}) {
        run<0>("chain", rows, n, out, cyc);
        run<1>("chain+store", rows, n, out, cyc);
        run<2>("chain+store4", rows, n, out, cyc);
        run<3>("2chains", rows, n, out, cyc);
        run<4>("2chains+store", rows, n, out, cyc);
        run<5>("chain+store_pairs", rows, n, out, cyc);
        run<0>("chain", rows, n, out, cyc, 64);
        run<1>("chain+store", rows, n, out, cyc, 64);
        run<5>("chain+store_pairs", rows, n, out, cyc, 64);
        run<6>("chain+buffer_store", rows, n, out, cyc, 64);
        run<7>("chain+uniform_base_store", rows, n, out, cyc, 64);
        run<8>("chain+buffer_store_late", rows, n, out, cyc, 64);
    }
    return 0;
}
