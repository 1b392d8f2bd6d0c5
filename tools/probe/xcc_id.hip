#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(int *out) {
    if (threadIdx.x == 0) {
        unsigned v = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);   // HW_REG_XCC_ID[3:0]
        out[blockIdx.x] = (int)v;
    }
}
int main() {
    const int n = 4096;
    int *d; hipMalloc(&d, n * 4);
    hipLaunchKernelGGL(k, dim3(n), dim3(256), 0, 0, d);
    int h[n]; hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost);
    int match = 0, cnt[16] = {0};
    for (int i = 0; i < n; i++) { match += (h[i] == (i & 7)); cnt[h[i] & 15]++; }
    printf("round-robin matches %d / %d\n", match, n);
    for (int i = 0; i < 16; i++) printf("%d ", cnt[i]);
    printf("\nfirst 24: "); for (int i = 0; i < 24; i++) printf("%d ", h[i]); printf("\n");
    return 0;
}
