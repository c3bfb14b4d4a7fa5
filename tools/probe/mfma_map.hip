// Checks the v_mfma_f32_16x16x32_bf16 operand / result maps with exact integer data:
// A[i][k] = (i == k%16 && k < 16), B[k][j] = 16k + j  ->  C = B[0:16].
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ float Aval(int i, int k) { return (k < 16 && i == k) ? 1.0f : 0.0f; }
__device__ float Bval(int k, int j) { return (float)(16 * k + j); }
__global__ void k(float *out) {
    const int l = threadIdx.x;
    bf16x8 a, b;
    for (int j = 0; j < 8; j++) {
        const int kk = 8 * (l >> 4) + j;
        a[j] = (__bf16)Aval(l & 15, kk);
        b[j] = (__bf16)Bval(kk, l & 15);
    }
    f32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) out[((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}
int main() {
    float *d, h[256];
    (void)hipMalloc(&d, 1024);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 16; i++) {
        for (int j = 0; j < 16; j++) {
            printf("%5.0f", h[i * 16 + j]);
            bad += h[i * 16 + j] != (float)(16 * i + j);
        }
        printf("\n");
    }
    printf("bad %d\n", bad);
    return 0;
}
