// Prints what ds_read_b64_tr_b16 delivers: LDS holds value = element index (16-bit), lane l
// reads at the address row (l>>2)&3, cols 4*(l&3) of a 16-column image (plus group offset).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
__global__ void k(short *out, int mode) {
    __shared__ short lds[64 * 16];
    for (int i = threadIdx.x; i < 64 * 16; i += 64) lds[i] = (short)i;
    __syncthreads();
    const int l = threadIdx.x, g = l >> 4, q = (l >> 2) & 3, p = l & 3;
    int row = 4 * g + q, col = 4 * p;
    if (mode == 1) { row = l; col = 0; }
    const s16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(lds + row * 16 + col));
    for (int e = 0; e < 4; e++) out[l * 4 + e] = t[e];
}
int main() {
    short *d, h[256];
    hipMalloc(&d, 512);
    for (int mode = 0; mode < 2; mode++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
        hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
        printf("mode %d (value = row*16 + col)\n", mode);
        for (int l = 0; l < 64; l++) {
            printf("lane %2d:", l);
            for (int e = 0; e < 4; e++) printf(" (%2d,%2d)", h[l * 4 + e] / 16, h[l * 4 + e] % 16);
            printf("\n");
        }
    }
    return 0;
}
