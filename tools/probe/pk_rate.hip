// Issue rate of packed vs scalar fp32 FMA on gfx950, one wave per SIMD (4 waves per block, one block
// per CU): cycles per instruction from s_memtime around a chain of independent FMAs.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/pk_rate tools/probe/pk_rate.hip && /tmp/pk_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <bool PK>
__global__ __launch_bounds__(256) void rate(float *out, long long *cyc, float s) {
    float a[16];
    f2 p[8];
#pragma unroll
    for (int i = 0; i < 16; i++) a[i] = threadIdx.x * 0.001f + i;
#pragma unroll
    for (int i = 0; i < 8; i++) p[i] = f2{a[2 * i], a[2 * i + 1]};
    const f2 s2 = f2{s, s};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 1024; it++) {
        if (PK) {
#pragma unroll
            for (int i = 0; i < 8; i++) p[i] = __builtin_elementwise_fma(p[i], s2, s2);
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) a[i] = __builtin_fmaf(a[i], s, s);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float r = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; i++) r += PK ? p[i].x + p[i].y : a[2 * i] + a[2 * i + 1];
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float *out;
    long long *cyc;
    hipMalloc(&out, 256 * 256 * 4);
    hipMalloc(&cyc, 256 * 8);
    long long h[256];
    for (int pk = 0; pk < 2; pk++) {
        for (int rep = 0; rep < 2; rep++) {
            if (pk) hipLaunchKernelGGL(rate<true>, dim3(256), dim3(256), 0, 0, out, cyc, 0.999f);
            else hipLaunchKernelGGL(rate<false>, dim3(256), dim3(256), 0, 0, out, cyc, 0.999f);
            hipDeviceSynchronize();
        }
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        double m = 0;
        for (int i = 0; i < 256; i++) m += h[i];
        m /= 256;
        // 1024 iterations x 16 fp32 FMAs per lane: scalar = 16 instructions, packed = 8
        printf("%s: %.1f cycles per iteration (16 fp32 FMAs per lane) = %.2f cycles per instruction\n",
               pk ? "v_pk_fma_f32" : "v_fma_f32", m / 1024, m / 1024 / (pk ? 8 : 16));
    }
    return 0;
}
