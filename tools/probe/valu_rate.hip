// VALU issue-rate probe: cycles per wave-instruction of integer VALU ops at 1, 2 and 4 waves per SIMD.
//   ./valu_rate        (prints one line per op and occupancy)
// Each wave runs `iters` x 16 independent instructions on 8 accumulators (no dependency stalls);
// cycles come from s_memtime around the loop, the wall time from hipEvents.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int Op>
__device__ __forceinline__ void body(uint32_t (&a)[8], uint32_t k) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        if constexpr (Op == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 3) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 4) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 5) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 6) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 7) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 9) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(a[j]) : "v"(k) : "s20", "s21");
        if constexpr (Op == 10) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 11) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 12) asm volatile("v_mad_u64_u32 %0, s[20:21], %1, %1, %0" : "+v"(*(uint64_t *)&a[j & 6]) : "v"(k) : "s20", "s21");
        if constexpr (Op == 13) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(a[j]) : "v"(k));
        if constexpr (Op == 8) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t *)&a[j & 6]) : "v"((uint64_t)k));
    }
}

template <int Op>
__global__ __launch_bounds__(1024) void probe(uint32_t *out, uint64_t *cyc, int iters, uint32_t k) {
    uint32_t a[8];
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] = threadIdx.x + j;
    if constexpr (Op == 4) asm volatile("v_cmp_gt_u32 vcc, %0, 37" :: "v"(threadIdx.x) : "vcc");
    if constexpr (Op == 9) asm volatile("v_cmp_gt_u32 s[20:21], %0, 37" :: "v"(threadIdx.x) : "s20", "s21");
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; i++) {
        body<Op>(a, k);
        body<Op>(a, k);
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int Op>
int run(const char *name, uint32_t *out, uint64_t *cyc, uint64_t *hcyc) {
    const int iters = 20000;
    for (int w = 1; w <= 4; w *= 2) {
        const int threads = 256 * w, blocks = 256;  // one block per CU, w waves per SIMD
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        hipLaunchKernelGGL(probe<Op>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 100, 1u);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(probe<Op>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 1u);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const int waves = blocks * threads / 64;
        CHECK(hipMemcpy(hcyc, cyc, waves * sizeof(uint64_t), hipMemcpyDeviceToHost));
        double avg = 0;
        for (int i = 0; i < waves; i++) avg += (double)hcyc[i];
        avg /= waves;
        const double instr = (double)iters * 16;
        // per SIMD: w waves each issuing instr instructions in `ms`
        const double ns_per_instr_simd = ms * 1e6 / (instr * w);
        printf("%-16s waves/SIMD=%d  wall %.3f ms  %.3f ns per wave-instr per SIMD (=%.2f cyc @2.4GHz)  memtime/wave-instr %.2f\n",
               name, w, ms, ns_per_instr_simd, ns_per_instr_simd * 2.4, avg / instr);
    }
    return 0;
}

int main() {
    uint32_t *out;
    uint64_t *cyc;
    CHECK(hipMalloc(&out, 256 * 1024 * sizeof(uint32_t)));
    CHECK(hipMalloc(&cyc, 256 * 16 * sizeof(uint64_t)));
    static uint64_t hcyc[256 * 16];
    run<0>("v_add_u32", out, cyc, hcyc);
    run<1>("v_xor_b32", out, cyc, hcyc);
    run<2>("v_bitop3_b32", out, cyc, hcyc);
    run<3>("v_bcnt_u32_b32", out, cyc, hcyc);
    run<4>("v_cndmask_b32", out, cyc, hcyc);
    run<5>("v_mul_hi_u32", out, cyc, hcyc);
    run<6>("v_add_f32", out, cyc, hcyc);
    run<7>("v_pk_add_u16", out, cyc, hcyc);
    run<8>("v_lshl_add_u64", out, cyc, hcyc);
    run<9>("v_cndmask_e64", out, cyc, hcyc);
    run<10>("v_perm_b32", out, cyc, hcyc);
    run<11>("v_or3_b32", out, cyc, hcyc);
    run<12>("v_mad_u64_u32", out, cyc, hcyc);
    run<13>("v_and_b32_e32", out, cyc, hcyc);
    return 0;
}
