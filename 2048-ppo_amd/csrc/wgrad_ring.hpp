// wgrad_ring.hpp -- the LDS-DMA ring of the weight-gradient products dW = A^T B over many rows
// (A bf16 [m][N1], B bf16 [m][N2], fp32 partial per block), shared by mlp_wgrad.hip (the four GameMLP
// products in one launch) and urm.hip (g2048_urm_wgrad, the GameURM projections).  See
// mlp_wgrad.hip's header for the design: per stage 32 rows of each operand land in LDS exactly as
// they lie in HBM (lane-linear buffer_load ... lds, chunks past the range read zero), kStages - 1
// stages in flight behind counted vmcnt waits and one raw s_barrier per stage, and the MFMA
// operands come back through the transposing ds_read_b64_tr_b16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace g2048 {
namespace wgr {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kThreads = 512;  // 8 waves: two per SIMD
constexpr int kRows = 32;      // rows (the reduction index) per stage = one MFMA k-step
constexpr int kStages = 4;     // LDS ring: 3 stages in flight while one is consumed
constexpr int kRegion = 16384;  // bytes per operand per stage (1024 16-byte chunks: 32 rows x <= 256 bf16)
constexpr int kStageBytes = 2 * kRegion;
constexpr int kLds = kStages * kStageBytes;  // 128 KiB
constexpr int kMaxBlocks = 256;

struct Prod {
    const char *a, *b;  // row-major bf16 [m][n1], [m][n2]
    float *part;        // [nb][n1][n2]
    int64_t rows;       // rows per block (multiple of kRows)
    int nb, blk0;
};


// A' / B' fragment of a 32-row k-step: lane (g, q, p) reads rows 4 g + q and 16 + 4 g + q at columns
// c0 + 4 p .. + 3 of the row-major image (pitch bytes per row) -- the same k permutation for both
// operands, so the products pair up.
__device__ __forceinline__ bf16x8_t frag(const char *img, int pitch, int c0, int lane) {
    const int g = (lane >> 4) & 3, q = (lane >> 2) & 3, p = lane & 3;
    const char *a1 = img + (4 * g + q) * pitch + (c0 + 4 * p) * 2;
    const s16x4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)a1);
    const s16x4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(a1 + 16 * pitch));
    return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(t1, t2, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));

// A raw buffer descriptor (base, no stride, num_records bytes, the raw-buffer format word): offsets
// at or past num_records read as zero
__device__ __forceinline__ i32x4_t buffer_desc(const char *base, uint32_t bytes) {
    const uint64_t b = (uint64_t)base;
    return i32x4_t{__builtin_amdgcn_readfirstlane((int)(uint32_t)b), __builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32)),
                   __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}

// One LDS-DMA wave-instruction: lane i's 16 bytes at desc + voff land at LDS byte lds + 16 i.  In
// inline asm so the compiler does not treat every later LDS read as possibly aliasing a pending DMA
// (it would drain the whole ring with vmcnt(0) before each stage's fragment reads); the waits are
// the explicit counted ones, and the "memory" clobbers keep the LDS reads after them.  m0 is not in
// the clobber list (listing it makes hipcc put the same vmcnt(0) drain in front of every LDS read):
// nothing else in this kernel uses m0 (no compiler-emitted m0 in the .s outside these statements).
__device__ __forceinline__ void dma16(const i32x4_t &desc, uint32_t voff, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(desc),
                 "s"(lds)
                 : "memory");
}

// One block's product C[n1][n2] = sum over its rows of A[r][:]^T B[r][:], waves tiled WI (i) x
// 8 / WI (j), each BI x BJ 16x16 output tiles.
template <int N1, int N2, int BI, int BJ, int WI>
__device__ __forceinline__ void product(const Prod &pr, int64_t m, int blk, char *smem) {
    constexpr int TI = (N1 + 15) / 16, TJ = (N2 + 15) / 16;
    constexpr int CA = kRows * N1 * 2 / 16, CB = kRows * N2 * 2 / 16;  // 16-byte chunks per stage
    constexpr int LA = (CA + kThreads - 1) / kThreads, LB = (CB + kThreads - 1) / kThreads;
    constexpr int L = LA + LB;  // LDS-DMA instructions per wave and stage
    static_assert(CA * 16 <= kRegion && CB * 16 <= kRegion, "stage region");
    static_assert(L * (kStages - 1) <= 63, "vmcnt range");
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wi = wave % WI, wj = wave / WI;
    const int ti0 = wi * BI, tj0 = wj * BJ;  // wave-uniform
    const int64_t r0 = (int64_t)blk * pr.rows, r1 = r0 + pr.rows < m ? r0 + pr.rows : m;
    const int nst = r1 > r0 ? (int)((r1 - r0 + kRows - 1) / kRows) : 0;
    const uint32_t bytes_a = r1 > r0 ? (uint32_t)((r1 - r0) * N1 * 2) : 0u;
    const uint32_t bytes_b = r1 > r0 ? (uint32_t)((r1 - r0) * N2 * 2) : 0u;
    const i32x4_t ra = buffer_desc(pr.a + (r1 > r0 ? r0 * N1 * 2 : 0), bytes_a);
    const i32x4_t rb = buffer_desc(pr.b + (r1 > r0 ? r0 * N2 * 2 : 0), bytes_b);
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)smem;
    // stage s -> ring slot s % kStages; chunk c of an operand lands at region + 16 c
    auto issue = [&](int s) {
        const uint32_t slot = lds0 + (uint32_t)((s % kStages) * kStageBytes);
#pragma unroll
        for (int u = 0; u < LA; u++) {
            const int c = (wave + 8 * u) * 64 + lane;
            const uint32_t off = c < CA ? (uint32_t)(s * (kRows * N1 * 2) + 16 * c) : 0xFFFFFFF0u;
            dma16(ra, off, __builtin_amdgcn_readfirstlane(slot + (wave + 8 * u) * 1024));
        }
#pragma unroll
        for (int u = 0; u < LB; u++) {
            const int c = (wave + 8 * u) * 64 + lane;
            const uint32_t off = c < CB ? (uint32_t)(s * (kRows * N2 * 2) + 16 * c) : 0xFFFFFFF0u;
            dma16(rb, off, __builtin_amdgcn_readfirstlane(slot + kRegion + (wave + 8 * u) * 1024));
        }
    };
    f32x4_t acc[BI][BJ];
#pragma unroll
    for (int i = 0; i < BI; i++)
#pragma unroll
        for (int j = 0; j < BJ; j++) acc[i][j] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
    const bool active = ti0 < TI && tj0 < TJ;
#pragma unroll
    for (int s = 0; s < kStages - 1; s++)
        if (s < nst) issue(s);
    for (int s = 0; s < nst; s++) {
        // stage s landed (this wave's part): the younger stages may stay in flight
        const int ahead = nst - 1 - s;  // stages issued after s (at most kStages - 2 here)
        if (ahead >= 2) wait_vm<2 * L>();
        else if (ahead == 1) wait_vm<L>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();  // every wave's part landed; every wave done with stage s - 1's slot
        if (s + kStages - 1 < nst) issue(s + kStages - 1);
        if (active) {  // wave-uniform; inside, every MFMA unconditional
            const char *sa = smem + (s % kStages) * kStageBytes, *sb = sa + kRegion;
            bf16x8_t fb[BJ];
#pragma unroll
            for (int j = 0; j < BJ; j++) fb[j] = frag(sb, N2 * 2, 16 * (tj0 + j), lane);
#pragma unroll
            for (int i = 0; i < BI; i++) {
                const bf16x8_t fa = frag(sa, N1 * 2, 16 * (ti0 + i), lane);
#pragma unroll
                for (int j = 0; j < BJ; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
            }
        }
    }
    if (!active) return;
    float *out = pr.part + (int64_t)blk * N1 * N2;
    const int c = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < BI; i++)
#pragma unroll
        for (int j = 0; j < BJ; j++) {
            const int ii = 16 * (ti0 + i) + rq, jj = 16 * (tj0 + j) + c;
            if (ti0 + i < TI && tj0 + j < TJ && jj < N2)
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (ii + r < N1) out[(int64_t)(ii + r) * N2 + jj] = acc[i][j][r];
        }
}


}  // namespace wgr
}  // namespace g2048
