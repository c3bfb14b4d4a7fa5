// optim.hip -- the optimizer step of the PPO update (train.py:553-568: clip_grad_norm_(1.0),
// Muon for the 2-D weights, AdamW for the 1-D LayerNorm / bias parameters; torch.optim.Muon with
// adjust_lr_fn="match_rms_adamw", nesterov, 5 Newton-Schulz steps in bf16) as three launches:
//
//   grad_sumsq/norm      ||g|| over the flat gradient bucket and the clip coefficient
//                        clamp(max_norm / (||g|| + 1e-6), max=1) into device scalars (NaN kept)
//   muon_kernel          one 512-thread block per weight matrix: momentum + nesterov, bf16 cast,
//                        Frobenius normalisation, the 5 Newton-Schulz iterations
//                            G = X X^T;  U = b G + c G G;  X = a X + U X
//                        entirely in LDS on bf16 MFMA (v_mfma_f32_16x16x32_bf16, fp32 accumulate,
//                        one bf16 rounding per product like the library addmm), then decoupled
//                        weight decay + the scaled update, and the bf16 copy of the new weight
//   adamw_kernel         every 1-D group in one grid-stride pass
//
// The library path spends ~500 us per 196 x 196 matrix on 15 separately launched tiny GEMMs; here
// a matrix is one block and all matrices of the model run concurrently.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/g2048_ppo.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(uint32_t b) { return __uint_as_float(b << 16); }

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// round-to-nearest-even float -> bf16 on the hardware converter (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
    const bf16x2_t v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ uint32_t f2bf(float f) { return pack_bf2(f, 0.0f) & 0xFFFFu; }

__device__ __forceinline__ float round_bf(float f) { return (float)(__bf16)f; }

// ------------------------------------------------------------------ gradient norm ------------
// Two deterministic stages: kNormBlocks partial sums of squares, then one block sums them in order.
constexpr int kNormBlocks = 64;

__global__ __launch_bounds__(256) void grad_sumsq_kernel(const float *__restrict__ g, int64_t n,
                                                         float *__restrict__ part, float *__restrict__ tick = nullptr) {
    __shared__ float red[4];
    if (tick && blockIdx.x == 0 && threadIdx.x == 0) *tick += 1.0f;  // the optimizer's step count
    float s = 0.0f;
    const int64_t n4 = n >> 2;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)kNormBlocks * 256) {
        const float4 v = reinterpret_cast<const float4 *>(g)[i];
        s += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
    }
    if (blockIdx.x == 0)
        for (int64_t i = 4 * n4 + threadIdx.x; i < n; i += 256) s += g[i] * g[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// torch.nn.utils.clip_grad_norm_'s coefficient (train.py:560): clamp(max_norm / (norm + 1e-6), max=1).
// torch.clamp passes a NaN through, so a NaN norm makes the step NaN exactly as in the reference;
// fminf(c, 1) returned 1 for a NaN c (v_min_f32 drops the NaN operand): the step then ran unclipped
// with finite weights and only the logged norm showed the fault (round-5 verdict).  The
// trainer raises on a non-finite norm at its one metrics read.
__device__ __forceinline__ float clip_coef(float max_norm, float nrm) {
    const float c = max_norm / (nrm + 1e-6f);
    return c > 1.0f ? 1.0f : c;  // NaN > 1 is false: the NaN is kept
}

__global__ __launch_bounds__(64) void grad_norm_kernel(const float *__restrict__ part, float max_norm,
                                                       float *__restrict__ norm_out, float *__restrict__ coef_out) {
    float s = part[threadIdx.x];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (threadIdx.x == 0) {
        const float nrm = sqrtf(s);
        *norm_out = nrm;
        *coef_out = clip_coef(max_norm, nrm);
    }
}

// ------------------------------------------------------------------ AdamW --------------------
constexpr int kAdamMaxGroups = 4;

struct AdamGroup {
    float *param;
    const float *grad;
    float *m, *v;
    int64_t n;
    int lr_index, pad;
};

struct AdamArgs {
    AdamGroup g[kAdamMaxGroups];
    int count;
    float b1, b2, eps, wd;
    const float *lr;
    const float *step;
    const float *clip;
};

// one AdamW update of element i (torch.optim.AdamW: decoupled decay, bias corrections)
__device__ __forceinline__ void adamw_elem(const AdamGroup &gr, int64_t i, float lr, float coef, float b1, float b2,
                                           float eps, float wd, float bc1, float bc2s) {
    const float g = gr.grad[i] * coef;
    float p = gr.param[i] * (1.0f - lr * wd);
    const float m = gr.m[i] + (1.0f - b1) * (g - gr.m[i]);
    const float v = gr.v[i] * b2 + (1.0f - b2) * g * g;
    gr.m[i] = m;
    gr.v[i] = v;
    p -= (lr / bc1) * m / (sqrtf(v) / bc2s + eps);
    gr.param[i] = p;
}

// ------------------------------------------------------------------ Muon ---------------------
constexpr int kMuonThreads = 1024;       // 16 waves (4 per SIMD: LDS latency hidden by the others)
constexpr int kMuonWaves = kMuonThreads / 64;
constexpr int kBI = 4, kBJ = 4;          // generic schedule: 4 x 4 waves of 4 x 4 16x16 tiles = 256 x 256
constexpr int kMuonMaxMats = 16;  // GameMLP: 5, GameURM (2 layers): 11
static_assert(sizeof(g2048_muon_matrix) == 56 && offsetof(g2048_muon_matrix, head_frag) == 32,
              "g2048_muon_matrix layout (tests/test_abi.py)");
static_assert(sizeof(g2048_muon_cfg) == 48 && offsetof(g2048_muon_cfg, workspace) == 40,
              "g2048_muon_cfg layout (tests/test_abi.py)");
constexpr int kMuonMaxJobs = 128;  // grid blocks: Muon parts, AdamW blocks, idle gaps (XCD placement)
constexpr uint8_t kRoleAdam = 0xFE, kRoleIdle = 0xFF;
// one 64-byte line per matrix (exchange / prologue / done counters, the matrix's timeout flag),
// then one line whose first word counts every timed-out wait of every launch (sticky: only the host
// clears it -- FusedMuonAdamW reads it with the train step's metrics and raises, g2048_ppo.h)
constexpr int kMuonSyncBytes = kMuonMaxMats * 64 + 64;
constexpr int kMuonErrWord = kMuonMaxMats * 16;  // uint32 index of the sticky timeout count
constexpr int kMuonLds = 160 * 1024 - 256;  // minus the static red[] / s_norm

struct MuonMat {
    float *param;
    const float *grad;
    float *mom;
    uint16_t *pbf;
    uint16_t *frag;  // head matrices: the passes' three-term bf16 fragment image (g2048_head_split)
    int rows, cols, lr_index, frag_row;
};

// g2048_head_split's arithmetic for one weight w of head row `which`, column k (h columns): the exact
// terms hi = bf16(w), mid = bf16(w - hi), lo = bf16(w - hi - mid) into fragment rows which, 5 + which,
// 10 + which at k-step k / 32, lane group (k % 32) / 8, element k % 8
__device__ __forceinline__ void head_frag_put(uint16_t *frag, int which, int k, float w) {
    const __bf16 hi = (__bf16)w;
    const float r1 = w - (float)hi;
    const __bf16 mid = (__bf16)r1;
    const __bf16 lo = (__bf16)(r1 - (float)mid);
    const int ks = k >> 5, g = (k >> 3) & 3, e = k & 7;
    const int base = (ks * 64 + 16 * g) * 8 + e;
    frag[base + which * 8] = __builtin_bit_cast(uint16_t, hi);
    frag[base + (5 + which) * 8] = __builtin_bit_cast(uint16_t, mid);
    frag[base + (10 + which) * 8] = __builtin_bit_cast(uint16_t, lo);
}

struct MuonArgs {
    MuonMat m[kMuonMaxMats];
    int count;
    float momentum, wd, a, b, c, eps;
    int steps, nesterov;
    const float *lr;
    const float *clip;
    const float *partials;  // non-null: clip coefficient from the grad_sumsq partials (grad_norm folded in)
    float max_norm;
    float *norm_out, *coef_out;  // written by block 0 when partials is set
    AdamArgs adam;               // adam.count > 0: blocks count .. count + nadam - 1 run AdamW
    int nadam;
    int generic_ns;              // 1: square matrices on the generic schedule too (A/B timing, tests)
    // per grid block: job_mat = the matrix (a square matrix of the multi-CU path is split over
    // job_nparts blocks: row blocks of its Newton-Schulz products, one exchange of X per iteration),
    // kRoleAdam (job_part = the AdamW block index) or kRoleIdle (a gap of the XCD placement)
    int njobs;  // grid size
    int npartials;  // clip partial sums (64: g2048_grad_sumsq's)
    uint8_t job_mat[kMuonMaxJobs], job_part[kMuonMaxJobs], job_nparts[kMuonMaxJobs];
    uint32_t *sync;              // per matrix: the exchange counter (zeroed before every launch)
    uint32_t spin_limit;         // polls of a hand-off counter before a wait gives up (~0.2 s by default)
    char *xg;                    // per matrix: two N x P-byte bf16 exchange images (X of even / odd iterations)
    int64_t xg_stride;           // bytes per matrix
    uint64_t *trace;             // MUON_TRACE builds: phase clocks
};

// LDS images are row-major bf16 with the K dimension zero-padded to a multiple of 8 (pitch =
// 2 * round8(cols) bytes, a multiple of 16), so a fragment is one aligned 16-byte read and every
// out-of-range fragment is redirected to a zero block: the MFMA loops are branch-free per lane.

// acc += A[M x K] B[K x N] over this wave's tile block (ti0, tj0: wave-uniform).  B is given by
// the rows of B^T (B[k][n] = Bt[n][k]).  A is read by rows (a_rows) or, for A = X^T of a
// row-major X [K][M], with the transposing read.  kp = round8(K) = the padded K of row images.
// One copy of this loop serves all three Newton-Schulz products (a_rows is wave-uniform): the
// kernel has to fit the instruction cache, unrolled per product it does not.
template <int BI = kBI, int BJ = kBJ>
__device__ __forceinline__ void gemm_block(f32x4_t (&acc)[BI][BJ], const char *A, int pa, bool a_rows,
                                           const char *B, int pb, int M, int N, int K, int ti0, int tj0,
                                           const char *zero, int lane) {
    const int TI = (M + 15) >> 4, TJ = (N + 15) >> 4, kp = (K + 7) & ~7;
    if (ti0 >= TI || tj0 >= TJ) return;  // wave-uniform: nothing of this wave's block is in range
    // Per-lane row offsets are fixed for the whole product (-1: out of range -> zero block).
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    int boff[BJ], aoff[BI];
#pragma unroll
    for (int j = 0; j < BJ; j++) {
        const int row = 16 * (tj0 + j) + (lane & 15);
        boff[j] = row < N ? row * pb : -1;
    }
#pragma unroll
    for (int i = 0; i < BI; i++) {
        const int row = 16 * (ti0 + i) + (lane & 15);
        aoff[i] = a_rows ? (row < M ? row * pa : -1) : (16 * (ti0 + i) + 4 * p) * 2;  // col bytes for tr reads
    }
    // Every MFMA of the block is issued unconditionally (out-of-range tiles multiply zero fragments
    // and are never stored): a guarded MFMA makes the compiler copy its accumulator out and wait
    // for it, serialising the whole loop.
    for (int k0 = 0; k0 < kp; k0 += 32) {
        const int kl = k0 + 8 * g;
        const bool kin = kl < kp;
        bf16x8_t fb[BJ], fa[BI];
#pragma unroll
        for (int j = 0; j < BJ; j++) {
            const char *pp = (kin && boff[j] >= 0) ? B + boff[j] + 2 * kl : zero;
            fb[j] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4 *>(pp));
        }
        if (a_rows) {
#pragma unroll
            for (int i = 0; i < BI; i++) {
                const char *pp = (kin && aoff[i] >= 0) ? A + aoff[i] + 2 * kl : zero;
                fa[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4 *>(pp));
            }
        } else {  // A = X^T: lane (g, i) needs X[k0 + 8g + j][m0 + i], two transposing reads
            const int r1 = k0 + 8 * g + q, r2 = r1 + 4;
            const char *b1 = A + r1 * pa, *b2 = A + r2 * pa;
#pragma unroll
            for (int i = 0; i < BI; i++) {
                const char *a1 = r1 < K ? b1 + aoff[i] : zero;
                const char *a2 = r2 < K ? b2 + aoff[i] : zero;
                const s16x4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)a1);
                const s16x4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)a2);
                fa[i] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(t1, t2, 0, 1, 2, 3, 4, 5, 6, 7));
            }
        }
#pragma unroll
        for (int i = 0; i < BI; i++)
#pragma unroll
            for (int j = 0; j < BJ; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
}

// The accumulators start from the scaled previous output, (beta / alpha) * out[col][row] (zero when
// beta == 0, and for tiles outside the product), read BEFORE the GEMM: the read and its conversion
// overlap the MFMA work instead of sitting between the two barriers, and the store is a plain write.
template <int BI = kBI, int BJ = kBJ>
__device__ __forceinline__ void init_block_t(f32x4_t (&acc)[BI][BJ], const char *out, int pitch, int M, int N,
                                             int ti0, int tj0, float ratio, bool use_old, int lane) {
#pragma unroll
    for (int i = 0; i < BI; i++)
#pragma unroll
        for (int j = 0; j < BJ; j++) {
            const int col = 16 * (tj0 + j) + (lane & 15);
            const int row0 = 16 * (ti0 + i) + 4 * (lane >> 4);
            f32x4_t a = {0.0f, 0.0f, 0.0f, 0.0f};
            if (use_old && col < N && row0 < M) {
                const uint2 q = *reinterpret_cast<const uint2 *>(out + col * pitch + row0 * 2);
                a = f32x4_t{ratio * bf2f(q.x & 0xFFFFu), ratio * bf2f(q.x >> 16), ratio * bf2f(q.y & 0xFFFFu),
                            ratio * bf2f(q.y >> 16)};
            }
            acc[i][j] = a;
        }
}

// Stores the TRANSPOSE of the accumulated block: out[col][row] = bf16(alpha * acc[row][col]) for
// cols < N and rows < round4(M) (acc already holds (beta / alpha) * the old value: init_block_t).
// A lane holds 4 consecutive rows of one column, i.e. 4 consecutive elements of one output row:
// one 8-byte LDS write.  Rows M .. round4(M)-1 land in the zero K padding and are zero (their
// operands are zero fragments).  Callers put a barrier between the GEMM's last read of `out` and this.
template <int BI = kBI, int BJ = kBJ>
__device__ __forceinline__ void store_block_t(const f32x4_t (&acc)[BI][BJ], char *out, int pitch, int M, int N,
                                              int ti0, int tj0, float alpha, int lane) {
    const int TI = (M + 15) >> 4, TJ = (N + 15) >> 4;
    if (ti0 >= TI || tj0 >= TJ) return;
#pragma unroll
    for (int i = 0; i < BI; i++)
#pragma unroll
        for (int j = 0; j < BJ; j++) {
            const int col = 16 * (tj0 + j) + (lane & 15);
            const int row0 = 16 * (ti0 + i) + 4 * (lane >> 4);
            if (col < N && row0 < M)
                *reinterpret_cast<uint2 *>(out + col * pitch + row0 * 2) =
                    make_uint2(pack_bf2(alpha * acc[i][j][0], alpha * acc[i][j][1]),
                               pack_bf2(alpha * acc[i][j][2], alpha * acc[i][j][3]));
        }
}

// momentum + nesterov + bf16 rounding of 4 elements: bv = the new momentum, ub = the bf16-valued
// update; returns the sum of squares of ub
__device__ __forceinline__ float momentum4(const float4 &g4, const float4 &b4, float coef, float mu, bool nesterov,
                                          float bv[4], float ub[4]) {
    // no fma contraction: the one-CU, generic and multi-CU schedules inline this in different places
    // and must round identically (their bitwise equality is tested)
#pragma clang fp contract(off)
    const float gv[4] = {g4.x * coef, g4.y * coef, g4.z * coef, g4.w * coef};
    bv[0] = b4.x;
    bv[1] = b4.y;
    bv[2] = b4.z;
    bv[3] = b4.w;
    float ss = 0.0f;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        bv[u] = bv[u] + (1.0f - mu) * (gv[u] - bv[u]);                               // buf.lerp_(g, 1 - mu)
        const float up = nesterov ? bv[u] - (bv[u] - gv[u]) * (1.0f - mu) : bv[u];  // g.lerp(buf, mu)
        ub[u] = round_bf(up);
        ss = __builtin_fmaf(ub[u], ub[u], ss);  // explicit: the same rounding wherever this is inlined
    }
    return ss;
}

// momentum + nesterov + bf16 cast (+ transpose) of the gradient into the LDS image X; returns the
// thread's sum of squares of the bf16 values.  Separate function so the restrict qualifiers let the
// compiler overlap the iterations' loads with the previous stores.
__device__ __forceinline__ float muon_prologue(const float *__restrict__ grad, float *__restrict__ mom, char *sX,
                                               int px, int R, int C, bool tr, float coef, float mu, bool nesterov,
                                               int tid, int mr0 = 0, int mr1 = 1 << 30) {
    // (rows [mr0, mr1) of the momentum are written back: a multi-CU part computes the whole image
    // -- every part the same values -- and owns the momentum rows of its row block)
    float ss = 0.0f;
    if (C & 3) {  // a row length that is not a whole number of float4 (GameURM's [64, 3] stem): per element
        for (int e = tid; e < R * C; e += kMuonThreads) {
            const float gv = grad[e] * coef;
            const float bv = mom[e] + (1.0f - mu) * (gv - mom[e]);
            const float ub = round_bf(nesterov ? bv - (bv - gv) * (1.0f - mu) : bv);
            ss += ub * ub;
            const int i = e / C, j = e - i * C;
            reinterpret_cast<uint16_t *>(sX + (tr ? j * px : i * px))[tr ? i : j] = (uint16_t)f2bf(ub);
            mom[e] = bv;
        }
        return ss;
    }
    const int n4 = (R * C) >> 2;
    // kB float4 of the gradient and of the momentum in flight per thread before any is used: one
    // HBM round trip per batch instead of one per element group (a single CU streams the matrix)
    constexpr int kB = 6;
    for (int base = tid; base < n4; base += kB * kMuonThreads) {
        float4 g4[kB], b4[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int e4 = base + u * kMuonThreads;
            g4[u] = e4 < n4 ? reinterpret_cast<const float4 *>(grad)[e4] : make_float4(0.f, 0.f, 0.f, 0.f);
            b4[u] = e4 < n4 ? reinterpret_cast<const float4 *>(mom)[e4] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int v = 0; v < kB; v++) {
            const int e4 = base + v * kMuonThreads;
            if (e4 >= n4) continue;
            float bv[4], ub[4];
            ss += momentum4(g4[v], b4[v], coef, mu, nesterov, bv, ub);
            const int i = (4 * e4) / C, j0 = 4 * e4 - i * C;  // C % 4 == 0: a float4 stays in one row
            if (tr) {
#pragma unroll
                for (int u = 0; u < 4; u++) reinterpret_cast<uint16_t *>(sX + (j0 + u) * px)[i] = (uint16_t)f2bf(ub[u]);
            } else {
                *reinterpret_cast<uint2 *>(sX + i * px + 2 * j0) = make_uint2(pack_bf2(ub[0], ub[1]), pack_bf2(ub[2], ub[3]));
            }
            if (i >= mr0 && i < mr1) reinterpret_cast<float4 *>(mom)[e4] = make_float4(bv[0], bv[1], bv[2], bv[3]);
        }
    }
    return ss;
}

// p decay - x step without contraction: the same bits in every inlining context (the one-CU epilogue
// and the multi-CU parts' prefetched form)
__device__ __forceinline__ float muon_update(float p, float decay, float x, float step) {
#pragma clang fp contract(off)
    return p * decay - x * step;
}

__device__ __forceinline__ void muon_epilogue(float *__restrict__ param, uint16_t *__restrict__ pbf, const char *sX,
                                              int px, int R, int C, bool tr, float decay, float step, int tid,
                                              int pr0 = 0, int pr1 = 1 << 30, uint16_t *frag = nullptr,
                                              int frag_row = 0) {  // parameter rows [pr0, pr1)
    if (C & 3) {  // per element (see muon_prologue)
        for (int e = tid; e < R * C; e += kMuonThreads) {
            const int i = e / C, j = e - i * C;
            const float x = bf2f(reinterpret_cast<const uint16_t *>(sX + (tr ? j * px : i * px))[tr ? i : j]);
            const float pv = muon_update(param[e], decay, x, step);
            param[e] = pv;
            if (pbf) pbf[e] = (uint16_t)f2bf(pv);
        }
        return;
    }
    const int e0 = tr ? 0 : (pr0 < R ? pr0 : R) * C / 4;  // (the multi-CU parts are square: tr false)
    const int n4 = tr ? (R * C) >> 2 : (pr1 < R ? pr1 : R) * C / 4;
    constexpr int kB = 8;
    for (int base = e0 + tid; base < n4; base += kB * kMuonThreads) {
        float4 p4[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int e4 = base + u * kMuonThreads;
            p4[u] = e4 < n4 ? reinterpret_cast<const float4 *>(param)[e4] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int v = 0; v < kB; v++) {
            const int e4 = base + v * kMuonThreads;
            if (e4 >= n4) continue;
            float pv[4] = {p4[v].x, p4[v].y, p4[v].z, p4[v].w};
            const int i = (4 * e4) / C, j0 = 4 * e4 - i * C;
            float x[4];
            if (tr) {
#pragma unroll
                for (int u = 0; u < 4; u++) x[u] = bf2f(reinterpret_cast<const uint16_t *>(sX + (j0 + u) * px)[i]);
            } else {
                const uint2 w = *reinterpret_cast<const uint2 *>(sX + i * px + 2 * j0);
                x[0] = bf2f(w.x & 0xFFFFu);
                x[1] = bf2f(w.x >> 16);
                x[2] = bf2f(w.y & 0xFFFFu);
                x[3] = bf2f(w.y >> 16);
            }
#pragma unroll
            for (int u = 0; u < 4; u++) pv[u] = muon_update(pv[u], decay, x[u], step);
            reinterpret_cast<float4 *>(param)[e4] = make_float4(pv[0], pv[1], pv[2], pv[3]);
            if (pbf) reinterpret_cast<uint2 *>(pbf)[e4] = make_uint2(pack_bf2(pv[0], pv[1]), pack_bf2(pv[2], pv[3]));
            if (frag && !tr)
#pragma unroll
                for (int u = 0; u < 4; u++) head_frag_put(frag, frag_row + i, j0 + u, pv[u]);
        }
    }
}

// ------------------------------------------------------------------ square Newton-Schulz ------
// the square sizes of the fast path: 0 = generic schedule
__host__ __device__ constexpr int ns_square_kind(int n) {
    return n == 196 ? 1 : n == 192 ? 2 : n == 128 ? 3 : n == 64 ? 4 : n == 32 ? 5 : 0;
}

// Row pitch (bytes) of an LDS image with `cols` columns of a matrix whose other side is `rows`.
// The square fast path pads to a pitch of 16 * (2 * odd) bytes: a 16 x 16 row-fragment read
// (ds_read_b128, lane (g, c) -> row c, 16-byte unit g) then hits 16 distinct 4-bank groups in each
// of its four lane groups (P / 16 = 25 at 196 columns puts lanes 3 and 20 on one group: 2-way).
__host__ __device__ constexpr int muon_pitch(int rows, int cols) {
    return rows == cols && ns_square_kind(cols) ? (cols == 196 || cols == 192 ? 416 : cols == 128 ? 288 : cols == 64 ? 160 : 96)
                                                : ((cols + 7) & ~7) * 2;
}
// The h x h block weights (the update's critical path: every matrix of the model runs in its own
// block of one launch, the square ones take the longest) on a schedule fixed at compile time:
//   * the NT = ceil(n / 16) tile rows split into parts of at most 4 tiles (13 = 4+3+3+3, 12 =
//     3+3+3+3, 8 = 4+4); a block is part x part (up to 16 accumulators: 8 fragment reads per k-step for 16
//     MFMAs -- the CU's LDS, shared by its four SIMDs, then keeps pace with the matrix cores);
//   * the blocks of a product go to the 8 waves by a greedy longest-first assignment that balances
//     the four SIMDs, then the two waves (w, w + 4) of each; every wave runs its own straight-line
//     code (a switch on the wave index), so accumulators, LDS addresses and edge clamps are all
//     compile-time: rows past n are clamped to the last (they only feed outputs that are never
//     stored) and the K overflow of the last k-step (k >= round8(n): the next row's data) is cut by
//     zeroing those B fragments;
//   * G = X X^T and U = b G + c G G are symmetric: only tiles on and above the diagonal are
//     computed, each off-diagonal one stored twice (transposed and mirrored).
// Per output tile the MFMA sequence (init from the scaled old value, k-steps in order) is the
// generic path's, so both compute bitwise the same iterate.
constexpr int kNsMaxBlocks = 4;  // per wave and product
constexpr int kNsMaxTiles = 16;  // accumulator tiles per wave (64 of the 128 VGPRs at 4 waves per SIMD)

constexpr int ns_nparts(int NT, bool sym) {
    int n = NT >= 4 ? ((NT + 3) / 4 > 4 ? (NT + 3) / 4 : 4) : NT;
    const int n3 = (NT + 2) / 3;
    if (sym && n3 > n && n3 * (n3 + 1) / 2 <= kMuonWaves && n3 <= 8) n = n3;
    return n;
}

struct NsParts {
    int n, start[8], size[8];
    // 4 parts (16 blocks: one per wave of the full product) from 4 tiles up, of at most 4 tiles.
    // Symmetric products (sym: the upper-triangle blocks only) take parts of at most 3 tiles when
    // their block count still fits the 16 waves (round 6: at h 196, 5 parts -> 15 blocks of <= 9 tiles
    // instead of 10 blocks of <= 12: the slowest wave of G = X X^T carries 3/4 of the MFMAs)
    constexpr NsParts(int NT, bool sym = false) : n(ns_nparts(NT, sym)), start{}, size{} {
        const int base = NT / n, extra = NT % n;
        int s0 = 0;
        for (int i = 0; i < n; i++) {
            size[i] = base + (i < extra ? 1 : 0);
            start[i] = s0;
            s0 += size[i];
        }
    }
};

struct NsSchedule {
    int bi[2][kMuonWaves][kNsMaxBlocks], bj[2][kMuonWaves][kNsMaxBlocks];  // [sym][wave][i]: part indices
    int cnt[2][kMuonWaves], tiles[2][kMuonWaves];
    constexpr NsSchedule(int NT) : bi{}, bj{}, cnt{}, tiles{} {
        for (int sym = 0; sym < 2; sym++) {
            const NsParts pt(NT, sym != 0);
            int ai[16] = {}, aj[16] = {}, cost[16] = {}, n = 0;
            for (int i = 0; i < pt.n; i++)
                for (int j = sym ? i : 0; j < pt.n; j++) {
                    ai[n] = i;
                    aj[n] = j;
                    // MFMA work: a symmetric product's diagonal block runs its upper triangle only
                    cost[n] = sym && i == j ? pt.size[i] * (pt.size[i] + 1) / 2 : pt.size[i] * pt.size[j];
                    n++;
                }
            for (int i = 1; i < n; i++)  // stable insertion sort, cost descending
                for (int j = i; j > 0 && cost[j] > cost[j - 1]; j--) {
                    int t = cost[j]; cost[j] = cost[j - 1]; cost[j - 1] = t;
                    t = ai[j]; ai[j] = ai[j - 1]; ai[j - 1] = t;
                    t = aj[j]; aj[j] = aj[j - 1]; aj[j - 1] = t;
                }
            int simd[4] = {}, wave[kMuonWaves] = {};
            for (int i = 0; i < n; i++) {
                int sm = 0;
                for (int k = 1; k < 4; k++)
                    if (simd[k] < simd[sm]) sm = k;
                int w = sm;  // the SIMD's least loaded wave (waves w, w + 4, ... share SIMD w % 4)
                for (int k = sm + 4; k < kMuonWaves; k += 4)
                    if (wave[k] < wave[w]) w = k;
                simd[sm] += cost[i];
                wave[w] += cost[i];
                bi[sym][w][cnt[sym][w]] = ai[i];
                bj[sym][w][cnt[sym][w]] = aj[i];
                cnt[sym][w]++;
                tiles[sym][w] += pt.size[ai[i]] * pt.size[aj[i]];  // accumulator slots
            }
        }
    }
    constexpr int offset(int sym, int w, int u, const NsParts &pt) const {  // first slot of block u
        int o = 0;
        for (int i = 0; i < u; i++) o += pt.size[bi[sym][w][i]] * pt.size[bj[sym][w][i]];
        return o;
    }
};

constexpr bool ns_schedule_fits(int NT) {
    const NsSchedule s(NT);
    for (int sym = 0; sym < 2; sym++)
        for (int w = 0; w < kMuonWaves; w++)
            if (s.cnt[sym][w] > kNsMaxBlocks || s.tiles[sym][w] > kNsMaxTiles) return false;
    return true;
}
static_assert(ns_schedule_fits(13) && ns_schedule_fits(12) && ns_schedule_fits(8) && ns_schedule_fits(4) &&
                  ns_schedule_fits(2), "square Newton-Schulz schedule exceeds the register budget");

template <int N>
struct NsShape {
    static constexpr int NT = (N + 15) / 16, KPAD = (N + 7) & ~7, KS = (KPAD + 31) / 32;
    static constexpr int P = muon_pitch(N, N);
};

// the A / B fragments of k-step ks of a block (per-lane row bases pa / pb)
template <int N, bool AROWS, int BI, int BJ>
__device__ __forceinline__ void ns_frags(int ks, const char *const (&pa)[BI], const char *const (&pb)[BJ],
                                         bf16x8_t (&fa)[BI], bf16x8_t (&fb)[BJ], int g) {
    using S = NsShape<N>;
    constexpr int P = S::P;
#pragma unroll
    for (int y = 0; y < BJ; y++) {
        uint4 v = *reinterpret_cast<const uint4 *>(pb[y] + 64 * ks);
        if (ks == S::KS - 1 && 32 * S::KS > S::KPAD) {  // k >= round8(n) reads the next row: zero
            const bool kin = 32 * ks + 8 * g < S::KPAD;
            v = kin ? v : make_uint4(0u, 0u, 0u, 0u);
        }
        fb[y] = __builtin_bit_cast(bf16x8_t, v);
    }
#pragma unroll
    for (int x = 0; x < BI; x++) {
        if (AROWS) {
            fa[x] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4 *>(pa[x] + 64 * ks));
        } else {  // A = X^T: X[32 ks + 8 g + j][16 ti + i], two transposing reads (rows past n fall in
                  // the G image behind X: finite, and their B is zero)
            const char *a1 = pa[x] + 32 * ks * P;
            const s16x4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)a1);
            const s16x4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(a1 + 4 * P));
            fa[x] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(t1, t2, 0, 1, 2, 3, 4, 5, 6, 7));
        }
    }
}

// init + k loop of one BI x BJ block at tiles (TI0, TJ0) into acc[OFF ...]
template <int N, bool SYM, bool AROWS, int KEEP, int BI, int BJ, int TI0, int TJ0, int OFF, int T>
__device__ __forceinline__ void ns_block(f32x4_t (&acc)[T], uint2 (&kept)[T], const char *A, const char *B,
                                         const char *out, float ratio, bool init, int g, int c, int ltr) {
    using S = NsShape<N>;
    constexpr int P = S::P;
    constexpr bool DIAG = SYM && TI0 == TJ0;  // upper triangle only
#pragma unroll
    for (int x = 0; x < BI; x++)
#pragma unroll
        for (int y = 0; y < BJ; y++) {
            if (DIAG && x > y) continue;
            f32x4_t a0 = {0.0f, 0.0f, 0.0f, 0.0f};
            if (KEEP == 2) {  // the old value is this lane's own output of the previous product
                const uint2 w = kept[OFF + x * BJ + y];
                a0 = f32x4_t{ratio * bf2f(w.x & 0xFFFFu), ratio * bf2f(w.x >> 16), ratio * bf2f(w.y & 0xFFFFu),
                             ratio * bf2f(w.y >> 16)};
            } else if (init) {  // the old value, scaled (clamped into the image: unused lanes never store)
                const int orow = min(16 * (TJ0 + y) + c, N - 1), ocol = min(16 * (TI0 + x) + 4 * g, N - 4);
                const uint2 w = *reinterpret_cast<const uint2 *>(out + orow * P + ocol * 2);
                a0 = f32x4_t{ratio * bf2f(w.x & 0xFFFFu), ratio * bf2f(w.x >> 16), ratio * bf2f(w.y & 0xFFFFu),
                             ratio * bf2f(w.y >> 16)};
            }
            acc[OFF + x * BJ + y] = a0;
        }
    const char *pa[BI];
    const char *pb[BJ];
#pragma unroll
    for (int x = 0; x < BI; x++)
        pa[x] = AROWS ? A + min(16 * (TI0 + x) + c, N - 1) * P + 16 * g : A + ltr + 32 * (TI0 + x);
#pragma unroll
    for (int y = 0; y < BJ; y++) pb[y] = B + min(16 * (TJ0 + y) + c, N - 1) * P + 16 * g;
    // (4 waves per SIMD: the other waves' MFMAs cover one wave's fragment reads)
#pragma unroll
    for (int ks = 0; ks < S::KS; ks++) {
        bf16x8_t fa[BI], fb[BJ];
        ns_frags<N, AROWS, BI, BJ>(ks, pa, pb, fa, fb, g);
#pragma unroll
        for (int x = 0; x < BI; x++)
#pragma unroll
            for (int y = 0; y < BJ; y++) {
                if (DIAG && x > y) continue;
                acc[OFF + x * BJ + y] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[x], fb[y], acc[OFF + x * BJ + y], 0, 0, 0);
            }
    }
}

// The mirrored tile of a symmetric product, out[row][col] for the lane's D[4g .. 4g+3][c]: a 4 x 4
// transpose within each quad of lanes (c = 4m + k; two DPP exchanges, at k ^ 2 on whole dwords and
// at k ^ 1 on bf16 halves) gives lane k row 4g + k, columns 4m .. 4m + 3 -- one 8-byte write whose
// 16-lane groups cover 16 distinct bank quads (4 rows x 4 column chunks at the 416-byte pitch).
__device__ __forceinline__ uint2 quad_transpose_bf16(uint32_t w0, uint32_t w1, int k) {
    // stage A: lanes k < 2 keep rows {0,1} (w0) and take the partner's w0; lanes k >= 2 rows {2,3}
    const uint32_t sa = k < 2 ? w1 : w0;
    const uint32_t ra = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sa, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
    const uint32_t p0 = k < 2 ? w0 : ra, p1 = k < 2 ? ra : w1;
    // stage B: even lanes send their high halves, odd lanes their low halves
    const bool even = (k & 1) == 0;
    const uint32_t sb = __builtin_amdgcn_perm(p1, p0, even ? 0x07060302u : 0x05040100u);
    const uint32_t rb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sb, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
    return make_uint2(__builtin_amdgcn_perm(rb, p0, even ? 0x05040100u : 0x03020504u),
                      __builtin_amdgcn_perm(rb, p1, even ? 0x07060100u : 0x03020706u));
}

// the transposed (and for symmetric products mirrored) bf16 store of one block; KEEP == 1: the
// lane's packed values also stay in `kept` (the next product's initial value)
template <int N, bool SYM, int KEEP, int BI, int BJ, int TI0, int TJ0, int OFF, int T>
__device__ __forceinline__ void ns_store(const f32x4_t (&acc)[T], uint2 (&kept)[T], char *out, float alpha, int g,
                                         int c) {
    constexpr int P = NsShape<N>::P;
    constexpr bool DIAG = SYM && TI0 == TJ0;
    const int k = c & 3, m = c >> 2;
#pragma unroll
    for (int x = 0; x < BI; x++)
#pragma unroll
        for (int y = 0; y < BJ; y++) {
            if (DIAG && x > y) continue;
            const int ti = TI0 + x, tj = TJ0 + y;
            const f32x4_t v = acc[OFF + x * BJ + y];
            const uint32_t w0 = pack_bf2(alpha * v[0], alpha * v[1]), w1 = pack_bf2(alpha * v[2], alpha * v[3]);
            if (KEEP == 1) kept[OFF + x * BJ + y] = make_uint2(w0, w1);
            if (SYM && ti < tj) {  // the mirrored tile: all lanes take part in the exchange
                const uint2 t = quad_transpose_bf16(w0, w1, k);
                const int row = 16 * ti + 4 * g + k, col0 = 16 * tj + 4 * m;
                if (row < N && col0 < N) *reinterpret_cast<uint2 *>(out + row * P + col0 * 2) = t;
            }
            const int col = 16 * tj + c, row0 = 16 * ti + 4 * g;
            if (col < N && row0 < N) *reinterpret_cast<uint2 *>(out + col * P + row0 * 2) = make_uint2(w0, w1);
        }
}

template <int N, bool SYM, bool AROWS, int KEEP, int W, int U, int T>
__device__ __forceinline__ void ns_blocks(f32x4_t (&acc)[T], uint2 (&kept)[T], const char *A, const char *B,
                                          const char *out, float ratio, bool init, int g, int c, int ltr) {
    constexpr NsParts pt(NsShape<N>::NT, SYM);
    constexpr NsSchedule sch(NsShape<N>::NT);
    if constexpr (U < sch.cnt[SYM][W]) {
        constexpr int bi = sch.bi[SYM][W][U], bj = sch.bj[SYM][W][U];
        ns_block<N, SYM, AROWS, KEEP, pt.size[bi], pt.size[bj], pt.start[bi], pt.start[bj], sch.offset(SYM, W, U, pt)>(
            acc, kept, A, B, out, ratio, init, g, c, ltr);
        ns_blocks<N, SYM, AROWS, KEEP, W, U + 1>(acc, kept, A, B, out, ratio, init, g, c, ltr);
    }
}

template <int N, bool SYM, int KEEP, int W, int U, int T>
__device__ __forceinline__ void ns_stores(const f32x4_t (&acc)[T], uint2 (&kept)[T], char *out, float alpha, int g,
                                          int c) {
    constexpr NsParts pt(NsShape<N>::NT, SYM);
    constexpr NsSchedule sch(NsShape<N>::NT);
    if constexpr (U < sch.cnt[SYM][W]) {
        constexpr int bi = sch.bi[SYM][W][U], bj = sch.bj[SYM][W][U];
        ns_store<N, SYM, KEEP, pt.size[bi], pt.size[bj], pt.start[bi], pt.start[bj], sch.offset(SYM, W, U, pt)>(
            acc, kept, out, alpha, g, c);
        ns_stores<N, SYM, KEEP, W, U + 1>(acc, kept, out, alpha, g, c);
    }
}

template <int N, bool SYM>
constexpr int ns_tiles(int w) {
    constexpr NsSchedule sch(NsShape<N>::NT);
    return sch.tiles[SYM][w] > 0 ? sch.tiles[SYM][w] : 1;
}

// One product on wave W: out <- transpose(alpha * (init + A B)), init = (beta / alpha) * old out
// (transposed) when beta != 0.  KEEP == 1: the packed outputs also stay in `kept`; KEEP == 2: the
// old values come from `kept` (this wave computed them in the previous product, same schedule).
template <int N, bool SYM, bool AROWS, int KEEP, int W>
__device__ __forceinline__ void ns_product_w(const char *A, const char *B, char *out, float alpha, float beta,
                                             uint2 (&kept)[ns_tiles<N, SYM>(W)], int lane) {
    constexpr int T = ns_tiles<N, SYM>(W);
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, c = lane & 15;
    const int ltr = (8 * g + q) * NsShape<N>::P + 8 * p;  // transposing reads: row 8 g + q, column 4 p
    f32x4_t acc[T];
    ns_blocks<N, SYM, AROWS, KEEP, W, 0>(acc, kept, A, B, out, beta / alpha, beta != 0.0f, g, c, ltr);
    __syncthreads();  // every read of the old `out` (and of A / B when they alias it) is done
    ns_stores<N, SYM, KEEP, W, 0>(acc, kept, out, alpha, g, c);
    __syncthreads();
}

// The Newton-Schulz iterations on wave W: its own straight-line code for all three products, the
// lane index laundered per product so the compiler recomputes the few per-lane addresses instead
// of hoisting every product's out of the loop (register spills at 128 VGPRs).
template <int N, int W>
__device__ __forceinline__ void ns_square_w(char *sX, char *sG, const MuonArgs &args, int lane) {
    for (int it = 0; it < args.steps; it++) {
        uint2 kept[ns_tiles<N, true>(W)];  // G's tiles, U's initial value
        uint2 unused[ns_tiles<N, false>(W)];
        int l = lane;
        asm volatile("" : "+v"(l));
        ns_product_w<N, true, true, 1, W>(sX, sX, sG, 1.0f, 0.0f, kept, l);          // G = X X^T
        l = lane;
        asm volatile("" : "+v"(l));
        ns_product_w<N, true, true, 2, W>(sG, sG, sG, args.c, args.b, kept, l);      // U = b G + c G G
        l = lane;
        asm volatile("" : "+v"(l));
        ns_product_w<N, false, false, 0, W>(sX, sG, sX, 1.0f, args.a, unused, l);    // X = a X + U X
    }
}

template <int N>
__device__ __forceinline__ void ns_square(char *sX, char *sG, const MuonArgs &args, int wave, int lane) {
    switch (wave) {  // wave-uniform
    case 0: ns_square_w<N, 0>(sX, sG, args, lane); break;
    case 1: ns_square_w<N, 1>(sX, sG, args, lane); break;
    case 2: ns_square_w<N, 2>(sX, sG, args, lane); break;
    case 3: ns_square_w<N, 3>(sX, sG, args, lane); break;
    case 4: ns_square_w<N, 4>(sX, sG, args, lane); break;
    case 5: ns_square_w<N, 5>(sX, sG, args, lane); break;
    case 6: ns_square_w<N, 6>(sX, sG, args, lane); break;
    case 7: ns_square_w<N, 7>(sX, sG, args, lane); break;
    case 8: ns_square_w<N, 8>(sX, sG, args, lane); break;
    case 9: ns_square_w<N, 9>(sX, sG, args, lane); break;
    case 10: ns_square_w<N, 10>(sX, sG, args, lane); break;
    case 11: ns_square_w<N, 11>(sX, sG, args, lane); break;
    case 12: ns_square_w<N, 12>(sX, sG, args, lane); break;
    case 13: ns_square_w<N, 13>(sX, sG, args, lane); break;
    case 14: ns_square_w<N, 14>(sX, sG, args, lane); break;
    default: ns_square_w<N, 15>(sX, sG, args, lane); break;
    }
}

// ------------------------------------------------------------------ multi-CU Newton-Schulz ----
// A square h x h matrix (h = 196 / 192) on `np` blocks (CUs).  Every block holds the whole X and
// computes G = X X^T whole (the symmetric schedule above: replicated, so no exchange of G); each
// block then computes only its row block R of U = b G + c G G and of X' = a X + U X (tile rows
// [t0, t1)), and the blocks exchange their rows of X' once per iteration through a global image
// (agent-scope hand-off, cdna_hip_programming.md Guideline 16: write-through 8-byte stores, one
// counter add per block after a drain + barrier, a relaxed poll, one acquire, plain loads).  Per
// output tile the MFMA sequence (init from the scaled old value, k-steps in order) is the
// single-block path's, with the operand roles of the X product swapped (A = U rows, B = X by the
// transposing read instead of A = X^T, B^T = U rows): the same products summed in the same order.
typedef __attribute__((address_space(1))) uint32_t gu32_t;
typedef __attribute__((address_space(1))) uint64_t gu64_t;

// MUON_TRACE builds (tools/trace_muon.py): per block, the shader clock at phase points, in the
// workspace after the exchange images ([block][64] uint64, slot 0 = number of points)
#ifdef MUON_TRACE
constexpr int kMuonTraceBytes = kMuonMaxJobs * 64 * 8;
#define MUON_TP(args_)                                                                      \
    do {                                                                                    \
        if (threadIdx.x == 0 && (args_).trace) {                                            \
            if (blockIdx.x >= (unsigned)kMuonMaxJobs) {                                     \
                printf("MUON_CHECK trace block %u out of range\n", blockIdx.x);              \
            } else {                                                                        \
                uint64_t *t_ = (args_).trace + 64 * blockIdx.x;                             \
                const uint64_t k_ = t_[0] + 1;                                              \
                if (k_ < 64) t_[k_] = __builtin_amdgcn_s_memtime();                         \
                t_[0] = k_;                                                                 \
            }                                                                               \
        }                                                                                   \
    } while (0)
// trace builds also bound-check every exchange-image access and the job table (printf + skip)
#define MUON_CHECK(cond_, what_, a_, b_)                                                    \
    do {                                                                                    \
        if (!(cond_)) printf("MUON_CHECK %s blk %u tid %u: %lld %lld\n", what_, blockIdx.x, threadIdx.x, \
                             (long long)(a_), (long long)(b_));                             \
    } while (0)
#else
constexpr int kMuonTraceBytes = 0;
#define MUON_TP(args_) do {} while (0)
#define MUON_CHECK(cond_, what_, a_, b_) do {} while (0)
#endif

// G = X X^T alone, on the square schedule (no kept tiles: the row-block U product re-reads G)
template <int N, int W>
__device__ __forceinline__ void ns_g_w(char *sX, char *sG, int lane) {
    uint2 unused[ns_tiles<N, true>(W)];
    int l = lane;
    asm volatile("" : "+v"(l));
    ns_product_w<N, true, true, 0, W>(sX, sX, sG, 1.0f, 0.0f, unused, l);
}

template <int N>
__device__ __forceinline__ void ns_square_g(char *sX, char *sG, int wave, int lane) {
    switch (wave) {  // wave-uniform
    case 0: ns_g_w<N, 0>(sX, sG, lane); break;
    case 1: ns_g_w<N, 1>(sX, sG, lane); break;
    case 2: ns_g_w<N, 2>(sX, sG, lane); break;
    case 3: ns_g_w<N, 3>(sX, sG, lane); break;
    case 4: ns_g_w<N, 4>(sX, sG, lane); break;
    case 5: ns_g_w<N, 5>(sX, sG, lane); break;
    case 6: ns_g_w<N, 6>(sX, sG, lane); break;
    case 7: ns_g_w<N, 7>(sX, sG, lane); break;
    case 8: ns_g_w<N, 8>(sX, sG, lane); break;
    case 9: ns_g_w<N, 9>(sX, sG, lane); break;
    case 10: ns_g_w<N, 10>(sX, sG, lane); break;
    case 11: ns_g_w<N, 11>(sX, sG, lane); break;
    case 12: ns_g_w<N, 12>(sX, sG, lane); break;
    case 13: ns_g_w<N, 13>(sX, sG, lane); break;
    case 14: ns_g_w<N, 14>(sX, sG, lane); break;
    default: ns_g_w<N, 15>(sX, sG, lane); break;
    }
}

template <int N>
struct McShape {
    static constexpr int NT = (N + 15) / 16, KPAD = (N + 7) & ~7, KS = (KPAD + 31) / 32;
    static constexpr int P = muon_pitch(N, N);
};

// The old value of output tile (ti, tj) in the accumulator layout (lane (g, c): rows 16 ti + 4 g ..
// + 3 of column 16 tj + c), scaled: from a SYMMETRIC image by one 8-byte read of the transposed
// position, else by a row read + the quad transpose (a 4 x 4 transpose is its own inverse).
template <int N, bool SYM>
__device__ __forceinline__ f32x4_t mc_init(const char *img, int ti, int tj, float ratio, int g, int c) {
    constexpr int P = McShape<N>::P;
    uint32_t w0, w1;
    if (SYM) {
        const int row = min(16 * tj + c, N - 1), col = min(16 * ti + 4 * g, N - 4);
        const uint2 w = *reinterpret_cast<const uint2 *>(img + row * P + col * 2);
        w0 = w.x;
        w1 = w.y;
    } else {
        const int k = c & 3, m = c >> 2;
        const int row = min(16 * ti + 4 * g + k, N - 1), col = 16 * tj + 4 * m;  // col < 16 NT: inside the pitch
        const uint2 w = *reinterpret_cast<const uint2 *>(img + row * P + col * 2);
        const uint2 t = quad_transpose_bf16(w.x, w.y, k);
        w0 = t.x;
        w1 = t.y;
    }
    return f32x4_t{ratio * bf2f(w0 & 0xFFFFu), ratio * bf2f(w0 >> 16), ratio * bf2f(w1 & 0xFFFFu), ratio * bf2f(w1 >> 16)};
}

// acc[x] (+)= sum_ks A[16 (t0 + x) + ..][k] B[k][16 tj + ..] for the RB tile rows of the block.
// A: rows of image A (row reads; rows past N clamped, k past KPAD cut to zero: they read the next
// row).  B: BT_ROWS -- B^T rows = rows 16 tj + c of image B (row reads; B symmetric), else B = image
// B read by columns (the transposing read; rows past N read the image behind it: finite, times a
// zero A fragment).
template <int N, int RB, bool BT_ROWS>
__device__ __forceinline__ void mc_mfma(const char *A, const char *B, int t0, int tj, int lane, f32x4_t (&acc)[RB]) {
    using S = McShape<N>;
    constexpr int P = S::P;
    const int g = lane >> 4, c = lane & 15, q = (lane >> 2) & 3, p = lane & 3;
    const char *pa[RB];
#pragma unroll
    for (int x = 0; x < RB; x++) pa[x] = A + min(16 * (t0 + x) + c, N - 1) * P + 16 * g;
    const char *pb = BT_ROWS ? B + min(16 * tj + c, N - 1) * P + 16 * g : B + (8 * g + q) * P + 8 * p + 32 * tj;
#pragma unroll
    for (int ks = 0; ks < S::KS; ks++) {
        const bool kin = 32 * ks + 8 * g < S::KPAD;
        bf16x8_t fb;
        if (BT_ROWS) {
            uint4 v = *reinterpret_cast<const uint4 *>(pb + 64 * ks);
            if (ks == S::KS - 1 && 32 * S::KS > S::KPAD) v = kin ? v : make_uint4(0u, 0u, 0u, 0u);
            fb = __builtin_bit_cast(bf16x8_t, v);
        } else {
            const char *b1 = pb + 32 * ks * P;
            const s16x4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)b1);
            const s16x4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(b1 + 4 * P));
            fb = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(t1, t2, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int x = 0; x < RB; x++) {
            uint4 v = *reinterpret_cast<const uint4 *>(pa[x] + 64 * ks);
            if (ks == S::KS - 1 && 32 * S::KS > S::KPAD) v = kin ? v : make_uint4(0u, 0u, 0u, 0u);
            acc[x] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, v), fb, acc[x], 0, 0, 0);
        }
    }
}

// lane (g, c) of tile (ti, tj): alpha * acc as rows 16 ti + 4 g + k, columns 16 tj + 4 m .. + 3
// (c = 4 m + k) -- one 8-byte row segment per lane; columns past N become zero (the image padding)
template <int N>
__device__ __forceinline__ uint2 mc_row_segment(const f32x4_t &v, float alpha, int tj, int c) {
    const uint32_t w0 = pack_bf2(alpha * v[0], alpha * v[1]), w1 = pack_bf2(alpha * v[2], alpha * v[3]);
    const uint2 t = quad_transpose_bf16(w0, w1, c & 3);
    return 16 * tj + 4 * (c >> 2) < N ? t : make_uint2(0u, 0u);
}

// One row-block product of this block: tiles (t0 .. t0 + RB - 1, tj = wave) for waves < NT.
// SYM_B: U = c (b/c G + G G) (A = G rows, B^T = G rows, old value G); else X' = a X + U X (A = U
// rows of sG, B = X columns of sX, old value X).  The result stays in acc (stored by the caller).
template <int N, int RB, bool U_PRODUCT>
__device__ __forceinline__ void mc_product(const char *sX, const char *sG, int t0, int wave, int lane, float ratio,
                                           f32x4_t (&acc)[RB]) {
    const int g = lane >> 4, c = lane & 15;
    const int tj = wave;
#pragma unroll
    for (int x = 0; x < RB; x++) acc[x] = mc_init<N, U_PRODUCT>(U_PRODUCT ? sG : sX, t0 + x, tj, ratio, g, c);
    if (U_PRODUCT) mc_mfma<N, RB, true>(sG, sG, t0, tj, lane, acc);
    else mc_mfma<N, RB, false>(sG, sX, t0, tj, lane, acc);
}

// bounded relaxed poll of a counter (one wave); false after `limit` polls (~0.2 s at the default
// 2^21: a part that never became resident).  No wave spins forever; the results of the launch are
// then garbage, so the timeout is recorded in the matrix's flag and counted in the sticky error word
// that the host reads with the train step's metrics and raises on (FusedMuonAdamW.check_errors).
__device__ __forceinline__ bool mc_wait(gu32_t *ctr, uint32_t target, gu32_t *err, gu32_t *errors, uint32_t limit) {
    for (uint32_t spins = 0;; spins++) {
        if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
        if (spins >= limit) {
            if ((threadIdx.x & 63) == 0) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_add(errors, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

template <int N, int RB>
__device__ __forceinline__ void ns_square_mc_rb(char *sX, char *sG, const MuonArgs &args, int mat, int part, int np,
                                                int wave, int lane, uint32_t ctr0) {
    using S = McShape<N>;
    constexpr int P = S::P;
    const int tid = threadIdx.x, g = lane >> 4, c = lane & 15;
    const int t0 = part * S::NT / np;  // tile rows t0 .. t0 + RB - 1 (RB = (part + 1) NT / np - t0)
    gu32_t *ctr = (gu32_t *)(args.sync + 16 * mat);
    gu32_t *err = (gu32_t *)(args.sync + 16 * mat + 1);
    char *xg = args.xg + mat * args.xg_stride;
    for (int it = 0; it < args.steps; it++) {
        // G = X X^T, whole (the single-block symmetric schedule; two barriers inside)
        ns_square_g<N>(sX, sG, wave, lane);
        MUON_TP(args);
        f32x4_t acc[RB];
        // U rows of this block, in place over G's rows once every wave is done reading G
        if (wave < S::NT) mc_product<N, RB, true>(sX, sG, t0, wave, lane, args.b / args.c, acc);
        __syncthreads();
        if (wave < S::NT)
#pragma unroll
            for (int x = 0; x < RB; x++) {
                const int row = 16 * (t0 + x) + 4 * g + (c & 3);
                const uint2 v = mc_row_segment<N>(acc[x], args.c, wave, c);
                if (row < N) *reinterpret_cast<uint2 *>(sG + row * P + (16 * wave + 4 * (c >> 2)) * 2) = v;
            }
        __syncthreads();
        MUON_TP(args);
        // X' rows of this block
        if (wave < S::NT) mc_product<N, RB, false>(sX, sG, t0, wave, lane, args.a, acc);
        __syncthreads();  // every read of X is done
        MUON_TP(args);
        const bool last = it == args.steps - 1;
        char *img = last ? sX : xg + (it & 1) * N * P;
        if (wave < S::NT)
#pragma unroll
            for (int x = 0; x < RB; x++) {
                const int row = 16 * (t0 + x) + 4 * g + (c & 3);
                const uint2 v = mc_row_segment<N>(acc[x], 1.0f, wave, c);
                if (row < N) {
                    char *dst = img + row * P + (16 * wave + 4 * (c >> 2)) * 2;
                    MUON_CHECK(last || (dst >= xg && dst + 8 <= xg + args.xg_stride), "xg store", dst - xg, args.xg_stride);
                    MUON_CHECK(!last || (16 * wave + 4 * (c >> 2)) * 2 + 8 <= P, "sX store", (16 * wave + 4 * (c >> 2)) * 2, P);
                    if (last) {
                        *reinterpret_cast<uint2 *>(dst) = v;
                    } else {  // write-through: no release fence needed before the counter add
                        const uint64_t w = (uint64_t)v.x | ((uint64_t)v.y << 32);
                        __hip_atomic_store((gu64_t *)dst, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
        if (last) {
            __syncthreads();
            break;
        }
        // hand-off: every storing wave drains, the barrier, one lane adds; one wave polls, acquires
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        MUON_TP(args);
        if (tid == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (wave == 0)
            mc_wait(ctr, ctr0 + (uint32_t)(np * (it + 1)), err, (gu32_t *)(args.sync + kMuonErrWord), args.spin_limit);
        __syncthreads();
        MUON_TP(args);
        // the whole X' (every block's rows, padding columns zero) into the LDS image: every load in
        // flight before the first LDS store (one L2 round trip, not one per 16 KB).  No acquire
        // fence (its L1 invalidate was ~1.7 us per hand-off): the loads are sc1 buffer loads, served
        // by L2 past this CU's L1, every byte was stored sc1 by its producer, whose storing waves all
        // drained (vmcnt(0)) before the barrier behind which one lane adds to the counter, and only
        // the polling wave's match releases the barrier above (MI355X_MICROARCH.md, the hand-off
        // table's first row).  Offsets past N * P read zero (the descriptor's record count).
        const char *src = xg + (it & 1) * N * P;
        MUON_CHECK(src + N * P <= xg + args.xg_stride, "xg image", (it & 1) * N * P + N * P, args.xg_stride);
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(src), (short)0, N * P, 0x00020000);
        constexpr int kCopy = (N * P / 16 + kMuonThreads - 1) / kMuonThreads;
        constexpr int kSc1 = 16;  // cache-policy bit of the buffer load: sc1
        uint4 cv[kCopy];
#pragma unroll
        for (int u = 0; u < kCopy; u++)
            cv[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, (tid + u * kMuonThreads) * 16, 0, kSc1));
#pragma unroll
        for (int u = 0; u < kCopy; u++) {
            const int o = (tid + u * kMuonThreads) * 16;
            if (o < N * P) *reinterpret_cast<uint4 *>(sX + o) = cv[u];
        }
        __syncthreads();
        MUON_TP(args);
    }
}

template <int N>
__device__ __forceinline__ void ns_square_mc(char *sX, char *sG, const MuonArgs &args, int mat, int part, int np,
                                             int wave, int lane, uint32_t ctr0) {
    constexpr int NT = McShape<N>::NT;
    const int rb = (part + 1) * NT / np - part * NT / np;  // block-uniform; the host picks np >= NT / 2
    if (rb == 1) ns_square_mc_rb<N, 1>(sX, sG, args, mat, part, np, wave, lane, ctr0);
    else ns_square_mc_rb<N, 2>(sX, sG, args, mat, part, np, wave, lane, ctr0);
}


// ---- the update's sum of squares of a square 196 / 192 matrix, in ONE order for every schedule
// (one CU, generic, multi-CU): per 16-row tile row t, thread i < 16 N / 4 holds float4 i of the tile
// row (momentum4's fma order), the block sum is a fixed tree (wave xor butterfly, lane 0 of each
// wave, the waves in order), and the tile-row sums are added in tile order.  A multi-CU part
// computes the sums of its own tile rows only and publishes them with its rows of X.

// lane 0's butterfly sum per wave, the waves in order: the same value in every thread
__device__ __forceinline__ float block_sum_fixed(float v, float *red, int tid) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    float t = 0.0f;
#pragma unroll
    for (int w = 0; w < kMuonWaves; w++) t += red[w];
    __syncthreads();
    return t;
}

// the new momentum and the bf16 update of float4 e of a row-major [N, N] matrix: momentum stored,
// the update's 8 bf16 bytes returned, its fma-ordered sum of squares in ss
__device__ __forceinline__ uint2 momentum_q(const float4 &g4, const float4 &b4, float *mom, int e, float coef,
                                            float mu, bool nesterov, float &ss) {
    float bv[4], ub[4];
    ss = momentum4(g4, b4, coef, mu, nesterov, bv, ub);
    reinterpret_cast<float4 *>(mom)[e] = make_float4(bv[0], bv[1], bv[2], bv[3]);
    return make_uint2(pack_bf2(ub[0], ub[1]), pack_bf2(ub[2], ub[3]));
}

// One CU: the momentum of the whole square matrix, its bf16 update into the LDS image X (pitch P),
// and the sum of squares in tile-row order (four tile rows of loads in flight per batch).
template <int N>
__device__ __forceinline__ float tile_prologue(const float *__restrict__ grad, float *__restrict__ mom, char *sX,
                                               float coef, float mu, bool nesterov, float *red, int tid) {
    constexpr int P = muon_pitch(N, N), NT = (N + 15) / 16, C4 = N / 4, TR4 = 16 * C4;
    float total = 0.0f;
    for (int t0 = 0; t0 < NT; t0 += 4) {
        float4 g4[4], b4[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int e = (t0 + u) * TR4 + tid;
            const bool ok = t0 + u < NT && tid < TR4 && e < N * C4;
            g4[u] = ok ? reinterpret_cast<const float4 *>(grad)[e] : make_float4(0.f, 0.f, 0.f, 0.f);
            b4[u] = ok ? reinterpret_cast<const float4 *>(mom)[e] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (t0 + u >= NT) break;  // block-uniform
            const int e = (t0 + u) * TR4 + tid;
            float ss = 0.0f;
            if (tid < TR4 && e < N * C4) {
                const uint2 q = momentum_q(g4[u], b4[u], mom, e, coef, mu, nesterov, ss);
                const int row = e / C4, j0 = 4 * (e - row * C4);
                *reinterpret_cast<uint2 *>(sX + row * P + 2 * j0) = q;
            }
            total += block_sum_fixed(ss, red, tid);
        }
    }
    return total;
}

// X /= max(bf16(sqrt(ss)), eps) over the flat LDS image of nbytes (the zero padding stays zero): 4
// elements per access, four 8-byte groups per thread in flight per pass.  The quotient of the uniform
// divisor: q0 = y (1/nrm), one fma residual, one fma correction -- the correctly rounded fp32 y / nrm
// for every pair of bf16 operands (all 128 x 128 significand pairs checked exactly,
// tools/check_bf16_division.py), zeros passed through with their sign
// y / nrm correctly rounded (the reference's X / X.norm() in fp32), zero kept
__device__ __forceinline__ float norm_qdiv(float y, float nrm, float inv) {
    const float q0 = y * inv;
    const float q = __builtin_fmaf(__builtin_fmaf(-q0, nrm, y), inv, q0);
    return y == 0.0f ? y : q;
}

// 8 bf16 of an image / nrm, re-rounded to bf16 (normalise_image's arithmetic on a 16-byte chunk)
__device__ __forceinline__ uint4 normalise16(const uint4 v, float nrm) {
    const float inv = 1.0f / nrm;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
        o[k] = pack_bf2(norm_qdiv(bf2f(w[k] & 0xFFFFu), nrm, inv), norm_qdiv(bf2f(w[k] >> 16), nrm, inv));
    return make_uint4(o[0], o[1], o[2], o[3]);
}

__device__ __forceinline__ void normalise_image(char *sX, int nbytes, float nrm, int tid) {
    const float inv = 1.0f / nrm;
    auto qdiv = [&](float y) { return norm_qdiv(y, nrm, inv); };
    const int n8 = nbytes >> 3;
    uint2 *img = reinterpret_cast<uint2 *>(sX);
    for (int e0 = tid; e0 < n8; e0 += 4 * kMuonThreads) {
        uint2 w[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int e = e0 + u * kMuonThreads;
            w[u] = e < n8 ? img[e] : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int e = e0 + u * kMuonThreads;
            if (e < n8)
                img[e] = make_uint2(pack_bf2(qdiv(bf2f(w[u].x & 0xFFFFu)), qdiv(bf2f(w[u].x >> 16))),
                                    pack_bf2(qdiv(bf2f(w[u].y & 0xFFFFu)), qdiv(bf2f(w[u].y >> 16))));
        }
    }
}

// the whole N x P-byte global image `src` into the LDS image (sc1 buffer loads: every load in flight
// before the first LDS store; offsets past N * P read zero by the descriptor's record count)
template <int N>
__device__ __forceinline__ void mc_copy_image(char *sX, const char *src, int tid) {
    constexpr int P = McShape<N>::P;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(src), (short)0, N * P, 0x00020000);
    constexpr int kCopy = (N * P / 16 + kMuonThreads - 1) / kMuonThreads;
    constexpr int kSc1 = 16;  // cache-policy bit of the buffer load: sc1
    uint4 cv[kCopy];
#pragma unroll
    for (int u = 0; u < kCopy; u++)
        cv[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, (tid + u * kMuonThreads) * 16, 0, kSc1));
#pragma unroll
    for (int u = 0; u < kCopy; u++) {
        const int o = (tid + u * kMuonThreads) * 16;
        if (o < N * P) *reinterpret_cast<uint4 *>(sX + o) = cv[u];
    }
}

// The AdamW update of the 1-D groups by block b of nb (clip coefficient from the partials).
// the clip's sum of squares from the partials: lane l sums entries l, l + 64, ... in order (one entry
// per lane for g2048_grad_sumsq's 64: grad_norm_kernel's arithmetic), then the wave's xor tree
__device__ __forceinline__ float clip_sumsq(const MuonArgs &args, int lane) {
    float t = 0.0f;
    int i = lane;
    // 8 loads in flight, added in index order (round 5: one dependent L2 round trip per entry was ~2 us
    // on the critical path of every Muon part with the colsum's ~360 partials)
    for (; i + 64 * 7 < args.npartials; i += 64 * 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = args.partials[i + 64 * u];
#pragma unroll
        for (int u = 0; u < 8; u++) t += v[u];
    }
    for (; i < args.npartials; i += 64) t += args.partials[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    return t;
}

__device__ __forceinline__ void adam_blocks(const MuonArgs &args, int b, int nb) {
    float cf = 1.0f;
    if (args.partials) {  // grad_norm_kernel's arithmetic, as in the Muon blocks (same result)
        const float t = clip_sumsq(args, threadIdx.x & 63);
        cf = clip_coef(args.max_norm, sqrtf(t));
    }
    const AdamArgs &a = args.adam;
    const float t = *a.step;
    const float bc1 = 1.0f - powf(a.b1, t), bc2s = sqrtf(1.0f - powf(a.b2, t));
    for (int k = 0; k < a.count; k++) {
        const AdamGroup gr = a.g[k];
        const float lr = a.lr[gr.lr_index];
        for (int64_t i = (int64_t)b * blockDim.x + threadIdx.x; i < gr.n; i += (int64_t)nb * blockDim.x)
            adamw_elem(gr, i, lr, cf, a.b1, a.b2, a.eps, a.wd, bc1, bc2s);
    }
}

// The gradient-clip coefficient of this step: grad_norm_kernel's arithmetic on the grad_sumsq
// partials, in every block (same order, same result); `publish`: write norm / coefficient out.
__device__ __forceinline__ float block_clip_coef(const MuonArgs &args, int tid, bool publish) {
    __shared__ float s_coef;
    if (!args.partials) return args.clip ? *args.clip : 1.0f;
    if (tid < 64) {
        const float t = clip_sumsq(args, tid);
        const float nrm = sqrtf(t);
        const float cf = clip_coef(args.max_norm, nrm);
        if (tid == 0) {
            s_coef = cf;
            if (publish) {
                *args.norm_out = nrm;
                *args.coef_out = cf;
            }
        }
    }
    __syncthreads();
    return s_coef;
}

// A split square matrix (h = 196 / 192) on part `part` of np blocks, the whole job:
//   prologue  this part's tile rows only: gradient + old momentum (loads issued before the clip
//             coefficient's read), the new momentum written back at once (no other part reads these
//             rows), the bf16 update rows into exchange image 1 and the tile rows' sums of squares
//             into the matrix's sync line -- hand-off 0 -- then every part copies the whole image,
//             sums the NT tile-row sums in order and normalises (the one-CU arithmetic:
//             tile_prologue + normalise_image)
//   Newton-Schulz  ns_square_mc_rb, hand-offs 1 .. steps - 1 (image 0, 1, 0, ...)
//   epilogue  this part's parameter rows, then the counters back to zero by the last part.
// The old path read the whole gradient and momentum on every part (308 KB per part for h = 196) and
// wrote its momentum rows only after a second counter said every part had read them.
template <int N>
__device__ __forceinline__ void mc_matrix(char *smem, float *red, const MuonArgs &args, const MuonMat &mt, int mat,
                                          int part, int np, int tid, int wave, int lane) {
    using S = McShape<N>;
    constexpr int P = S::P, NT = S::NT, C4 = N / 4, TR4 = 16 * C4;
    constexpr int PAD8 = (P / 2 - N) / 4;  // 8-byte zero groups of a row's padding columns
    char *sX = smem;
    char *sG = smem + ((N * P + 127) & ~127);
    const int t0 = part * NT / np, rb = (part + 1) * NT / np - t0;  // this part's tile rows (1 or 2)
    gu32_t *line = (gu32_t *)(args.sync + 16 * mat);  // [0] exchange counter [1] timeout flag [2] done [3 + t] tile-row ss
    gu32_t *errors = (gu32_t *)(args.sync + kMuonErrWord);
    char *xg = args.xg + mat * args.xg_stride;
    char *img1 = xg + N * P;
    // own rows' gradient and momentum in flight first
    float4 g4[2], b4[2];
#pragma unroll
    for (int x = 0; x < 2; x++) {
        const int e = (t0 + x) * TR4 + tid;
        const bool ok = x < rb && tid < TR4 && e < N * C4;
        g4[x] = ok ? reinterpret_cast<const float4 *>(mt.grad)[e] : make_float4(0.f, 0.f, 0.f, 0.f);
        b4[x] = ok ? reinterpret_cast<const float4 *>(mt.mom)[e] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    {  // zero both LDS images (their K padding must read as zero) and the 64 bytes behind them (part of
       // the allocation, muon_lds_bytes): the last k-step of a row of G reads 32 bytes past the row (B is
       // zero there), and for G's last row that is past the image -- uninitialised LDS, whose NaN / Inf
       // bit patterns (left by an earlier kernel on the CU) made X NaN for h = 196 on one box (round 5;
       // h = 192 has no ragged k-step; the one-CU path always zeroed them)
        const int bytes = (int)(sG - smem) + ((N * P + 127) & ~127) + 64;
        for (int o = tid * 16; o < bytes; o += kMuonThreads * 16) *reinterpret_cast<uint4 *>(smem + o) = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const float coef = block_clip_coef(args, tid, blockIdx.x == 0);
    MUON_TP(args);
#pragma unroll
    for (int x = 0; x < 2; x++) {
        if (x >= rb) break;  // block-uniform
        const int e = (t0 + x) * TR4 + tid;
        float ss = 0.0f;
        if (tid < TR4 && e < N * C4) {
            const uint2 q = momentum_q(g4[x], b4[x], mt.mom, e, coef, args.momentum, args.nesterov != 0, ss);
            const int row = e / C4, j0 = 4 * (e - row * C4);
            __hip_atomic_store((gu64_t *)(img1 + row * P + 2 * j0), (uint64_t)q.x | ((uint64_t)q.y << 32),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through (the hand-off)
        } else if (tid >= TR4 && tid < TR4 + 16 * PAD8) {  // the rows' padding columns stay zero
            const int k = tid - TR4, row = 16 * (t0 + x) + k / PAD8;
            if (row < N)
                __hip_atomic_store((gu64_t *)(img1 + row * P + 2 * N + 8 * (k % PAD8)), (uint64_t)0,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const float tss = block_sum_fixed(ss, red, tid);
        if (tid == 0) __hip_atomic_store(line + 3 + t0 + x, __float_as_uint(tss), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    MUON_TP(args);
    // hand-off 0: every storing wave drains, the barrier, one lane adds; one wave polls
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(line, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wave == 0) mc_wait(line, (uint32_t)np, line + 1, errors, args.spin_limit);
    __syncthreads();
    MUON_TP(args);
    // the NT tile-row sums: one relaxed load per thread < NT (not NT dependent loads in every thread),
    // summed in tile order from LDS
    static_assert(NT <= kMuonThreads / 64, "tile-row sums staged in red[]");
    if (tid < NT) red[tid] = __uint_as_float(__hip_atomic_load(line + 3 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    // the whole image in flight into registers, then normalised there on its way into LDS
    // (normalise_image's per-element arithmetic: no LDS round trip and barrier of its own)
    {
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(img1, (short)0, N * P, 0x00020000);
        constexpr int kCopy = (N * P / 16 + kMuonThreads - 1) / kMuonThreads;
        uint4 cv[kCopy];
#pragma unroll
        for (int u = 0; u < kCopy; u++)
            cv[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, (tid + u * kMuonThreads) * 16, 0, 16));
        __syncthreads();
        float total = 0.0f;
#pragma unroll
        for (int t = 0; t < NT; t++) total += red[t];
        const float nrm = fmaxf(round_bf(sqrtf(total)), args.eps);  // x.norm() of the bf16 X, clamped
#pragma unroll
        for (int u = 0; u < kCopy; u++) {
            const int o = (tid + u * kMuonThreads) * 16;
            if (o < N * P) *reinterpret_cast<uint4 *>(sX + o) = normalise16(cv[u], nrm);
        }
    }
    __syncthreads();
    MUON_TP(args);
    // the epilogue's learning rate in flight now, not after the last product
    const float lr_pre = args.lr[mt.lr_index];
    ns_square_mc<N>(sX, sG, args, mat, part, np, wave, lane, (uint32_t)np);
    // the last part through here puts the matrix's counters back to zero for the next launch (no
    // memset node per step): every other part has finished all its polls when it counts in.  Every
    // exchange-counter add of every part was OBSERVED complete before that part's done add: each
    // part's polling wave saw the counter reach np x (hand-offs so far), its own add included, and a
    // barrier separates that poll from the done add; the last part's poll (the last hand-off) came
    // before every done add likewise.  So the reset stores of the part whose done add comes last
    // (told by its returned value) follow every add and every poll with relaxed atomics alone.
    // Round 6: no agent release / acquire here any more -- the release wrote back the XCD's L2
    // (~1.7-6.5 us, MI355X_MICROARCH.md price list) on the last wave of every part.
    if (tid == kMuonThreads - 64) {
        gu32_t *done = line + 2;
        if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)(np - 1)) {
            __hip_atomic_store(line, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // decoupled weight decay + the match_rms_adamw-scaled update of this part's rows, bf16 copies
    // (the learning rate read before the products.  Round 5 also measured the parameter rows
    // prefetched there: the 8 registers they held through the products cost the first G product
    // ~3 k cycles more than the epilogue saved)
    const float step = lr_pre * (0.2f * sqrtf((float)N));
    muon_epilogue(mt.param, mt.pbf, sX, P, N, N, false, 1.0f - lr_pre * args.wd, step, tid, 16 * t0, 16 * (t0 + rb));
}

__global__ __launch_bounds__(1024) void lds_poison_kernel(uint32_t word) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint32_t *w = reinterpret_cast<uint32_t *>(smem);
    for (int i = threadIdx.x; i < kMuonLds / 4; i += 1024) w[i] = word;
    __syncthreads();
}

// One Newton-Schulz product of the generic (non-square) schedule on this wave's BI x BJ tile block:
// the 4 x 4 blocks of the original mapping (waves 4 x 4, 256 x 256), or blocks of one column of BI
// tiles numbered down the TI tile rows first
template <int BI, int BJ>
__device__ __forceinline__ void generic_phase(const char *A, int pa, bool a_rows, const char *B, int pb, char *out,
                                              int po, int M, int N, int K, float alpha, float beta, const char *zero,
                                              int wave, int lane, int TI) {
    int ti0, tj0;
    if constexpr (BI == kBI && BJ == kBJ) {
        ti0 = (wave & 3) * kBI;
        tj0 = (wave >> 2) * kBJ;
    } else {
        const int WI = (TI + BI - 1) / BI;
        ti0 = (wave % WI) * BI;
        tj0 = (wave / WI) * BJ;
    }
    f32x4_t acc[BI][BJ];
    init_block_t<BI, BJ>(acc, out, po, M, N, ti0, tj0, beta / alpha, beta != 0.0f, lane);
    gemm_block<BI, BJ>(acc, A, pa, a_rows, B, pb, M, N, K, ti0, tj0, zero, lane);
    __syncthreads();
    store_block_t<BI, BJ>(acc, out, po, M, N, ti0, tj0, alpha, lane);
    __syncthreads();
}

__global__ __launch_bounds__(kMuonThreads) void muon_kernel(MuonArgs args) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint8_t role = args.job_mat[blockIdx.x];
    if (role == kRoleIdle) return;
    if (role == kRoleAdam) {  // the 1-D parameters' AdamW, in the same launch
        adam_blocks(args, args.job_part[blockIdx.x], args.nadam);
        return;
    }
    const int mat = args.job_mat[blockIdx.x], part = args.job_part[blockIdx.x], np = args.job_nparts[blockIdx.x];
    MUON_CHECK(blockIdx.x < (unsigned)kMuonMaxJobs && mat < args.count && part < np, "job", mat, part * 256 + np);
    const MuonMat mt = args.m[mat];
    const int R = mt.rows, C = mt.cols;
    const bool tr = R > C;  // iterate on the wide orientation (r <= c), like torch
    const int r = tr ? C : R, c = tr ? R : C;
    const int px = muon_pitch(r, c), pg = muon_pitch(r, r);  // padded row pitches (bytes)
    char *sX = smem;
    char *sG = smem + ((r * px + 127) & ~127);
    char *zero = sG + ((r * pg + 127) & ~127);  // 64 zero bytes
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    MUON_TP(args);
    __shared__ float red[kMuonThreads / 64];
    __shared__ float s_norm;
    if (np > 1) {  // a part of a split square matrix (the host only splits h = 196 / 192)
        if (r == 196) mc_matrix<196>(smem, red, args, mt, mat, part, np, tid, wave, lane);
        else mc_matrix<192>(smem, red, args, mt, mat, part, np, tid, wave, lane);
        __syncthreads();
        MUON_TP(args);
        return;
    }
    // zero both images (their K padding must read as zero) and the zero block
    {
        const int bytes = (int)(zero - smem) + 64;
        for (int o = tid * 16; o < bytes; o += kMuonThreads * 16) *reinterpret_cast<uint4 *>(smem + o) = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();

    const float coef = block_clip_coef(args, tid, blockIdx.x == 0);
    MUON_TP(args);
    const bool sq196 = !tr && R == C && (R == 196 || R == 192);  // the multi-CU schedule's sum order
    float ss = 0.0f;
    if (sq196) {
        const float t = R == 196 ? tile_prologue<196>(mt.grad, mt.mom, sX, coef, args.momentum, args.nesterov != 0, red, tid)
                                 : tile_prologue<192>(mt.grad, mt.mom, sX, coef, args.momentum, args.nesterov != 0, red, tid);
        if (tid == 0) s_norm = fmaxf(round_bf(sqrtf(t)), args.eps);
    } else {
        ss = muon_prologue(mt.grad, mt.mom, sX, px, R, C, tr, coef, args.momentum, args.nesterov != 0, tid);
    }
    MUON_TP(args);
    if (!sq196) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
        if (lane == 0) red[wave] = ss;
        __syncthreads();
        if (tid == 0) {
            float t = 0.0f;
            for (int w = 0; w < kMuonThreads / 64; w++) t += red[w];
            s_norm = fmaxf(round_bf(sqrtf(t)), args.eps);  // x.norm() of a bf16 tensor, clamp(min=eps)
        }
    }
    __syncthreads();
    normalise_image(sX, r * px, s_norm, tid);
    __syncthreads();
    MUON_TP(args);

    // Newton-Schulz, three products per iteration, all through ONE gemm/store code path:
    //   0: G = X X^T                      (A = X rows, B^T = X rows; G symmetric)
    //   1: U = b G + c G G                (A = G rows, B^T = G rows; U symmetric)
    //   2: X^T = a X^T + X^T U            (A = X^T by the transposing read, B^T = U rows)
    // Every product stores its transpose (= G, U, and X itself for phase 2).
    const int kind = r == c && !args.generic_ns ? ns_square_kind(r) : 0;
    if (kind) {  // the square fast path (row pitch muon_pitch(n, n))
        switch (kind) {
        case 1: ns_square<196>(sX, sG, args, wave, lane); break;
        case 2: ns_square<192>(sX, sG, args, wave, lane); break;
        case 3: ns_square<128>(sX, sG, args, wave, lane); break;
        case 4: ns_square<64>(sX, sG, args, wave, lane); break;
        default: ns_square<32>(sX, sG, args, wave, lane); break;
        }
    } else {
    for (int ph = 0; ph < 3 * args.steps; ph++) {
        const int k = ph % 3;
        const char *A = k == 1 ? sG : sX;
        const int pa = k == 1 ? pg : px;
        const char *B = k == 0 ? sX : sG;
        const int pb = k == 0 ? px : pg;
        const int M = k == 2 ? c : r, N = r, K = k == 0 ? c : r;
        char *out = k == 2 ? sX : sG;
        const int po = k == 2 ? px : pg;
        const float alpha = k == 1 ? args.c : 1.0f;
        const float beta = k == 0 ? 0.0f : (k == 1 ? args.b : args.a);
        // round 6: the tiles of a small product spread over the 16 waves (one 16 x 16 tile per wave,
        // or a column of four) instead of one wave's 4 x 4 block -- the stem's 48 x 48 G and U ran on
        // ONE wave and made this block the launch's critical path (119 k cycles vs the 13-part
        // squares' 105-108 k, profiles/r06x/trace_muon_13.log).  Per tile the MFMA sequence (init,
        // k-steps in order, store) is unchanged: the same bits
        const int TI = (M + 15) >> 4, TJ = (N + 15) >> 4;
        if (TI * TJ <= kMuonWaves)
            generic_phase<1, 1>(A, pa, k != 2, B, pb, out, po, M, N, K, alpha, beta, zero, wave, lane, TI);
        else if (TJ <= 4 && ((TI + 3) >> 2) * TJ <= kMuonWaves)
            generic_phase<4, 1>(A, pa, k != 2, B, pb, out, po, M, N, K, alpha, beta, zero, wave, lane, TI);
        else
            generic_phase<kBI, kBJ>(A, pa, k != 2, B, pb, out, po, M, N, K, alpha, beta, zero, wave, lane, TI);
    }
    }

    // decoupled weight decay + the match_rms_adamw-scaled update, and the bf16 weight copy
    const float lr = args.lr[mt.lr_index];
    const float step = lr * (0.2f * sqrtf((float)(R > C ? R : C)));
    muon_epilogue(mt.param, mt.pbf, sX, px, R, C, tr, 1.0f - lr * args.wd, step, tid, 0, R, mt.frag, mt.frag_row);
    __syncthreads();
    MUON_TP(args);
}

__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a) {
    const float t = *a.step;
    const float bc1 = 1.0f - powf(a.b1, t);
    const float bc2s = sqrtf(1.0f - powf(a.b2, t));
    const float coef = a.clip ? *a.clip : 1.0f;
    for (int k = 0; k < a.count; k++) {
        const AdamGroup gr = a.g[k];
        const float lr = a.lr[gr.lr_index];
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < gr.n; i += (int64_t)gridDim.x * 256)
            adamw_elem(gr, i, lr, coef, a.b1, a.b2, a.eps, a.wd, bc1, bc2s);
    }
}

inline int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}

// CUs of the current device (cached per device)
inline int device_cus() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (!cached[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
        cached[dev] = n;
    }
    return cached[dev];
}

inline bool muon_splits(const g2048_muon_matrix &m, int parts) {
    return parts > 1 && m.rows == m.cols && (m.rows == 196 || m.rows == 192);
}

inline size_t muon_lds_bytes(int R, int C) {
    const int r = R > C ? C : R, c = R > C ? R : C;
    const int px = muon_pitch(r, c), pg = muon_pitch(r, r);
    return (size_t)((r * px + 127) & ~127) + (size_t)((r * pg + 127) & ~127) + 64;
}

}  // namespace

extern "C" {

int g2048_grad_clip(g2048_stream_t stream, const float *grad, int64_t n, float max_norm, float *norm_out,
                    float *coef_out, float *partials) {
    if (!grad || !norm_out || !coef_out || !partials || n <= 0 || ((uintptr_t)grad & 15u)) return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(grad_sumsq_kernel, dim3(kNormBlocks), dim3(256), 0, s, grad, n, partials);
    hipLaunchKernelGGL(grad_norm_kernel, dim3(1), dim3(kNormBlocks), 0, s, partials, max_norm, norm_out, coef_out);
    return status();
}

size_t g2048_muon_workspace_bytes(void) {
    return (size_t)kMuonSyncBytes + (size_t)kMuonMaxMats * 2 * max(196 * muon_pitch(196, 196), 192 * muon_pitch(192, 192)) +
           kMuonTraceBytes;
}

size_t g2048_muon_error_offset(void) { return (size_t)kMuonErrWord * sizeof(uint32_t); }

int g2048_lds_poison(g2048_stream_t stream, uint32_t word) {
    // 2 blocks per CU of the whole LDS each, every dword = word (tests: kernels must not read LDS
    // they did not write -- a NaN pattern left behind turns such a read into a NaN)
    hipLaunchKernelGGL(lds_poison_kernel, dim3(512), dim3(1024), kMuonLds, (hipStream_t)stream, word);
    return hipGetLastError() == hipSuccess ? G2048_OK : G2048_EINVAL;
}

int g2048_muon_supported(int32_t rows, int32_t cols) {
    if (rows <= 0 || cols <= 0) return 0;
    const int r = rows > cols ? cols : rows, c = rows > cols ? rows : cols;
    if (r > 16 * 4 * kBI || c > 16 * 4 * kBJ) return 0;
    return muon_lds_bytes(rows, cols) <= (size_t)kMuonLds ? 1 : 0;
}

int g2048_grad_sumsq(g2048_stream_t stream, const float *grad, int64_t n, float *partials) {
    if (!grad || !partials || n <= 0 || ((uintptr_t)grad & 15u)) return G2048_EINVAL;
    hipLaunchKernelGGL(grad_sumsq_kernel, dim3(kNormBlocks), dim3(256), 0, (hipStream_t)stream, grad, n, partials);
    return status();
}

static int muon_launch(g2048_stream_t stream, const g2048_muon_matrix *mats, int32_t count, const float *lr_dev,
                       const float *clip_coef_dev, const float *partials, float max_norm, float *norm_out,
                       float *coef_out, const g2048_muon_cfg *cfg, const AdamArgs *adam = nullptr);
static int adam_args(const g2048_adamw_group *groups, int32_t count, const float *lr_dev, const float *step_dev,
                     const float *clip_coef_dev, float beta1, float beta2, float eps, float weight_decay, AdamArgs &a,
                     int64_t &nmax);

int g2048_muon_step(g2048_stream_t stream, const g2048_muon_matrix *mats, int32_t count, const float *lr_dev,
                    const float *clip_coef_dev, const g2048_muon_cfg *cfg) {
    return muon_launch(stream, mats, count, lr_dev, clip_coef_dev, nullptr, 0.0f, nullptr, nullptr, cfg);
}

int g2048_muon_step_clip(g2048_stream_t stream, const g2048_muon_matrix *mats, int32_t count, const float *lr_dev,
                         const float *partials, float max_norm, float *norm_out, float *coef_out,
                         const g2048_muon_cfg *cfg) {
    if (!partials || !norm_out || !coef_out) return G2048_EINVAL;
    return muon_launch(stream, mats, count, lr_dev, nullptr, partials, max_norm, norm_out, coef_out, cfg);
}

int g2048_grad_sumsq_tick(g2048_stream_t stream, const float *grad, int64_t n, float *partials, float *step_dev) {
    if (!grad || !partials || !step_dev || n <= 0 || ((uintptr_t)grad & 15u)) return G2048_EINVAL;
    hipLaunchKernelGGL(grad_sumsq_kernel, dim3(kNormBlocks), dim3(256), 0, (hipStream_t)stream, grad, n, partials,
                       step_dev);
    return status();
}

int g2048_muon_adamw_step_clip(g2048_stream_t stream, const g2048_muon_matrix *mats, int32_t count,
                               const g2048_adamw_group *groups, int32_t ngroups, const float *lr_dev,
                               const float *step_dev, const float *partials, float max_norm, float *norm_out,
                               float *coef_out, const g2048_muon_cfg *cfg, float beta1, float beta2, float eps,
                               float adam_weight_decay) {
    if (!partials || !norm_out || !coef_out || ngroups < 0) return G2048_EINVAL;
    AdamArgs a{};
    int64_t nmax = 0;
    if (ngroups > 0) {
        const int st = adam_args(groups, ngroups, lr_dev, step_dev, nullptr, beta1, beta2, eps, adam_weight_decay, a, nmax);
        if (st) return st;
    }
    return muon_launch(stream, mats, count, lr_dev, nullptr, partials, max_norm, norm_out, coef_out, cfg,
                       ngroups > 0 ? &a : nullptr);
}

static int muon_launch(g2048_stream_t stream, const g2048_muon_matrix *mats, int32_t count, const float *lr_dev,
                       const float *clip_coef_dev, const float *partials, float max_norm, float *norm_out,
                       float *coef_out, const g2048_muon_cfg *cfg, const AdamArgs *adam) {
    if (!mats || count <= 0 || count > kMuonMaxMats || !lr_dev || !cfg) return G2048_EINVAL;
    MuonArgs a{};
    size_t lds = 0;
    for (int i = 0; i < count; i++) {
        const g2048_muon_matrix &m = mats[i];
        if (!m.param || !m.grad || !m.momentum || !g2048_muon_supported(m.rows, m.cols)) return G2048_EINVAL;
        if (((uintptr_t)m.param | (uintptr_t)m.grad | (uintptr_t)m.momentum) % 16 || (uintptr_t)m.param_bf16 % 8)
            return G2048_EINVAL;
        if (m.head_frag && (m.rows > m.cols || m.cols % 4 || m.frag_row < 0 || m.frag_row + m.rows > 5 || m.cols > 1024))
            return G2048_EINVAL;  // a head matrix: <= 5 rows of h columns, row-major epilogue
        a.m[i] = MuonMat{m.param, m.grad, m.momentum, m.param_bf16, (uint16_t *)m.head_frag, m.rows, m.cols, m.lr_index,
                         m.frag_row};
        const size_t b = muon_lds_bytes(m.rows, m.cols);
        lds = b > lds ? b : lds;
    }
    a.count = count;
    a.momentum = cfg->momentum;
    a.wd = cfg->weight_decay;
    a.a = cfg->ns_a;
    a.b = cfg->ns_b;
    a.c = cfg->ns_c;
    a.eps = cfg->ns_eps;
    a.steps = cfg->ns_steps;
    a.nesterov = cfg->nesterov;
    a.lr = lr_dev;
    a.clip = clip_coef_dev;
    a.partials = partials;
    a.npartials = cfg->npartials > 0 ? cfg->npartials : 64;
    if (a.npartials > G2048_COLSUM_SQ_MAX) return G2048_EINVAL;
    a.max_norm = max_norm;
    a.norm_out = norm_out;
    a.coef_out = coef_out;
    a.generic_ns = getenv("G2048_MUON_GENERIC") ? 1 : 0;
    // blocks: one per matrix, or cfg->parts (7 .. 13, at most one per 16-row tile row) per h = 196 /
    // 192 square matrix with a workspace.  Placement (speed only: the hand-off is agent-scope): the
    // parts of split matrix k sit on blocks k, k + 8, k + 16, ... -- one XCD under the round-robin
    // dispatch, so their exchange images are read from that XCD's L2; the other matrices and the
    // AdamW blocks fill the remaining slots in order, the rest of the grid idles.
    int parts = cfg->workspace && !a.generic_ns && !getenv("G2048_MUON_ONE_CU") ? cfg->parts : 1;
    if (parts > 1 && (parts < 7 || parts > 13)) return G2048_EINVAL;  // one or two tile rows per block
    const char *spin = getenv("G2048_MUON_SPIN_LIMIT");  // tests: force the timeout path
    a.spin_limit = spin ? (uint32_t)strtoul(spin, nullptr, 0) : (1u << 21);
    if (adam) {  // AdamW blocks: ~2 elements per thread, at most 8 blocks
        int64_t nmax = 0;
        for (int k = 0; k < adam->count; k++) nmax = adam->g[k].n > nmax ? adam->g[k].n : nmax;
        const int64_t nb = (nmax + 2 * kMuonThreads - 1) / (2 * kMuonThreads);
        a.nadam = (int)(nb < 1 ? 1 : (nb > 8 ? 8 : nb));
    }
    // the job table for `np_req` parts per split matrix; returns the grid size (-1: does not fit)
    auto place = [&](int np_req) {
        for (int b = 0; b < kMuonMaxJobs; b++) a.job_mat[b] = kRoleIdle;
        int nsplit = 0, grid = 0;
        for (int i = 0; i < count; i++) {  // split matrices first: their XCD columns
            const g2048_muon_matrix &m = mats[i];
            if (!muon_splits(m, np_req)) continue;
            const int nt = (m.rows + 15) / 16, np = np_req < nt ? np_req : nt;
            for (int p = 0; p < np; p++) {
                const int b = nsplit < 8 ? nsplit + 8 * p : -1;
                if (b < 0 || b >= kMuonMaxJobs) return -1;
                a.job_mat[b] = (uint8_t)i;
                a.job_part[b] = (uint8_t)p;
                a.job_nparts[b] = (uint8_t)np;
                grid = b + 1 > grid ? b + 1 : grid;
            }
            nsplit++;
        }
        int next = 0;
        auto free_slot = [&]() {
            while (next < kMuonMaxJobs && a.job_mat[next] != kRoleIdle) next++;
            return next < kMuonMaxJobs ? next++ : -1;
        };
        for (int i = 0; i < count; i++) {  // one-block matrices
            if (muon_splits(mats[i], np_req)) continue;
            const int b = free_slot();
            if (b < 0) return -1;
            a.job_mat[b] = (uint8_t)i;
            a.job_part[b] = 0;
            a.job_nparts[b] = 1;
            grid = b + 1 > grid ? b + 1 : grid;
        }
        for (int k = 0; k < (adam ? a.nadam : 0); k++) {
            const int b = free_slot();
            if (b < 0) return -1;
            a.job_mat[b] = kRoleAdam;
            a.job_part[b] = (uint8_t)k;
            grid = b + 1 > grid ? b + 1 : grid;
        }
        return grid;
    };
    int grid = place(parts);
    // the split parts poll each other, so every block of the grid must be resident at once (one per
    // CU: 1 024 threads, ~160 KB of LDS): a device with fewer CUs than the grid (a partitioned GPU, a
    // smaller part) runs every matrix on one CU instead
    if (parts > 1 && (grid < 0 || grid > device_cus())) {
        parts = 1;
        grid = place(1);
    }
    if (grid < 0) return G2048_EINVAL;
    a.njobs = grid;
    if (parts > 1) {  // the counters: zero from the caller's first fill, left zero by every launch
        char *ws = static_cast<char *>(cfg->workspace);
        a.sync = reinterpret_cast<uint32_t *>(ws);
        a.xg = ws + kMuonSyncBytes;
        a.xg_stride = 2 * (int64_t)max(196 * muon_pitch(196, 196), 192 * muon_pitch(192, 192));
    }
#ifdef MUON_TRACE
    if (cfg->workspace) {
        a.trace = reinterpret_cast<uint64_t *>(static_cast<char *>(cfg->workspace) + kMuonSyncBytes +
                                               (size_t)kMuonMaxMats * 2 * max(196 * muon_pitch(196, 196), 192 * muon_pitch(192, 192)));
        const hipError_t e = hipMemsetAsync(a.trace, 0, kMuonTraceBytes, (hipStream_t)stream);
        if (e != hipSuccess) return (int)e;
    }
#endif
    if (adam) a.adam = *adam;
    hipLaunchKernelGGL(muon_kernel, dim3(a.njobs), dim3(kMuonThreads), lds, (hipStream_t)stream, a);
    return status();
}

static int adam_args(const g2048_adamw_group *groups, int32_t count, const float *lr_dev, const float *step_dev,
                     const float *clip_coef_dev, float beta1, float beta2, float eps, float weight_decay, AdamArgs &a,
                     int64_t &nmax) {
    if (!groups || count <= 0 || count > kAdamMaxGroups || !lr_dev || !step_dev) return G2048_EINVAL;
    nmax = 0;
    for (int i = 0; i < count; i++) {
        const g2048_adamw_group &g = groups[i];
        if (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq || g.n < 0) return G2048_EINVAL;
        a.g[i] = AdamGroup{g.param, g.grad, g.exp_avg, g.exp_avg_sq, g.n, g.lr_index, 0};
        nmax = g.n > nmax ? g.n : nmax;
    }
    a.count = count;
    a.b1 = beta1;
    a.b2 = beta2;
    a.eps = eps;
    a.wd = weight_decay;
    a.lr = lr_dev;
    a.step = step_dev;
    a.clip = clip_coef_dev;
    return G2048_OK;
}

int g2048_adamw_step(g2048_stream_t stream, const g2048_adamw_group *groups, int32_t count, const float *lr_dev,
                     const float *step_dev, const float *clip_coef_dev, float beta1, float beta2, float eps,
                     float weight_decay) {
    AdamArgs a{};
    int64_t nmax = 0;
    const int st = adam_args(groups, count, lr_dev, step_dev, clip_coef_dev, beta1, beta2, eps, weight_decay, a, nmax);
    if (st) return st;
    int64_t blocks = (nmax + 255) / 256;
    blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
    hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
    return status();
}

}  // extern "C"
