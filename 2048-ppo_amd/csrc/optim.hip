// optim.hip -- the optimizer step of the PPO update (train.py:553-568: clip_grad_norm_(1.0),
// Muon for the 2-D weights, AdamW for the 1-D LayerNorm / bias parameters; torch.optim.Muon with
// adjust_lr_fn="match_rms_adamw", nesterov, 5 Newton-Schulz steps in bf16) as three launches:
//
//   grad_norm_kernel     ||g|| over the flat gradient bucket and the clip coefficient
//                        min(max_norm / (||g|| + 1e-6), 1) into device scalars
//   muon_kernel          one 256-thread block per weight matrix: momentum + nesterov, bf16 cast,
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

#include "../../include/g2048_ppo.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(uint32_t b) { return __uint_as_float(b << 16); }

__device__ __forceinline__ uint32_t f2bf(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7FFFFFFFu) > 0x7F800000u) return 0x7FC0u;
    u += 0x7FFFu + ((u >> 16) & 1u);
    return u >> 16;
}

__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

// ------------------------------------------------------------------ gradient norm ------------
constexpr int kNormThreads = 1024;

__global__ __launch_bounds__(kNormThreads) void grad_norm_kernel(const float *__restrict__ g, int64_t n, float max_norm,
                                                                 float *__restrict__ norm_out,
                                                                 float *__restrict__ coef_out) {
    __shared__ float red[kNormThreads / 64];
    float s = 0.0f;
    for (int64_t i = threadIdx.x; i < n; i += kNormThreads) s += g[i] * g[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.0f;
        for (int w = 0; w < kNormThreads / 64; w++) t += red[w];
        const float nrm = sqrtf(t);
        *norm_out = nrm;
        *coef_out = fminf(max_norm / (nrm + 1e-6f), 1.0f);
    }
}

// ------------------------------------------------------------------ Muon ---------------------
constexpr int kMuonThreads = 256;        // 4 waves (one per SIMD, 512 registers), 2 x 2 tile blocks
constexpr int kBI = 7, kBJ = 7;          // 16x16 tiles per wave: the block covers 224 x 224
constexpr int kMuonMaxMats = 8;
constexpr int kMuonLds = 160 * 1024 - 1024;

struct MuonMat {
    float *param;
    const float *grad;
    float *mom;
    uint16_t *pbf;
    int rows, cols, lr_index, pad;
};

struct MuonArgs {
    MuonMat m[kMuonMaxMats];
    int count;
    float momentum, wd, a, b, c, eps;
    int steps, nesterov;
    const float *lr;
    const float *clip;
};

// A-operand style fragment: 8 consecutive k of one row of a row-major bf16 LDS matrix (pitch in
// bytes); rows >= nrows and k >= K read as zero.
__device__ __forceinline__ bf16x8_t row_frag(const char *base, int pitch, int row, int nrows, int k0, int K) {
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (row < nrows) {
        const char *p = base + row * pitch + k0 * 2;
        const uint2 lo = *reinterpret_cast<const uint2 *>(p);
        const uint2 hi = *reinterpret_cast<const uint2 *>(p + 8);
        w = make_uint4(lo.x, lo.y, hi.x, hi.y);
        if (k0 + 8 > K) {  // K tail: zero the elements k >= K
            const int valid = K - k0;  // < 8, may be <= 0
            w.x = valid >= 2 ? w.x : (valid == 1 ? (w.x & 0xFFFFu) : 0u);
            w.y = valid >= 4 ? w.y : (valid == 3 ? (w.y & 0xFFFFu) : 0u);
            w.z = valid >= 6 ? w.z : (valid == 5 ? (w.z & 0xFFFFu) : 0u);
            w.w = valid == 7 ? (w.w & 0xFFFFu) : 0u;
        }
    }
    return __builtin_bit_cast(bf16x8_t, w);
}

// B-operand fragment of a row-major [K][N] bf16 LDS matrix via the transposing read: lane (g, i)
// gets B[k0 + 8g + j][n0 + i]; rows >= K come from a zero row.
__device__ __forceinline__ bf16x8_t col_frag(const char *base, int pitch, int k0, int K, int n0, const char *zero,
                                             int lane) {
    const int g = (lane >> 4) & 3, q = (lane >> 2) & 3, p = lane & 3;
    const int r1 = k0 + 8 * g + q, r2 = r1 + 4;
    const char *a1 = r1 < K ? base + r1 * pitch + (n0 + 4 * p) * 2 : zero;
    const char *a2 = r2 < K ? base + r2 * pitch + (n0 + 4 * p) * 2 : zero;
    const s16x4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)a1);
    const s16x4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)a2);
    return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(t1, t2, 0, 1, 2, 3, 4, 5, 6, 7));
}

// acc += A[M x K] B[K x N] over this wave's tile block.  A: rows of a row-major matrix.  B: either
// given by the rows of B^T (BT_ROWS, so B[k][n] = Bt[n][k]) or row-major (transposing read).
// The A fragments of a k-step stay in registers; B fragments are loaded one tile column at a time.
template <bool BT_ROWS>
__device__ __forceinline__ void gemm_block(f32x4_t (&acc)[kBI][kBJ], const char *A, int pa, const char *B, int pb,
                                        int M, int N, int K, int ti0, int tj0, const char *zero, int lane) {
    const int TI = (M + 15) >> 4, TJ = (N + 15) >> 4;
    const int ni = min(kBI, TI - ti0), nj = min(kBJ, TJ - tj0);  // wave-uniform
    if (ni <= 0 || nj <= 0) return;
    for (int k0 = 0; k0 < K; k0 += 32) {
        const int kl = k0 + 8 * (lane >> 4);
        bf16x8_t fa[kBI];
#pragma unroll
        for (int i = 0; i < kBI; i++)
            if (i < ni) fa[i] = row_frag(A, pa, 16 * (ti0 + i) + (lane & 15), M, kl, K);
#pragma unroll
        for (int j = 0; j < kBJ; j++) {
            if (j >= nj) break;
            const bf16x8_t fb = BT_ROWS ? row_frag(B, pb, 16 * (tj0 + j) + (lane & 15), N, kl, K)
                                        : col_frag(B, pb, k0, K, 16 * (tj0 + j), zero, lane);
#pragma unroll
            for (int i = 0; i < kBI; i++)
                if (i < ni) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc[i][j], 0, 0, 0);
        }
    }
}

__device__ __forceinline__ void zero_acc(f32x4_t (&acc)[kBI][kBJ]) {
#pragma unroll
    for (int i = 0; i < kBI; i++)
#pragma unroll
        for (int j = 0; j < kBJ; j++) acc[i][j] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
}

// out[row][col] (row-major bf16, pitch) = round_bf(alpha * acc + beta * prev[row][col]) for the
// tile block; prev may alias out (read here, by the same lane, before the write -- callers put a
// barrier between the GEMM's last operand read and this).
__device__ __forceinline__ void store_block(const f32x4_t (&acc)[kBI][kBJ], char *out, int pitch, int M, int N,
                                            int ti0, int tj0, float alpha, float beta, int lane) {
    const int TI = (M + 15) >> 4, TJ = (N + 15) >> 4;
#pragma unroll
    for (int i = 0; i < kBI; i++)
#pragma unroll
        for (int j = 0; j < kBJ; j++) {
            if (ti0 + i >= TI || tj0 + j >= TJ) continue;
            const int col = 16 * (tj0 + j) + (lane & 15);
            if (col >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = 16 * (ti0 + i) + 4 * (lane >> 4) + r;
                if (row >= M) continue;
                uint16_t *p = reinterpret_cast<uint16_t *>(out + row * pitch) + col;
                const float prev = beta != 0.0f ? bf2f(*p) : 0.0f;
                *p = (uint16_t)f2bf(alpha * acc[i][j][r] + beta * prev);
            }
        }
}

__global__ __launch_bounds__(kMuonThreads) void muon_kernel(MuonArgs args) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const MuonMat mt = args.m[blockIdx.x];
    const int R = mt.rows, C = mt.cols;
    const bool tr = R > C;  // iterate on the wide orientation (r <= c), like torch
    const int r = tr ? C : R, c = tr ? R : C;
    const int px = c * 2, pg = r * 2;  // row pitches (bytes), multiples of 8 since r, c % 4 == 0
    char *sX = smem;
    char *sG = smem + ((r * px + 127) & ~127);
    char *zero = sG + ((r * pg + 127) & ~127);  // 64 zero bytes (+ slack for tail reads)
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ti0 = (wave & 1) * kBI, tj0 = (wave >> 1) * kBJ;  // wave-uniform
    __shared__ float red[kMuonThreads / 64];
    __shared__ float s_norm;
    if (tid < 64) reinterpret_cast<uint32_t *>(zero)[tid] = 0u;

    // momentum + nesterov + bf16 cast (+ transpose) into sX; sum of squares of the bf16 values
    const float coef = args.clip ? *args.clip : 1.0f;
    const float mu = args.momentum;
    float ss = 0.0f;
    for (int e = tid; e < R * C; e += kMuonThreads) {
        const float g = mt.grad[e] * coef;
        float buf = mt.mom[e];
        buf = buf + (1.0f - mu) * (g - buf);                      // buf.lerp_(g, 1 - mu)
        mt.mom[e] = buf;
        const float u = args.nesterov ? buf - (buf - g) * (1.0f - mu) : buf;  // g.lerp(buf, mu)
        const float ub = round_bf(u);
        ss += ub * ub;
        const int i = e / C, j = e - i * C;
        const int xr = tr ? j : i, xc = tr ? i : j;
        reinterpret_cast<uint16_t *>(sX + xr * px)[xc] = (uint16_t)f2bf(ub);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    if (tid == 0) {
        float t = 0.0f;
        for (int w = 0; w < kMuonThreads / 64; w++) t += red[w];
        s_norm = fmaxf(round_bf(sqrtf(t)), args.eps);  // x.norm() of a bf16 tensor, clamp(min=eps)
    }
    __syncthreads();
    const float nrm = s_norm;
    for (int e = tid; e < r * c; e += kMuonThreads) {
        const int i = e / c, j = e - i * c;
        uint16_t *p = reinterpret_cast<uint16_t *>(sX + i * px) + j;
        *p = (uint16_t)f2bf(bf2f(*p) / nrm);
    }
    __syncthreads();

    f32x4_t acc[kBI][kBJ];
    for (int it = 0; it < args.steps; it++) {
        // G = X X^T
        zero_acc(acc);
        gemm_block<true>(acc, sX, px, sX, px, r, r, c, ti0, tj0, zero, lane);
        store_block(acc, sG, pg, r, r, ti0, tj0, 1.0f, 0.0f, lane);  // sG is free (last read before a barrier)
        __syncthreads();
        // U = b G + c G G   (G symmetric: G[k][n] = G[n][k], read by rows)
        zero_acc(acc);
        gemm_block<true>(acc, sG, pg, sG, pg, r, r, r, ti0, tj0, zero, lane);
        __syncthreads();
        store_block(acc, sG, pg, r, r, ti0, tj0, args.c, args.b, lane);
        __syncthreads();
        // X = a X + U X
        zero_acc(acc);
        gemm_block<false>(acc, sG, pg, sX, px, r, c, r, ti0, tj0, zero, lane);
        __syncthreads();
        store_block(acc, sX, px, r, c, ti0, tj0, 1.0f, args.a, lane);
        __syncthreads();
    }

    // decoupled weight decay + the match_rms_adamw-scaled update, and the bf16 weight copy
    const float lr = args.lr[mt.lr_index];
    const float step = lr * (0.2f * sqrtf((float)(R > C ? R : C)));
    const float decay = 1.0f - lr * args.wd;
    for (int e = tid; e < R * C; e += kMuonThreads) {
        const int i = e / C, j = e - i * C;
        const int xr = tr ? j : i, xc = tr ? i : j;
        const float x = bf2f(reinterpret_cast<const uint16_t *>(sX + xr * px)[xc]);
        const float p = mt.param[e] * decay - x * step;
        mt.param[e] = p;
        if (mt.pbf) mt.pbf[e] = (uint16_t)f2bf(p);
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

__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a) {
    const float t = *a.step;
    const float bc1 = 1.0f - powf(a.b1, t);
    const float bc2s = sqrtf(1.0f - powf(a.b2, t));
    const float coef = a.clip ? *a.clip : 1.0f;
    for (int k = 0; k < a.count; k++) {
        const AdamGroup gr = a.g[k];
        const float lr = a.lr[gr.lr_index];
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < gr.n; i += (int64_t)gridDim.x * 256) {
            const float g = gr.grad[i] * coef;
            float p = gr.param[i] * (1.0f - lr * a.wd);
            const float m = gr.m[i] + (1.0f - a.b1) * (g - gr.m[i]);
            const float v = gr.v[i] * a.b2 + (1.0f - a.b2) * g * g;
            gr.m[i] = m;
            gr.v[i] = v;
            p -= (lr / bc1) * m / (sqrtf(v) / bc2s + a.eps);
            gr.param[i] = p;
        }
    }
}

inline int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}

inline size_t muon_lds_bytes(int R, int C) {
    const int r = R > C ? C : R, c = R > C ? R : C;
    return (size_t)((r * c * 2 + 127) & ~127) + (size_t)((r * r * 2 + 127) & ~127) + 1024;
}

}  // namespace

extern "C" {

int g2048_grad_clip(g2048_stream_t stream, const float *grad, int64_t n, float max_norm, float *norm_out,
                    float *coef_out) {
    if (!grad || !norm_out || !coef_out || n <= 0) return G2048_EINVAL;
    hipLaunchKernelGGL(grad_norm_kernel, dim3(1), dim3(kNormThreads), 0, (hipStream_t)stream, grad, n, max_norm,
                       norm_out, coef_out);
    return status();
}

int g2048_muon_supported(int32_t rows, int32_t cols) {
    if (rows <= 0 || cols <= 0) return 0;
    const int r = rows > cols ? cols : rows, c = rows > cols ? rows : cols;
    if (c % 4 || (r % 4 && r != 1)) return 0;  // 8-byte LDS row pitches (a single row needs none)
    if (r > 16 * 2 * kBI || c > 16 * 2 * kBJ) return 0;
    return muon_lds_bytes(rows, cols) <= (size_t)kMuonLds ? 1 : 0;
}

int g2048_muon_step(g2048_stream_t stream, const g2048_muon_matrix *mats, int32_t count, const float *lr_dev,
                    const float *clip_coef_dev, const g2048_muon_cfg *cfg) {
    if (!mats || count <= 0 || count > kMuonMaxMats || !lr_dev || !cfg) return G2048_EINVAL;
    MuonArgs a{};
    size_t lds = 0;
    for (int i = 0; i < count; i++) {
        const g2048_muon_matrix &m = mats[i];
        if (!m.param || !m.grad || !m.momentum || !g2048_muon_supported(m.rows, m.cols)) return G2048_EINVAL;
        a.m[i] = MuonMat{m.param, m.grad, m.momentum, m.param_bf16, m.rows, m.cols, m.lr_index, 0};
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
    hipLaunchKernelGGL(muon_kernel, dim3(count), dim3(kMuonThreads), lds, (hipStream_t)stream, a);
    return status();
}

int g2048_adamw_step(g2048_stream_t stream, const g2048_adamw_group *groups, int32_t count, const float *lr_dev,
                     const float *step_dev, const float *clip_coef_dev, float beta1, float beta2, float eps,
                     float weight_decay) {
    if (!groups || count <= 0 || count > kAdamMaxGroups || !lr_dev || !step_dev) return G2048_EINVAL;
    AdamArgs a{};
    int64_t nmax = 0;
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
    int64_t blocks = (nmax + 255) / 256;
    blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
    hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
    return status();
}

}  // extern "C"
