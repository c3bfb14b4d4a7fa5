// ppo_fused.hip -- the PPO minibatch's forward passes of GameMLP (model_optimize_step,
// train.py:414-642; GameMLP.forward, game.py:1145-1220) as ONE persistent launch each:
//
//   train pass   boards[idx] -> to_model_format (game.py:92-101) -> stem Linear + LayerNorm + ReLU
//                -> 2 x ResidualBlock with nn.Dropout (train mode) -> action / value heads
//                -> masked log-softmax, PPO-clip ratio, clamped-logit entropy, smooth-L1 value loss
//                   and their gradient dz = dloss / d(logits, value)            (train.py:491-546)
//   KL pass      the same forward with the updated weights and the second dropout draw -> the
//                action head -> KL(old || new) per row, summed / maxed           (train.py:578-601)
//
// replacing g2048_obs_gather + three g2048_mlp_fwd + g2048_ppo_head_loss (train pass) and two
// g2048_mlp_fwd + g2048_mlp_fwd_kl (KL pass).  The layers run on the register hand-off of the fused
// rollout (mlp_tile.hpp): a wave owns 64 minibatch rows = 4 MFMA board tiles, the two h x h block
// weights sit in LDS, the stem weights and heads come from L1/L2, each layer's output becomes the
// next layer's B fragment by permlane swaps.  Every layer's epilogue is g2048_mlp_fwd's arithmetic
// (same MFMA k order from zero, ln_row.hpp, the same dropout keep masks), so the activations, G and
// the LayerNorm statistics are bitwise those of the per-layer kernels (tests/test_gpu_ppo_fused.py).
//
// Heads: one MFMA chain per board tile whose 16-row A operand is the fp32 head matrix [wa; wv]
// split exactly into three bf16 terms (rows 0-4 hi, 5-9 mid, 10-14 lo: all 24 mantissa bits, so
// the logits keep the fp32 weights as g2048_ppo_head_loss does); two permlane swap stages turn the
// four tiles' accumulators into "lane = row" (lane 16 q + c holds all 16 head rows of row 16 q + c
// of its 64), where the per-row loss / KL runs once per row.
//
// The train pass writes what the backward needs: x0 (bf16 obs, the stem weight-gradient operand),
// per layer G (bf16, pre-norm), H (bf16 output) and mean / rstd, masked logits (for the KL), dz as
// fp32 [m][8] (the blocks' output gradient source) and as two bf16 terms [m][16] (hi in columns
// 0-4, lo = bf16(dz - hi) in 8-12: the head weight gradient dz^T H2 runs on g2048_wgrad with fp32
// accuracy in dz, summing the hi and lo halves of its partial rows), and per block
// partials [dba 4 | dbv | sum ppo, sum H, sum v] summed by the deferred column sum.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "board.hpp"
#include "ln_row.hpp"
#include "mlp_tile.hpp"
#include "ppo_common.hpp"
#include "../../include/g2048_ppo.h"

using namespace g2048::tile;
namespace P = g2048::ppo;

static_assert(sizeof(g2048_mlp_pass_args) == 424 && offsetof(g2048_mlp_pass_args, drop) == 176 &&
                  offsetof(g2048_mlp_pass_args, partials) == 400 && offsetof(g2048_mlp_pass_args, keep) == 408 &&
                  offsetof(g2048_mlp_pass_args, idx_offset) == 416,
              "g2048_mlp_pass_args layout (tests/test_abi.py)");
static_assert(sizeof(g2048_ppo_stats_args) == 88 && offsetof(g2048_ppo_stats_args, idx_offset) == 72,
              "g2048_ppo_stats_args layout (tests/test_abi.py)");
static_assert(sizeof(g2048_mlp_back_args) == 312 && offsetof(g2048_mlp_back_args, keep) == 304,
              "g2048_mlp_back_args layout (tests/test_abi.py)");

namespace {

#ifndef FP_WAVES
#define FP_WAVES 8
#endif
#ifndef FP_KSB
#define FP_KSB 1
#endif
#ifndef FP_LUNROLL
#define FP_LUNROLL 0
#endif
constexpr int kFpThreads = 64 * FP_WAVES;  // 8 waves = 2 per SIMD sharing the one LDS weight image (one block per CU)
constexpr int kFpLdsMax = 163840;
constexpr int kFpRows = FP_WAVES == 8 ? 32 : 64;  // rows per wave iteration (the loss runs "lane = row")
constexpr int kFpTiles = kFpRows / 16;
#ifndef FP_Q
#define FP_Q (FP_WAVES == 8 ? 1 : 2)
#endif
constexpr int kFpQ = FP_Q;          // board tiles per MLP pass (accumulators of kFpQ x NT tiles: 256 registers per wave)
constexpr int kFpBlockRows = kFpThreads / 64 * kFpRows;
constexpr int kTrainParts = 8;   // partial floats per block: dba[4], dbv, sum ppo, sum H, sum v

struct FpArgs {
    const int8_t *boards;
    int64_t m;
    P::HeadLossArgs la;            // idx, action, legal, old_logp, adv, ret, beta_dev, rows, critic, clip, inv_m, decouple
    const uint16_t *w0, *w1, *w2;  // bf16 stem [h][48], blocks [h][h]
    const float *gamma[kMaxLayers], *beta[kMaxLayers];
    const float *ba, *bv;
    const uint4 *head;             // head_split_kernel's fragments [KS][64]
    P::DropArgs drop[2];           // blocks 1, 2
    uint16_t *x0;                  // train: bf16 [m][48] (nullable)
    uint16_t *g[kMaxLayers];       // train: bf16 [m][h] (nullable each)
    uint16_t *h[kMaxLayers];       // train: bf16 [m][h] (nullable each)
    float *mean[kMaxLayers], *rstd[kMaxLayers];
    float *masked;                 // train: [m][4] out; KL: the stored old masked logits (in)
    float *dz;                     // train: fp32 [m][8]
    uint16_t *dzb;                 // train: bf16 [m][16]: hi(dz) 0..4, lo(dz) 8..12
    float *part;                   // per block: train kTrainParts floats, KL {sum, max}
    uint2 *keep;                   // train, optional: the blocks' keep bits [block][m][lane group]
    P::StatsArgs st;               // KL, optional (st.stats): the last block folds g2048_ppo_stats in
    const int64_t *idx_off;        // optional: rows batch.idx[*idx_off + r]
};

// The head matrix [wa (4 rows); wv] as three exact bf16 terms in the 16 rows of the head chain's A
// operand, laid out in fragment order: frag[ks][lane] (uint4) holds row c = lane & 15, k = 32 ks +
// 8 (lane >> 4) .. + 7 (zero past h and in row 15), so a lane reads its fragment as one coalesced
// 16-byte load.  Rows 0-4 hi (wa 0..3, wv), 5-9 mid, 10-14 lo: hi + mid + lo = the fp32 weight.
__global__ __launch_bounds__(256) void head_split_kernel(const float *__restrict__ wa, const float *__restrict__ wv,
                                                         int h, int ks_n, uint4 *__restrict__ frag) {
    const int e = blockIdx.x * 256 + threadIdx.x;  // (ks, lane)
    if (e >= ks_n * 64) return;
    const int ks = e >> 6, lane = e & 63, g = lane >> 4, c = lane & 15;
    const int term = c < 5 ? 0 : c < 10 ? 1 : c < 15 ? 2 : 3, which = c - 5 * term;  // which: 0-3 wa row, 4 wv
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        uint32_t pr = 0;
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int k = 32 * ks + 8 * g + j + u;
            const float x = (term < 3 && k < h) ? (which < 4 ? wa[which * h + k] : (wv ? wv[k] : 0.0f)) : 0.0f;
            const __bf16 hi = (__bf16)x;
            const float r1 = x - (float)hi;
            const __bf16 mid = (__bf16)r1;
            const __bf16 lo = (__bf16)(r1 - (float)mid);
            const __bf16 t = term == 0 ? hi : term == 1 ? mid : lo;
            pr |= (uint32_t)__builtin_bit_cast(uint16_t, t) << (16 * u);
        }
        w[j / 2] = pr;
    }
    frag[e] = make_uint4(w[0], w[1], w[2], w[3]);
}

// The four board tiles' head accumulators (lane (g, c) of tile q: head rows 4 g .. 4 g + 3 of row
// 16 q + c) -> lane (q, c): R[g'] = head rows 4 g' .. 4 g' + 3 of its own row 16 q + c.
__device__ __forceinline__ void heads_to_rows(f32x4_t (&R)[4]) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(R[0][i]), __float_as_uint(R[2][i]), false, false);
        const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(R[1][i]), __float_as_uint(R[3][i]), false, false);
        const auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
        const auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
        R[0][i] = __uint_as_float(c[0]);
        R[1][i] = __uint_as_float(c[1]);
        R[2][i] = __uint_as_float(d[0]);
        R[3][i] = __uint_as_float(d[1]);
    }
}

// 8-byte feature groups of one layer output tile row: lane (g, c) stores its valid groups of the
// row at byte offset `off` (row * 2 H, < 2^32: a uniform base + 32-bit lane offset per store)
template <int NT, int H>
__device__ __forceinline__ void store_tile(uint16_t *dst, uint32_t off, const uint2 (&v)[NT], int g) {
    char *p = reinterpret_cast<char *>(dst) + (off + 8u * (uint32_t)g);
#pragma unroll
    for (int n = 0; n < NT; n++)
        if (16 * n + 4 * g < H) *reinterpret_cast<uint2 *>(p + 32 * n) = v[n];
}

template <int H, bool TRAIN, bool DROP>
__global__ __launch_bounds__(kFpThreads) void mlp_pass_kernel(FpArgs a) {
    constexpr int NT = (H + 15) / 16, KS = ((H + 7) / 8 * 8 + 31) / 32;
    constexpr int h = H;
    constexpr int PW = pr_pitch(h), WB = pr_wbytes(h);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *sLN = reinterpret_cast<float *>(smem + 2 * WB);  // [layer][gamma | beta][16 NT]
    char *sZero = smem + 2 * WB + 2 * kMaxLayers * pr_ln_floats(NT) * 4;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, col = lane & 15;
    const int64_t m = a.m;
    const int64_t mv = a.la.rows ? min(*a.la.rows, m) : m;  // rows >= mv: padding of a ragged minibatch
    const int64_t *idxp = a.la.idx + (a.idx_off ? *a.idx_off : 0);  // this minibatch's rows
    const float inv_m = a.la.rows ? 1.0f / (float)max(mv, (int64_t)1) : a.la.inv_m;

    // ---- the block weight images (bank-spread rows, zero K padding): 16 8-byte loads in flight per
    // thread per batch; LayerNorm affines; the zero fragment
    {
        constexpr int q8 = PW / 8, h4 = h / 4, per = h * q8;
        const uint16_t *wsrc[2] = {a.w1, a.w2};
#pragma unroll
        for (int l = 0; l < 2; l++)
            for (int c0 = 0; c0 < per; c0 += 16 * kFpThreads) {
                uint2 v[16];
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const int c = c0 + tid + u * kFpThreads, r = c / q8, q = c - r * q8;
                    v[u] = (c < per && q < h4) ? *reinterpret_cast<const uint2 *>(wsrc[l] + (int64_t)r * h + 4 * q)
                                               : make_uint2(0u, 0u);
                }
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const int c = c0 + tid + u * kFpThreads, r = c / q8, q = c - r * q8;
                    if (c < per) *reinterpret_cast<uint2 *>(smem + l * WB + pr_piece(h, r, q)) = v[u];
                }
            }
        for (int e = tid; e < kMaxLayers * 2 * 16 * NT; e += kFpThreads) {
            const int l = e / (32 * NT), rem = e - l * 32 * NT, which = rem / (16 * NT), f = rem - which * 16 * NT;
            const float *src = which ? a.beta[l] : a.gamma[l];
            sLN[e] = f < h ? src[f] : 0.0f;
        }
        if (tid < 4) reinterpret_cast<uint32_t *>(sZero)[tid] = 0u;
    }
    __syncthreads();

    constexpr float inv_n = 1.0f / (float)h;
    constexpr int hp8 = (h + 7) & ~7;
    constexpr int last_rows = h - 16 * (NT - 1);
    const StemRecipe sr = stem_recipe(g);
    const P::Drop d1 = P::make_drop(a.drop[0]), d2 = P::make_drop(a.drop[1]);
    const int wlane = col * PW + 16 * g, wlane_x = col * PW + 16 * (g ^ pr_swz(h, col));  // plain / swizzled k groups
    const int zoff = (int)(sZero - smem);
    const float bias[5] = {a.ba[0], a.ba[1], a.ba[2], a.ba[3], TRAIN ? a.bv[0] : 0.0f};
    const float beta_c = TRAIN ? *a.la.beta_dev : 0.0f;
    // per lane: TRAIN dba[4], dbv, sum ppo, sum H, sum v;  KL sum, max
    float acc_s[kTrainParts] = {0, 0, 0, 0, 0, 0, 0, 0};
    float kmax = -INFINITY;

    for (int64_t base = (int64_t)blockIdx.x * kFpBlockRows; base < m; base += (int64_t)gridDim.x * kFpBlockRows) {
        const int64_t r0 = base + kFpRows * wave;
        if (r0 >= m) continue;  // an empty wave (no barrier below)
        const int64_t r = r0 + lane;  // this lane's row for the loss / KL ("lane = row")
        const bool live = lane < kFpRows && r < m, real = live && r < mv;
        const uint4 b = live ? *reinterpret_cast<const uint4 *>(a.boards + idxp[r] * 16) : make_uint4(0u, 0u, 0u, 0u);

        int wlane_t = wlane, wlane_xt = wlane_x, glane_t = (col * 48 + 8 * g) * 2;
        asm volatile("" : "+v"(wlane_t), "+v"(wlane_xt), "+v"(glane_t));
        // the LayerNorm affines are re-read from LDS per layer: an opaque base keeps the compiler
        // from hoisting all 3 x 2 x NT float4 of them out of the row loop (registers: 2 waves per SIMD)
        int lnoff = 0;
        asm volatile("" : "+v"(lnoff));
        const float *sLNr = sLN + lnoff;
        // the stem weight fragments through a buffer descriptor: per-lane 32-bit offset + a constant
        // SGPR offset per (n, ks) -- no 64-bit address register pair per fragment.  Rows past h read
        // out of range (zero); k past 48 (ks 1, lane groups 2, 3) is sent out of range too.
        const __amdgpu_buffer_rsrc_t w0r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(a.w0), 0, h * 96, 0x00020000);
        const int w0off[2] = {glane_t, g < 2 ? glane_t + 64 : h * 96};
        f32x4_t accH[4];
#pragma unroll
        for (int t = kFpTiles; t < 4; t++) accH[t] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 1
        for (int pr = 0; pr < kFpTiles / kFpQ; pr++) {
            uint2 act[kFpQ][NT];
            // ---------------- stem: obs fragments from the board bytes ----------------------
            uint4 xs[kFpQ][2];
#pragma unroll
            for (int q = 0; q < kFpQ; q++) {
                const int s = 16 * (kFpQ * pr + q) + col;
                const uint32_t B0 = __shfl(b.x, s), B1 = __shfl(b.y, s), B2 = __shfl(b.z, s), B3 = __shfl(b.w, s);
#pragma unroll
                for (int ks = 0; ks < 2; ks++) xs[q][ks] = stem_frag(sr, ks, B0, B1, B2, B3);
                if (TRAIN && a.x0) {
                    const uint32_t row = (uint32_t)(r0 + s);
                    if ((int64_t)row < m) {
                        char *xo = reinterpret_cast<char *>(a.x0) + (row * 96u + 16u * (uint32_t)g);
                        *reinterpret_cast<uint4 *>(xo) = xs[q][0];
                        if (g < 2) *reinterpret_cast<uint4 *>(xo + 64) = xs[q][1];
                    }
                }
            }
            f32x4_t acc[kFpQ][NT];
            uint32_t kb[kFpQ][2] = {};  // the next block's dropout keep bits, drawn between its MFMAs
#pragma unroll
            for (int q = 0; q < kFpQ; q++)
#pragma unroll
                for (int n = 0; n < NT; n++) acc[q][n] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int ks = 0; ks < 2; ks++) {
#pragma unroll
                for (int n = 0; n < NT; n++) {
                    const uint4 fw = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w0r, w0off[ks], 2 * 16 * n * 48, 0));
#pragma unroll
                    for (int q = 0; q < kFpQ; q++)
                        acc[q][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(fw), as_frag(xs[q][ks]), acc[q][n], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            // ---------------- epilogue of layer l, tile q (row of lane (g, col) = r0 + 16 tq + col)
#define FP_EPILOGUE(L_, Q_, RES_, DROP_)                                                                           \
    do {                                                                                                        \
        const uint32_t row = (uint32_t)(r0 + 16 * (kFpQ * pr + (Q_)) + col);                                     \
        const float *lnp = sLNr + (L_) * 32 * NT;                                                               \
        const bool st = TRAIN && (int64_t)row < m;                                                              \
        float mean, rstd;                                                                                       \
        ln_epilogue_train_kb<NT, H, RES_, DROP_>(acc[Q_], act[Q_], lnp, lnp + 16 * NT, g, inv_n, d1.scale, kb[Q_],   \
                                                 st ? a.g[L_] : nullptr, row * (2u * H), mean, rstd);            \
        if (st) {                                                                                               \
            if (a.h[L_]) store_row16<NT, H>(reinterpret_cast<char *>(a.h[L_]) + row * (2u * H), act[Q_], g);     \
            if (g == 0 && a.mean[L_]) {                                                                         \
                a.mean[L_][row] = mean;                                                                         \
                a.rstd[L_][row] = rstd;                                                                         \
            }                                                                                                   \
        }                                                                                                       \
    } while (0)
#pragma unroll
            for (int q = 0; q < kFpQ; q++) FP_EPILOGUE(0, q, false, false);

            // ---------------- residual blocks (one copy of the code for both: instruction cache) ----
#if FP_LUNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
            for (int l = 0; l < 2; l++) {
#pragma unroll
                for (int q = 0; q < kFpQ; q++)
#pragma unroll
                    for (int n = 0; n < NT; n++) acc[q][n] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
                const int wbase = l * WB + wlane_t, wbase_x = l * WB + wlane_xt;
#pragma unroll
                for (int ks = 0; ks < KS; ks++) {
                    uint4 bf[kFpQ];
#pragma unroll
                    for (int q = 0; q < kFpQ; q++) bf[q] = act_frag<NT>(act[q], ks);
                    const bool kok = 32 * ks + 8 * g < hp8;
                    int kbase = (pr_ks_swz(h, ks) ? wbase_x : wbase) + 64 * ks;
                    asm volatile("" : "+v"(kbase));
                    // keep bits of feature tiles 2 ks, 2 ks + 1 (column groups 8 ks + g, + 4) of this
                    // block's dropout: VALU work beside the k-step's MFMAs instead of in the epilogue
                    if (DROP && 2 * ks < NT)
#pragma unroll
                        for (int q = 0; q < kFpQ; q++) {
                            const uint32_t row = (uint32_t)(r0 + 16 * (kFpQ * pr + q) + col);
                            kb[q][ks >> 2] |= P::drop_keep8(l ? d2 : d1, row, (uint32_t)(8 * ks + g)) << (8 * (ks & 3));
                        }
#pragma unroll
                    for (int n = 0; n < NT; n++) {
                        const bool rok = n < NT - 1 || col < last_rows;
                        const int off = (kok && rok) ? kbase + 16 * n * PW : zoff;
                        const uint4 fw = *reinterpret_cast<const uint4 *>(smem + off);
#pragma unroll
                        for (int q = 0; q < kFpQ; q++)
                            acc[q][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(fw), as_frag(bf[q]), acc[q][n], 0, 0, 0);
                    }
                    if (FP_KSB) __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int q = 0; q < kFpQ; q++) {
                    FP_EPILOGUE(l + 1, q, true, DROP);
                    if (TRAIN && DROP && a.keep) {  // for the backward: bit 4 n + e = feature 16 n + 4 g + e
                        const int64_t row = r0 + 16 * (kFpQ * pr + q) + col;
                        if (row < m) a.keep[((int64_t)l * m + row) * 4 + g] = make_uint2(kb[q][0], kb[q][1]);
                    }
                    kb[q][0] = kb[q][1] = 0u;
                }
            }
            // ---------------- heads: tile q's 16-row chain ----------------------------------------
#pragma unroll
            for (int q = 0; q < kFpQ; q++) {
                f32x4_t z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int ks = 0; ks < KS; ks++)
                    z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a.head[64 * ks + lane]), as_frag(act_frag<NT>(act[q], ks)),
                                                                z, 0, 0, 0);
                accH[kFpQ * pr + q] = z;
            }
        }
#undef FP_EPILOGUE
        // ---------------- lane = row: logits (hi + mid + lo), value; loss / KL -------------------
        // the row's loss inputs (KL: its stored old logits), loaded only now: they would otherwise
        // hold registers across the whole MLP
        P::RowIn in{};
        float4 old4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (TRAIN && real) in = P::load_row_in(a.la, idxp[r]);
        if (!TRAIN && real) old4 = *reinterpret_cast<const float4 *>(a.masked + r * 4);
        heads_to_rows(accH);
        float z5[5];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const int hi = k, mid = 5 + k, lo = 10 + k;
            z5[k] = (accH[hi >> 2][hi & 3] + accH[mid >> 2][mid & 3]) + accH[lo >> 2][lo & 3] + bias[k];
        }
        if (TRAIN) {
            float dz[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
            if (real) {
                float mk[4], ppo, ent, vl;
                P::HeadLossArgs la = a.la;
                la.inv_m = inv_m;
                P::row_loss(z5, in, la, beta_c, dz, mk, ppo, ent, vl);
                *reinterpret_cast<float4 *>(a.masked + r * 4) = make_float4(mk[0], mk[1], mk[2], mk[3]);
                acc_s[5] += ppo;
                acc_s[6] += ent;
                acc_s[7] += vl;
            }
#pragma unroll
            for (int k = 0; k < 5; k++) acc_s[k] += dz[k];
            if (live) {
                *reinterpret_cast<float4 *>(a.dz + r * 8) = make_float4(dz[0], dz[1], dz[2], dz[3]);
                *reinterpret_cast<float4 *>(a.dz + r * 8 + 4) = make_float4(dz[4], 0.0f, 0.0f, 0.0f);
                // dz as two bf16 terms (hi, lo = bf16(dz - hi)): the head weight gradient
                // dz^T H2 = hi^T H2 + lo^T H2 keeps ~16 mantissa bits of dz (g2048_ppo_head_loss's
                // fp32 dz x bf16 H2) on the bf16 weight-gradient kernel
                float lo[5];
                uint32_t hb[3];
#pragma unroll
                for (int k = 0; k < 5; k++) lo[k] = dz[k] - bf_lo(pack_bf2(dz[k], 0.0f));
                hb[0] = pack_bf2(dz[0], dz[1]);
                hb[1] = pack_bf2(dz[2], dz[3]);
                hb[2] = pack_bf2(dz[4], 0.0f);
                uint4 *zb = reinterpret_cast<uint4 *>(a.dzb + r * 16);
                zb[0] = make_uint4(hb[0], hb[1], hb[2], 0u);
                zb[1] = make_uint4(pack_bf2(lo[0], lo[1]), pack_bf2(lo[2], lo[3]), pack_bf2(lo[4], 0.0f), 0u);
            }
        } else if (real) {
            const float o[4] = {old4.x, old4.y, old4.z, old4.w};
            const float kl = P::kl_row(o, z5);
            acc_s[0] += kl;
            kmax = fmaxf(kmax, kl);
        }
    }
    // ---- per block: fixed-order wave sums (LDS after the last use of the images) ------------
    constexpr int NP = TRAIN ? kTrainParts : 2;
    float vals[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) {
        float v = TRAIN || k == 0 ? acc_s[k] : kmax;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float w = __shfl_xor(v, o);
            v = (!TRAIN && k == 1) ? fmaxf(v, w) : v + w;
        }
        vals[k] = v;
    }
    __syncthreads();
    float *red = reinterpret_cast<float *>(smem);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NP; k++) red[wave * NP + k] = vals[k];
    __syncthreads();
    const bool fold = !TRAIN && a.st.stats;  // the KL pass with the minibatch statistics folded in
    if (tid < NP) {
        float t = red[tid];
        for (int w = 1; w < kFpThreads / 64; w++) t = (!TRAIN && tid == 1) ? fmaxf(t, red[w * NP + tid]) : t + red[w * NP + tid];
        float *dst = a.part + (int64_t)blockIdx.x * NP + tid;
        if (fold) __hip_atomic_store(dst, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1: the hand-off below
        else *dst = t;
    }
    if (fold) {
        // the last block to finish reduces every block's {sum, max} and accumulates the minibatch
        // statistics (g2048_ppo_stats folded in).  The hand-off is MI355X_MICROARCH.md's table row 1
        // (one workgroup per CU here): partials stored sc1, every wave drains, a barrier, ONE lane's
        // relaxed agent-scope ticket add; the block whose add came last (told by its returned value)
        // reads the partials with sc1 loads behind a barrier (stats_block) and puts the ticket back to
        // zero.  Round 6: no agent release / acquire fence any more -- the release wrote back the XCD's
        // L2 in every one of the 256 blocks and the acquire invalidated L1 (~1.7 us each per the guide)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int *flag = reinterpret_cast<int *>(smem + 4096);
        if (tid == 0) {
            const uint32_t k = __hip_atomic_fetch_add((__attribute__((address_space(1))) uint32_t *)a.st.sync, 1u,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag = k == gridDim.x - 1u;
        }
        __syncthreads();
        if (!*flag) return;
        P::stats_block(a.st, a.part, (int)gridDim.x, smem, tid);
    }
}

// ------------------------------------------------------------------ fused backward ----------
// The minibatch's backward through the MLP in one persistent launch: for each 16-row tile the
// three LayerNorm backwards (top block first) and the two block input gradients, with every
// intermediate in registers:
//     dy2 = dz W_heads                                   (v_mfma_f32_16x16x4_f32, as ln_bwd196)
//     dG2 = LN/ReLU/Dropout backward(dy2; G2)  -> HBM    (ln_bwd196's arithmetic)
//     P2  = bf16(dG2 W2)                                 (W2^T by transposing LDS reads, the dG2 tile
//     dG1 = backward(dy2 + P2; G1)             -> HBM     as B fragments by permlane swaps: the
//     P1  = bf16(dG1 W1)                                  forward's layer hand-off run backwards)
//     dG0 = backward(dy2 + P1 + P2; G0)        -> HBM    (the stem: no dropout)
// replacing 3 g2048_ln_act_bwd + 2 g2048_linear_dgrad: dG, P and dy never round-trip through HBM
// except dG itself (the weight gradients' operand).  dG / P are bitwise those of the per-layer
// chain (same head MFMAs, same dgrad k order, same rounding points); dgamma / dbeta are summed in
// another order: per tile and layer a 16-lane reduce-scatter (DPP mirror / half-mirror / quad
// swaps) leaves lane c one of its feature group's 8 sums (4 dgamma, 4 dbeta), accumulated per lane
// -- 3 x NT registers instead of ln_bwd196's 8 NT per layer.
constexpr int kBpThreads = 256;  // 4 waves (1 per SIMD: 512 registers for the whole chain); one block per CU (LDS)
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

struct BpArgs {
    int64_t m;
    const uint16_t *w1, *w2;  // bf16 [h][h]
    const float *gamma[kMaxLayers], *beta[kMaxLayers];
    const float *wa, *wv;     // fp32 heads [4][h], [h] (wv null: decoupled critic)
    const float *dz;          // fp32 [m][8]
    const uint16_t *g[kMaxLayers];
    const float *mean[kMaxLayers], *rstd[kMaxLayers];
    P::DropArgs drop[2];      // blocks 1, 2 (the train pass's draws)
    uint16_t *dg[kMaxLayers];  // out bf16 [m][h]
    uint16_t *pout[2];        // optional out bf16 [m][h]: P1, P2
    float *part;              // out [layer][block][2 h]: dgamma | dbeta
    const uint2 *keep;        // optional: the train pass's keep bits [block][m][4] (else re-drawn)
};

// Sum of v[0..7] over the 16 lanes of a DPP row, scattered: lane c ends with the sum of
// v[4 b3 + 2 b2 + b1] (b = bits of c; lanes c, c ^ 1 hold the same value).
__device__ __forceinline__ float row16_scatter8(const float (&v)[8], int c) {
    const bool b3 = (c & 8) != 0, b2 = (c & 4) != 0, b1 = (c & 2) != 0;
    float h4[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {  // row_mirror: lane c <-> 15 - c (bit 3 differs)
        const float keep = b3 ? v[4 + j] : v[j], send = b3 ? v[j] : v[4 + j];
        h4[j] = keep + __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(send), 0x140, 0xF, 0xF, false));
    }
    float h2[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {  // row_half_mirror: c <-> 7 - c within each half (bit 2 differs)
        const float keep = b2 ? h4[2 + j] : h4[j], send = b2 ? h4[j] : h4[2 + j];
        h2[j] = keep + __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(send), 0x141, 0xF, 0xF, false));
    }
    // quad_perm 3,2,1,0 (bit 1 differs), then quad_perm 1,0,3,2 (bit 0)
    const float keep = b1 ? h2[1] : h2[0], send = b1 ? h2[0] : h2[1];
    const float h1 = keep + __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(send), 0x1B, 0xF, 0xF, false));
    return h1 + __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(h1), 0xB1, 0xF, 0xF, false));
}

#ifndef BP_STORE8  // 1: dG as 8-byte pieces per tile (round 4); 0: paired 16-byte stores
#define BP_STORE8 0
#endif
#ifndef BP_PK  // 1: the backward's LayerNorm pairs as packed fp32 (v_pk_*: few MFMAs beside them here)
#define BP_PK 1
#endif
#if BP_PK
typedef float bp2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bp2 bp_fma(bp2 a, bp2 b, bp2 c) { return __builtin_elementwise_fma(a, b, c); }
#else
using bp2 = g2048::lnrow::f32x2;
__device__ __forceinline__ bp2 bp_fma(bp2 a, bp2 b, bp2 c) { return g2048::lnrow::fma2(a, b, c); }
#endif

// dropout source of a block layer's backward: none, Philox re-draws, the train pass's stored keep bits
enum { kDmNone = 0, kDmDraw = 1, kDmBits = 2 };

// One layer's LayerNorm / ReLU / Dropout backward on the lane's tile row (ln_bwd196's two passes):
// dy = heads' share + P sources in order; dG rounded to bf16 into dgb (zero past h) and stored;
// the dgamma / dbeta partial sums of the tile go to gb[n].  The masked output gradient of each
// feature tile is held between the passes (52 registers: one wave per SIMD).  The keep multipliers
// (DM): Philox re-draws (one call per tile pair, as the per-layer kernels), or the train pass's
// stored keep bits kw (bit 4 n + e of kw.x | kw.y << 32: ppo::keep_mult) -- the same values.
template <int NT, int H, int DM, int NP>
__device__ __forceinline__ void bp_layer(const uint16_t *__restrict__ gsrc, float mu, float rs, const float *sgm,
                                         const float *sbt, const float (&wh)[NT][2], float b0, float b1,
                                         const uint2 *const (&pr)[NP > 0 ? NP : 1], const P::Drop &d, uint32_t rowu,
                                         uint2 kw, bool live, int gq, int col, uint2 (&dgb)[NT], uint16_t *dgout,
                                         float (&gb)[NT]) {
    namespace R = g2048::lnrow;
    constexpr float inv_h = 1.0f / (float)H;
    const bool lastok = 16 * (NT - 1) + 4 * gq < H;
    auto valid = [&](int n) { return n < NT - 1 || lastok; };
    uint2 gr[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) gr[n] = *reinterpret_cast<const uint2 *>(gsrc + 16 * n + 4 * gq * valid(n));
    bp2 dzr[NT][2];
    bp2 s1 = {0.0f, 0.0f}, s2 = {0.0f, 0.0f};
    const bp2 nmu = {-mu, -mu}, rs2 = {rs, rs};
    const uint32_t kb[2] = {kw.x, kw.y};
    uint4 dpair = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int n = 0; n < NT; n++) {
        const int f0 = 16 * n + 4 * gq;
        f32x4_t dy = {0.0f, 0.0f, 0.0f, 0.0f};
        dy = __builtin_amdgcn_mfma_f32_16x16x4f32(wh[n][0], b0, dy, 0, 0, 0);
        dy = __builtin_amdgcn_mfma_f32_16x16x4f32(wh[n][1], b1, dy, 0, 0, 0);
        float t[4] = {dy[0], dy[1], dy[2], dy[3]};
#pragma unroll
        for (int i = 0; i < NP; i++) {
            t[0] += R::bf_lo(pr[i][n].x);
            t[1] += R::bf_hi(pr[i][n].x);
            t[2] += R::bf_lo(pr[i][n].y);
            t[3] += R::bf_hi(pr[i][n].y);
        }
        const float4 gm = *reinterpret_cast<const float4 *>(sgm + f0);
        const float4 bt = *reinterpret_cast<const float4 *>(sbt + f0);
        const bp2 xh0 = (bp2{R::bf_lo(gr[n].x), R::bf_hi(gr[n].x)} + nmu) * rs2;
        const bp2 xh1 = (bp2{R::bf_lo(gr[n].y), R::bf_hi(gr[n].y)} + nmu) * rs2;
        const bp2 z0 = bp_fma(xh0, bp2{gm.x, gm.y}, bp2{bt.x, bt.y});
        const bp2 z1 = bp_fma(xh1, bp2{gm.z, gm.w}, bp2{bt.z, bt.w});
        const bool on = live && valid(n);
        float k[4] = {1.0f, 1.0f, 1.0f, 1.0f};
        if (DM == kDmDraw) {
            if ((n & 1) == 0) dpair = P::drop_draw4(d, rowu, (uint32_t)(f0 >> 2));
            P::drop_mult_bits(d, P::drop_half(dpair, (uint32_t)(f0 >> 2)), k);
        } else if (DM == kDmBits) {
            P::keep_mult(kb, n, d.scale, k);
        }
        const bp2 d0 = {(on && z0.x > 0.0f) ? t[0] * k[0] : 0.0f, (on && z0.y > 0.0f) ? t[1] * k[1] : 0.0f};
        const bp2 d1 = {(on && z1.x > 0.0f) ? t[2] * k[2] : 0.0f, (on && z1.y > 0.0f) ? t[3] * k[3] : 0.0f};
        dzr[n][0] = d0;
        dzr[n][1] = d1;
        const float v8[8] = {d0.x * xh0.x, d0.y * xh0.y, d1.x * xh1.x, d1.y * xh1.y, d0.x, d0.y, d1.x, d1.y};
        gb[n] += row16_scatter8(v8, col);
        const bp2 x0 = d0 * bp2{gm.x, gm.y}, x1 = d1 * bp2{gm.z, gm.w};  // dxhat
        s1 = s1 + x0 + x1;
        s2 = bp_fma(x1, xh1, bp_fma(x0, xh0, s2));
    }
    const float m1 = R::xor32_add(R::xor16_add(s1.x + s1.y)) * inv_h;
    const float m2 = R::xor32_add(R::xor16_add(s2.x + s2.y)) * inv_h;
    const bp2 nm1 = {-m1, -m1}, nm2 = {-m2, -m2};
#pragma unroll
    for (int n = 0; n < NT; n++) {
        const int f0 = 16 * n + 4 * gq;
        const float4 gm = *reinterpret_cast<const float4 *>(sgm + f0);
        const bp2 xh0 = (bp2{R::bf_lo(gr[n].x), R::bf_hi(gr[n].x)} + nmu) * rs2;
        const bp2 xh1 = (bp2{R::bf_lo(gr[n].y), R::bf_hi(gr[n].y)} + nmu) * rs2;
        const bp2 o0 = bp_fma(xh0, nm2, bp_fma(dzr[n][0], bp2{gm.x, gm.y}, nm1)) * rs2;
        const bp2 o1 = bp_fma(xh1, nm2, bp_fma(dzr[n][1], bp2{gm.z, gm.w}, nm1)) * rs2;
        dgb[n] = valid(n) ? make_uint2(R::pack_bf2(o0.x, o0.y), R::pack_bf2(o1.x, o1.y)) : make_uint2(0u, 0u);
#if BP_STORE8
        if (live && valid(n)) *reinterpret_cast<uint2 *>(dgout + f0) = dgb[n];
#endif
    }
#if !BP_STORE8
    if (live) store_row16<NT, H>(reinterpret_cast<char *>(dgout), dgb, gq);  // 16-byte stores (mlp_tile.hpp)
#endif
}

// P^T tile chain of one block layer: p[n] = bf16(sum_ks W^T[16 n ..][k-step ks] dG^T) -- the
// dgrad kernel's k order from zero.  A = W^T by two transposing reads of the row-major image
// (lane (g, q, p): rows 32 ks + 8 g + q and + 4, columns 16 n + 4 p); k-step rows past h are
// redirected to row 0 (their B is zero: dG past h is zero).
template <int NT, int H, int KS, int PW>
__device__ __forceinline__ void bp_dgrad(const char *wimg, const uint2 (&dgb)[NT], int lane, uint2 (&pout)[NT]) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
    f32x4_t acc[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) acc[n] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
        const uint4 bf = act_frag<NT>(dgb, ks);
        const int r1 = 32 * ks + 8 * g + q;
        const int ra = r1 < H ? r1 : 0, rb = r1 + 4 < H ? r1 + 4 : 0;
        int oa = ra * PW + 8 * p4, ob = rb * PW + 8 * p4;
        asm volatile("" : "+v"(oa), "+v"(ob));
#pragma unroll
        for (int n = 0; n < NT; n++) {
            const s16x4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(wimg + oa + 32 * n));
            const s16x4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(wimg + ob + 32 * n));
            const bf16x8_t fa = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(t1, t2, 0, 1, 2, 3, 4, 5, 6, 7));
            acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, as_frag(bf), acc[n], 0, 0, 0);
        }
    }
#pragma unroll
    for (int n = 0; n < NT; n++) pout[n] = make_uint2(pack_bf2(acc[n][0], acc[n][1]), pack_bf2(acc[n][2], acc[n][3]));
}

template <int H, int DM>
__global__ __launch_bounds__(kBpThreads, 1) void mlp_back_kernel(BpArgs a) {
    constexpr int NT = (H + 15) / 16, KS = ((H + 7) / 8 * 8 + 31) / 32;
    constexpr int PW = pr_pitch(H), WB = pr_wbytes(H);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *sLN = reinterpret_cast<float *>(smem + 2 * WB);  // [layer][gamma | beta][16 NT]
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int gq = lane >> 4, col = lane & 15;
    const int64_t m = a.m;
    {  // the block weight images (row-major, forward's pitch) and the LayerNorm affines
        constexpr int q8 = PW / 8, h4 = H / 4, per = H * q8;
        const uint16_t *wsrc[2] = {a.w1, a.w2};
#pragma unroll
        for (int l = 0; l < 2; l++)
            for (int c0 = 0; c0 < per; c0 += 8 * kBpThreads) {
                uint2 v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int c = c0 + tid + u * kBpThreads, r = c / q8, q = c - r * q8;
                    v[u] = (c < per && q < h4) ? *reinterpret_cast<const uint2 *>(wsrc[l] + (int64_t)r * H + 4 * q)
                                               : make_uint2(0u, 0u);
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int c = c0 + tid + u * kBpThreads, r = c / q8, q = c - r * q8;
                    if (c < per) *reinterpret_cast<uint2 *>(smem + l * WB + r * PW + 8 * q) = v[u];
                }
            }
        for (int e = tid; e < kMaxLayers * 2 * 16 * NT; e += kBpThreads) {
            const int l = e / (32 * NT), rem = e - l * 32 * NT, which = rem / (16 * NT), f = rem - which * 16 * NT;
            const float *src = which ? a.beta[l] : a.gamma[l];
            sLN[e] = f < H ? src[f] : 0.0f;
        }
    }
    // the heads' A fragments of v_mfma_f32_16x16x4_f32 for the whole launch: lane (k = gq, i = col)
    // holds W_heads[k][16 n + i] and W_heads[4 + k][..] (rows: wa 0..3, wv, zero)
    float wh[NT][2];
#pragma unroll
    for (int n = 0; n < NT; n++) {
        const int f = 16 * n + col;
        wh[n][0] = f < H ? a.wa[gq * H + f] : 0.0f;
        wh[n][1] = (f < H && gq == 0 && a.wv) ? a.wv[f] : 0.0f;
    }
    __syncthreads();
    const P::Drop d1 = P::make_drop(a.drop[0]), d2 = P::make_drop(a.drop[1]);
    float gb[kMaxLayers][NT];
#pragma unroll
    for (int l = 0; l < kMaxLayers; l++)
#pragma unroll
        for (int n = 0; n < NT; n++) gb[l][n] = 0.0f;
    const int64_t ntile = (m + 15) >> 4;
    for (int64_t tile = (int64_t)blockIdx.x * (kBpThreads / 64) + wave; tile < ntile;
         tile += (int64_t)gridDim.x * (kBpThreads / 64)) {
        const int64_t row = 16 * tile + col;
        const bool live = row < m;
        const int64_t rc = live ? row : 0;
        const uint32_t rowu = (uint32_t)rc;
        const float b0 = a.dz[rc * 8 + gq];
        const float b1 = gq == 0 ? a.dz[rc * 8 + 4] : 0.0f;
        uint2 kw1 = make_uint2(0u, 0u), kw2 = make_uint2(0u, 0u);
        if (DM == kDmBits) {  // [block][row][lane group]: the train pass's keep bits of this row
            kw1 = a.keep[rc * 4 + gq];
            kw2 = a.keep[(m + rc) * 4 + gq];
        }
        uint2 dgb[NT], p2[NT], p1[NT];
        // block 2 (top): dy = the heads' share
        {
            const uint2 *pr[1] = {nullptr};
            bp_layer<NT, H, DM, 0>(a.g[2] + rc * H, a.mean[2][rc], a.rstd[2][rc], sLN + 2 * 32 * NT,
                                   sLN + 2 * 32 * NT + 16 * NT, wh, b0, b1, pr, d2, rowu, kw2, live, gq, col, dgb,
                                   a.dg[2] + rc * H, gb[2]);
        }
        bp_dgrad<NT, H, KS, PW>(smem + WB, dgb, lane, p2);
        if (a.pout[1] && live) store_tile<NT, H>(a.pout[1], (uint32_t)rc * (2u * H), p2, gq);
        {  // block 1: + P2
            const uint2 *pr[1] = {p2};
            bp_layer<NT, H, DM, 1>(a.g[1] + rc * H, a.mean[1][rc], a.rstd[1][rc], sLN + 32 * NT, sLN + 48 * NT, wh,
                                   b0, b1, pr, d1, rowu, kw1, live, gq, col, dgb, a.dg[1] + rc * H, gb[1]);
        }
        bp_dgrad<NT, H, KS, PW>(smem, dgb, lane, p1);
        if (a.pout[0] && live) store_tile<NT, H>(a.pout[0], (uint32_t)rc * (2u * H), p1, gq);
        {  // the stem: + P1 + P2 (the per-layer chain's source order), no dropout
            const uint2 *pr[2] = {p1, p2};
            bp_layer<NT, H, kDmNone, 2>(a.g[0] + rc * H, a.mean[0][rc], a.rstd[0][rc], sLN, sLN + 16 * NT,
                                                  wh, b0, b1, pr, d1, rowu, kw1, live, gq, col, dgb, a.dg[0] + rc * H,
                                                  gb[0]);
        }
    }
    // dgamma / dbeta: lane (gq, col) even col holds slot s = col >> 1 of its feature groups
    // (s < 4: dgamma of feature 16 n + 4 gq + s, else dbeta of feature s - 4); block sum in LDS
    __syncthreads();
    float *red = reinterpret_cast<float *>(smem);  // [wave][layer][2][16 NT]
    constexpr int RW = kMaxLayers * 2 * 16 * NT;
    if ((col & 1) == 0) {
        const int s = col >> 1, which = s >> 2, e = s & 3;
#pragma unroll
        for (int l = 0; l < kMaxLayers; l++)
#pragma unroll
            for (int n = 0; n < NT; n++) red[wave * RW + (l * 2 + which) * 16 * NT + 16 * n + 4 * gq + e] = gb[l][n];
    }
    __syncthreads();
    const int nb = gridDim.x;
    for (int c = tid; c < kMaxLayers * 2 * H; c += kBpThreads) {  // partial rows [layer][block][dgamma h | dbeta h]
        const int l = c / (2 * H), rem = c - l * 2 * H, which = rem >= H, f = rem - which * H;
        const int src = (l * 2 + which) * 16 * NT + f;
        float t = 0.0f;
#pragma unroll
        for (int w = 0; w < kBpThreads / 64; w++) t += red[w * RW + src];
        a.part[((int64_t)l * nb + blockIdx.x) * 2 * H + rem] = t;
    }
}

inline int fp_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}

inline bool al(const void *p, unsigned n) { return ((uintptr_t)p % n) == 0u; }

size_t fp_lds(int h) { return (size_t)pr_lds_bytes(h, (h + 15) / 16); }

int fp_blocks(int64_t m) {
    const int64_t b = (m + kFpBlockRows - 1) / kFpBlockRows;
    return (int)(b < 1 ? 1 : (b > 256 ? 256 : b));
}

bool fp_shape(int h) { return (h == 196 || h == 192 || h == 128 || h == 64 || h == 32) && fp_lds(h) <= (size_t)kFpLdsMax; }

// Segments of the deferred / immediate column sums (ppo_update.hip's colsum, re-stated here for
// this translation unit's two kernels).
int fp_colsum(hipStream_t s, const float *part, int nb, int cols, int max_col, float *const *dst, const int *len,
              int nseg, g2048_colsum_job *defer) {
    g2048_colsum_job job{};
    job.part = part;
    job.nb = nb;
    job.cols = cols;
    job.max_col = max_col;
    job.nseg = nseg;
    for (int k = 0; k < nseg; k++) {
        job.dst[k] = dst[k];
        job.len[k] = len[k];
    }
    if (defer) {
        *defer = job;
        return fp_status();
    }
    return g2048_colsum_batch((g2048_stream_t)s, &job, 1);
}

int fp_fill(const g2048_mlp_pass_args *p, FpArgs &a, bool train) {
    const int h = p->hidden;
    // byte offsets of a row in the [m][h] bf16 outputs are 32-bit (m 2 h < 2^32: m up to ~10 M rows)
    if (!fp_shape(h) || p->m <= 0 || p->m * 2 * h >= (int64_t(1) << 32)) return G2048_EINVAL;
    if (!p->boards || !p->batch.idx || !p->w_stem || !p->w_block[0] || !p->w_block[1] || !p->head_frag || !p->ba ||
        !p->masked || !p->partials)
        return G2048_EINVAL;
    for (int l = 0; l < 3; l++)
        if (!p->ln_gamma[l] || !p->ln_beta[l]) return G2048_EINVAL;
    if (!al(p->boards, 16) || !al(p->head_frag, 16) || !al(p->w_stem, 16) || !al(p->w_block[0], 8) || !al(p->w_block[1], 8) || !al(p->masked, 16))
        return G2048_EINVAL;
    if (train) {
        if (!p->bv || !p->dz || !p->dz_bf16 || !p->beta_dev || !p->batch.action || !p->batch.legal ||
            !p->batch.old_logp || !p->batch.adv || !p->batch.ret)
            return G2048_EINVAL;
        if (!al(p->dz, 16) || !al(p->dz_bf16, 16) || (p->x0 && !al(p->x0, 16)) || !al(p->batch.old_logp, 16))
            return G2048_EINVAL;
        for (int l = 0; l < 3; l++)
            if ((p->g[l] && !al(p->g[l], 8)) || (p->h[l] && !al(p->h[l], 8)) || (!p->mean[l]) != (!p->rstd[l]))
                return G2048_EINVAL;
    }
    a = FpArgs{};
    a.boards = p->boards;
    a.m = p->m;
    a.la = P::HeadLossArgs{p->batch.idx, p->batch.action, p->batch.legal, p->batch.old_logp, p->batch.adv, p->batch.ret,
                           p->beta_dev, p->batch.rows, p->critic, 1.0f - p->clip_eps, 1.0f + p->clip_eps,
                           1.0f / (float)p->m, p->decouple_critic};
    a.w0 = (const uint16_t *)p->w_stem;
    a.w1 = (const uint16_t *)p->w_block[0];
    a.w2 = (const uint16_t *)p->w_block[1];
    for (int l = 0; l < 3; l++) {
        a.gamma[l] = p->ln_gamma[l];
        a.beta[l] = p->ln_beta[l];
        a.g[l] = (uint16_t *)p->g[l];
        a.h[l] = (uint16_t *)p->h[l];
        a.mean[l] = p->mean[l];
        a.rstd[l] = p->rstd[l];
    }
    a.ba = p->ba;
    a.bv = p->bv;
    a.head = (const uint4 *)p->head_frag;
    a.drop[0] = P::drop_args(&p->drop[0]);
    a.drop[1] = P::drop_args(&p->drop[1]);
    if ((a.drop[0].thr != 0u) != (a.drop[1].thr != 0u)) return G2048_EINVAL;  // both blocks share nn.Dropout(p)
    a.x0 = (uint16_t *)p->x0;
    a.masked = p->masked;
    a.dz = p->dz;
    a.dzb = (uint16_t *)p->dz_bf16;
    a.part = p->partials;
    if (train && p->keep && !al(p->keep, 8)) return G2048_EINVAL;
    a.keep = train ? (uint2 *)p->keep : nullptr;
    a.idx_off = p->idx_offset;
    return G2048_OK;
}

template <bool TRAIN, bool DROP>
int fp_launch2(hipStream_t s, const FpArgs &a, int h, int nb) {
    const size_t lds = fp_lds(h);
    switch (h) {
    case 196: hipLaunchKernelGGL((mlp_pass_kernel<196, TRAIN, DROP>), dim3(nb), dim3(kFpThreads), lds, s, a); break;
    case 192: hipLaunchKernelGGL((mlp_pass_kernel<192, TRAIN, DROP>), dim3(nb), dim3(kFpThreads), lds, s, a); break;
    case 128: hipLaunchKernelGGL((mlp_pass_kernel<128, TRAIN, DROP>), dim3(nb), dim3(kFpThreads), lds, s, a); break;
    case 64: hipLaunchKernelGGL((mlp_pass_kernel<64, TRAIN, DROP>), dim3(nb), dim3(kFpThreads), lds, s, a); break;
    case 32: hipLaunchKernelGGL((mlp_pass_kernel<32, TRAIN, DROP>), dim3(nb), dim3(kFpThreads), lds, s, a); break;
    default: return G2048_EINVAL;
    }
    return fp_status();
}

template <bool TRAIN>
int fp_launch(hipStream_t s, const FpArgs &a, int h, int nb) {
    return a.drop[0].thr != 0u ? fp_launch2<TRAIN, true>(s, a, h, nb) : fp_launch2<TRAIN, false>(s, a, h, nb);
}

int bp_blocks(int64_t m) {
    const int64_t t = ((m + 15) / 16 + kBpThreads / 64 - 1) / (kBpThreads / 64);
    return (int)(t < 1 ? 1 : (t > 256 ? 256 : t));
}

template <int DM>
int bp_launch2(hipStream_t s, const BpArgs &a, int h, int nb) {
    const size_t lds = fp_lds(h);
    switch (h) {
    case 196: hipLaunchKernelGGL((mlp_back_kernel<196, DM>), dim3(nb), dim3(kBpThreads), lds, s, a); break;
    case 192: hipLaunchKernelGGL((mlp_back_kernel<192, DM>), dim3(nb), dim3(kBpThreads), lds, s, a); break;
    case 128: hipLaunchKernelGGL((mlp_back_kernel<128, DM>), dim3(nb), dim3(kBpThreads), lds, s, a); break;
    case 64: hipLaunchKernelGGL((mlp_back_kernel<64, DM>), dim3(nb), dim3(kBpThreads), lds, s, a); break;
    case 32: hipLaunchKernelGGL((mlp_back_kernel<32, DM>), dim3(nb), dim3(kBpThreads), lds, s, a); break;
    default: return G2048_EINVAL;
    }
    return fp_status();
}

}  // namespace

extern "C" {

size_t g2048_head_split_bytes(int32_t hidden) { return hidden > 0 ? (size_t)16 * 64 * ((hidden + 31) / 32) : 0; }

int g2048_head_split(g2048_stream_t stream, const float *wa, const float *wv, int32_t hidden, void *frag) {
    if (hidden <= 0 || hidden > 1024 || !wa || !frag || !al(frag, 16)) return G2048_EINVAL;
    const int ks = (hidden + 31) / 32;
    hipLaunchKernelGGL(head_split_kernel, dim3((unsigned)((ks * 64 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, wa,
                       wv, (int)hidden, ks, (uint4 *)frag);
    return fp_status();
}

int g2048_mlp_pass_supported(int32_t hidden, int32_t num_layers) { return num_layers == 2 && fp_shape(hidden) ? 1 : 0; }

size_t g2048_mlp_pass_partials(int64_t m, int32_t train) {
    if (m <= 0) return 0;
    return (size_t)fp_blocks(m) * (train ? kTrainParts : 2);
}

int g2048_ppo_forward_loss(g2048_stream_t stream, const g2048_mlp_pass_args *p, float *dba, float *dbv, float *sums,
                           g2048_colsum_job *defer) {
    if (!p || !dba || !dbv || !sums) return G2048_EINVAL;
    FpArgs a;
    const int st = fp_fill(p, a, true);
    if (st) return st;
    const hipStream_t s = (hipStream_t)stream;
    const int nb = fp_blocks(p->m);
    const int rc = fp_launch<true>(s, a, p->hidden, nb);
    if (rc) return rc;
    float *dst[3] = {dba, dbv, sums};
    const int len[3] = {4, 1, 3};
    return fp_colsum(s, p->partials, nb, kTrainParts, -1, dst, len, 3, defer);
}

size_t g2048_mlp_back_partials(int64_t m, int32_t hidden) {
    if (m <= 0 || hidden <= 0) return 0;
    return (size_t)kMaxLayers * bp_blocks(m) * 2 * hidden;
}

int g2048_ppo_backward(g2048_stream_t stream, const g2048_mlp_back_args *p, float *const *dgamma, float *const *dbeta,
                       g2048_colsum_job *defer) {
    if (!p || !dgamma || !dbeta) return G2048_EINVAL;
    const int h = p->hidden;
    if (!fp_shape(h) || p->m <= 0 || p->m * 2 * h >= (int64_t(1) << 32)) return G2048_EINVAL;
    if (!p->w_block[0] || !p->w_block[1] || !p->wa || !p->dz || !p->partials || !al(p->dz, 16) ||
        !al(p->w_block[0], 8) || !al(p->w_block[1], 8))
        return G2048_EINVAL;
    BpArgs a{};
    a.m = p->m;
    a.w1 = (const uint16_t *)p->w_block[0];
    a.w2 = (const uint16_t *)p->w_block[1];
    for (int l = 0; l < kMaxLayers; l++) {
        if (!p->ln_gamma[l] || !p->ln_beta[l] || !p->g[l] || !p->mean[l] || !p->rstd[l] || !p->dg[l] || !dgamma[l] ||
            !dbeta[l] || !al(p->g[l], 8) || !al(p->dg[l], 8))
            return G2048_EINVAL;
        a.gamma[l] = p->ln_gamma[l];
        a.beta[l] = p->ln_beta[l];
        a.g[l] = (const uint16_t *)p->g[l];
        a.mean[l] = p->mean[l];
        a.rstd[l] = p->rstd[l];
        a.dg[l] = (uint16_t *)p->dg[l];
    }
    a.wa = p->wa;
    a.wv = p->wv;
    a.dz = p->dz;
    a.drop[0] = P::drop_args(&p->drop[0]);
    a.drop[1] = P::drop_args(&p->drop[1]);
    if ((a.drop[0].thr != 0u) != (a.drop[1].thr != 0u)) return G2048_EINVAL;
    a.part = p->partials;
    if (p->keep && !al(p->keep, 8)) return G2048_EINVAL;
    a.keep = (const uint2 *)p->keep;
    for (int i = 0; i < 2; i++) {
        if (p->p_out[i] && !al(p->p_out[i], 8)) return G2048_EINVAL;
        a.pout[i] = (uint16_t *)p->p_out[i];
    }
    const hipStream_t s = (hipStream_t)stream;
    const int nb = bp_blocks(p->m);
    const int rc = a.drop[0].thr == 0u ? bp_launch2<kDmNone>(s, a, h, nb)
                   : a.keep        ? bp_launch2<kDmBits>(s, a, h, nb)
                                   : bp_launch2<kDmDraw>(s, a, h, nb);
    if (rc) return rc;
    const int w = 2 * h;
    for (int l = 0; l < kMaxLayers; l++) {  // one column-sum job per layer: [dgamma | dbeta] rows of 2 h
        float *dst[2] = {dgamma[l], dbeta[l]};
        const int len[2] = {h, h};
        g2048_colsum_job job{};
        job.part = p->partials + (size_t)l * nb * w;
        job.nb = nb;
        job.cols = w;
        job.max_col = -1;
        job.nseg = 2;
        job.dst[0] = dst[0];
        job.dst[1] = dst[1];
        job.len[0] = len[0];
        job.len[1] = len[1];
        if (defer) {
            defer[l] = job;
        } else {
            const int st = g2048_colsum_batch(stream, &job, 1);
            if (st) return st;
        }
    }
    return fp_status();
}

int g2048_ppo_forward_kl_stats(g2048_stream_t stream, const g2048_mlp_pass_args *p, const g2048_ppo_stats_args *st) {
    if (!p || !st || !st->sums || !st->grad_norm || !st->beta_dev || !st->stats || !st->sync || st->m <= 0)
        return G2048_EINVAL;
    FpArgs a;
    const int rc0 = fp_fill(p, a, false);
    if (rc0) return rc0;
    a.st = P::StatsArgs{st->sums, st->grad_norm, st->beta_dev, st->rows, st->stats, st->counter, st->sync,
                        st->critic, (float)st->m, st->idx_offset, st->idx_step};
    return fp_launch<false>((hipStream_t)stream, a, p->hidden, fp_blocks(p->m));
}

int g2048_ppo_forward_kl(g2048_stream_t stream, const g2048_mlp_pass_args *p, float *out, g2048_colsum_job *defer) {
    if (!p || !out) return G2048_EINVAL;
    FpArgs a;
    const int st = fp_fill(p, a, false);
    if (st) return st;
    const hipStream_t s = (hipStream_t)stream;
    const int nb = fp_blocks(p->m);
    const int rc = fp_launch<false>(s, a, p->hidden, nb);
    if (rc) return rc;
    float *dst[1] = {out};
    const int len[1] = {2};
    return fp_colsum(s, p->partials, nb, 2, 1, dst, len, 1, defer);
}

}  // extern "C"
