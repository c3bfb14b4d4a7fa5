// policy_rollout.hip -- the fused persistent policy rollout: K consecutive
// steps of play_game_for_episode's loop body (train.py:240-337) for every env in ONE launch,
//
//     obs = to_model_format(board)                        game.py:92-101
//     logits, value = GameMLP(obs)  (eval mode)           game.py:1145-1220
//     action ~ masked softmax(logits)                     train.py:266-291, 326
//     board = Game2048.step(board, action)                game.py:952-1030
//
// writing the same time-major records as the per-step path of g2048/rollout.py (Rollout._step:
// obs_encode -> FusedPolicy = 3 x g2048_mlp_fwd + g2048_head_fwd -> g2048_sample_actions ->
// g2048_env_step), and with the same arithmetic: every operand fragment, MFMA accumulation chain,
// rounding and reduction order of those kernels is reproduced, so the records are bitwise those of
// the per-step path at the same seed and counter (tests/test_gpu_policy_rollout.py).
//
// Layout (one 256-thread workgroup per CU, persistent over groups of 256 boards):
//   * lane = board: each of the 4 waves owns 64 boards (4 MFMA board tiles of 16); the board, its
//     legal mask and the env step stay in the lane's registers for all K steps.
//   * GameMLP on v_mfma_f32_16x16x32_bf16 as Y^T = W X^T (g2048_mlp_fwd's orientation): lane (g, c)
//     of board tile bt holds features 16n + 4g + r of board 16 bt + c.  A layer's output becomes the
//     next layer's B operand in registers: for k-step ks, two v_permlane32_swap + two
//     v_permlane16_swap per dword pair turn tiles 2ks, 2ks+1 ("lane g holds features 4g..4g+3")
//     into the fragment ("lane g holds k = 8g..8g+7") -- no LDS round trip, natural k order.
//   * LDS (160 KiB): the two h x h block weights (bf16, row pitch round_up(h, 8)), the three
//     LayerNorm affines (fp32) and a zero fragment.  The stem
//     (h x 48) and the heads are read from global memory (L1/L2-resident, 19 KB + 2 KB).
//   * heads: one MFMA chain over (board tile, k-step) whose A operand is non-zero only in rows
//     4 bt .. 4 bt + 3 for board tile bt, so lane (g, c) ends with the 4 logits of board 16 g + c --
//     its own env lane -- with no transpose; a second chain does the value.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "board.hpp"
#include "step.hpp"
#include "ln_row.hpp"
#include "mlp_tile.hpp"
#include "../../include/g2048.h"
#include "../../include/g2048_ppo.h"

using namespace g2048;

namespace {

using namespace g2048::tile;

#ifndef PR_BPW
#define PR_BPW 32
#endif
// Round 5: 32 boards per wave, i.e. two waves per SIMD at 256 VGPRs each with one 16-board tile per
// MLP pass (kQ = 1).  The env step and the sampler then run on half-empty waves, but a partner wave's
// MFMAs cover each wave's LN epilogues and LDS waits: 31.4 -> 29.3 us per step at 65 536 envs
// (kQ = 1 at 64 boards per wave, one wave per SIMD, measured 37 us; kQ = 2 at 32 spills 376 B).
constexpr int kBpw = PR_BPW;               // boards per wave (64: one wave per SIMD; 32: two)
constexpr int kPrBoards = 256;             // boards per workgroup (one per CU: the LDS weight images)
constexpr int kPrThreads = kPrBoards / kBpw * 64;
constexpr int kPrLdsMax = 163840;
constexpr int kPrRecBytes = 4 * 80;  // the stem fragment recipes of the 4 lane groups (LDS, after the zero fragment)
#ifndef PR_PHPAIR
#define PR_PHPAIR (PR_BPW == 32)
#endif
static_assert(!PR_PHPAIR || PR_BPW == 32, "the paired Philox draws need half-empty waves");
#ifndef PR_CARRY
#define PR_CARRY PR_PHPAIR
#endif
static_assert(!PR_CARRY || PR_PHPAIR, "the carried step takes the paired spawn words");
#ifndef PR_NOSEL
#define PR_NOSEL 1
#endif
constexpr int kPrGap = PR_NOSEL ? 64 : 0;
#ifndef PR_TILES
#define PR_TILES 1
#endif
constexpr int kQ = PR_TILES;  // board tiles (of 16 boards) per MLP pass: accumulators of kQ x NT tiles
#ifndef PR_NSPLIT
#define PR_NSPLIT 0
#endif

struct PrArgs {
    uint4 *boards;      // [T+1][n][16] int8: row t0 read, rows t0+1 .. t1 written
    uint8_t *flags;     // [T+1][n]
    uint8_t *actions;   // [T][n]
    float *logp;        // [T][n][4]
    float *entropy;     // [T][n]
    float *value;       // [T][n]
    int32_t *points;    // [T][n]
    int8_t *max_tile;   // [T][n]
    uint32_t *pot;      // [T][n] (mono_b, mono_a, empt_b, empt_a)
    int64_t n;
    int32_t t0, t1, h, opts;
    const uint16_t *w0;            // stem Linear bf16 [h][48]
    const uint16_t *w1, *w2;       // block Linears bf16 [h][h]
    const float *gamma[kMaxLayers], *beta[kMaxLayers];
    const uint16_t *head;          // bf16 [5][32 KS]: action_head rows 0..3, value_head row 4, zero padded
    const float *ba, *bv;          // head biases (fp32)
    uint64_t seed;
    const uint64_t *counter_dev;
    uint64_t counter;
    uint32_t env_base;
    float *debug;  // optional test hook: layer outputs and head outputs of step t0
};

// debug: layer l's output (bf16 values as fp32) of board `board` into debug[(l n + board) 16 NT + f]
template <int NT>
__device__ __forceinline__ void debug_act(const PrArgs &a, int l, int64_t board, const uint2 (&act)[NT], int g) {
    if (board >= a.n) return;
    float *d = a.debug + ((int64_t)l * a.n + board) * (16 * NT);
#pragma unroll
    for (int n = 0; n < NT; n++) {
        const int f = 16 * n + 4 * g;
        d[f] = bf_lo(act[n].x);
        d[f + 1] = bf_hi(act[n].x);
        d[f + 2] = bf_lo(act[n].y);
        d[f + 3] = bf_hi(act[n].y);
    }
}

// The sampler of g2048_sample_actions (g2048.hip, sample_kernel; built there with
// -ffp-contract=off): masked softmax, inverse-CDF action of the stream-1 Philox uniform, entropy,
// log_softmax with -inf on illegal actions.
__device__ __forceinline__ uint32_t sample_row(const float (&l)[4], uint32_t legal, uint32_t u32, float (&lp)[4],
                                               float &ent) {
    float m = -INFINITY;
#pragma unroll
    for (int a = 0; a < 4; a++)
        if ((legal >> a) & 1u) m = fmaxf(m, l[a]);
    float e[4], s = 0.0f;
#pragma unroll
    for (int a = 0; a < 4; a++) {
        e[a] = ((legal >> a) & 1u) ? smp_exp(l[a] - m) : 0.0f;
        s += e[a];
    }
    const float ls = smp_log(s), inv = smp_rcp(s);
    const float u = (float)(u32 >> 8) * (1.0f / 16777216.0f);
    float cum = 0.0f, hh = 0.0f;
    uint32_t act = 0xFFu;
#pragma unroll
    for (int a = 0; a < 4; a++) {
        const bool ok = (legal >> a) & 1u;
        const float p = e[a] * inv, lq = (l[a] - m) - ls;
        if (ok) {
            cum += p;
            if (act == 0xFFu && u < cum) act = (uint32_t)a;
            if (p > 0.0f) hh -= p * lq;
        }
        lp[a] = ok ? lq : -INFINITY;
    }
    if (act == 0xFFu) {
#pragma unroll
        for (int a = 0; a < 4; a++)
            if ((legal >> a) & 1u) act = (uint32_t)a;
        if (!legal) act = 0u;
    }
    ent = legal ? hh : 0.0f;
    return act;
}

// H = the hidden size (compile time: every feature-validity test of the last tile folds away).
template <int H>
__global__ __launch_bounds__(kPrThreads, 1) void policy_rollout_kernel(PrArgs a) {
    constexpr int NT = (H + 15) / 16, KS = ((H + 7) / 8 * 8 + 31) / 32;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int h = H;
    constexpr int P = pr_pitch(h), WB = pr_wbytes(h);
    char *sW[2] = {smem, smem + WB};  // block weight images (LDS offsets 0 and WB)
    // kPrGap zero bytes behind the second image: the last k-step's reads past row h - 1 (PR_NOSEL)
    float *sLN = reinterpret_cast<float *>(smem + 2 * WB + kPrGap);  // [layer][gamma | beta][16 NT]
    char *sZero = smem + 2 * WB + kPrGap + 2 * kMaxLayers * pr_ln_floats(NT) * 4;
    char *sRec = sZero + 16;  // [g][sc0 sc1 ss0 ss1 {sx0 sx1 sd0 sd1}] uint4
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, col = lane & 15;

    // ---- stage the block weights (bank-spread rows, zero K padding), LayerNorm affines, zero block
    {
        const int q8 = P / 8, h4 = h / 4;  // 8-byte pieces per LDS row / per global row
        const uint16_t *wsrc[2] = {a.w1, a.w2};
        for (int l = 0; l < 2; l++)
            for (int c = tid; c < h * q8; c += kPrThreads) {
                const int r = c / q8, q = c - r * q8;
                const uint2 v = q < h4 ? *reinterpret_cast<const uint2 *>(wsrc[l] + (int64_t)r * h + 4 * q) : make_uint2(0u, 0u);
                *reinterpret_cast<uint2 *>(sW[l] + pr_piece(h, r, q)) = v;
            }
        for (int e = tid; e < kMaxLayers * 2 * 16 * NT; e += kPrThreads) {
            const int l = e / (32 * NT), rem = e - l * 32 * NT, which = rem / (16 * NT), f = rem - which * 16 * NT;
            const float *src = which ? a.beta[l] : a.gamma[l];
            sLN[e] = f < h ? src[f] : 0.0f;
        }
        if (tid < 4) reinterpret_cast<uint32_t *>(sZero)[tid] = 0u;
        if (tid < kPrGap / 4) reinterpret_cast<uint32_t *>(smem + 2 * WB)[tid] = 0u;
        if (tid < 20) {
            const StemFrag &e = kStem.f[tid / 5][0], &f = kStem.f[tid / 5][1];
            const int j = tid % 5;
            reinterpret_cast<uint4 *>(sRec)[tid] = j == 0 ? make_uint4(e.c[0], e.c[1], e.c[2], e.c[3])
                                                 : j == 1 ? make_uint4(f.c[0], f.c[1], f.c[2], f.c[3])
                                                 : j == 2 ? make_uint4(e.sel[0], e.sel[1], e.sel[2], e.sel[3])
                                                 : j == 3 ? make_uint4(f.sel[0], f.sel[1], f.sel[2], f.sel[3])
                                                          : make_uint4(e.xsel, f.xsel, e.d, f.d);
        }
    }
    __syncthreads();

    constexpr float inv_n = 1.0f / (float)h;
    constexpr int hp8 = (h + 7) & ~7;
    constexpr int KP = 32 * KS;  // padded row length of the head buffer
    const uint64_t ctr0 = a.counter + (a.counter_dev ? *a.counter_dev : 0ull);
    RngArgs rng{a.seed, 0ull, nullptr, a.env_base, nullptr, nullptr};

    const int recoff = (int)(sRec - smem) + 80 * g;  // this lane group's stem fragment recipe (kStem)
    // A-fragment LDS offsets of the block weights: row 16 n + col, k = 32 ks + 8 g (+ 16 n P per tile);
    // wlane_x in the swizzled k-step groups (pr_piece)
    const int wlane = col * P + 16 * g, wlane_x = col * P + 16 * (g ^ pr_swz(h, col));
    [[maybe_unused]] const int zoff = (int)(sZero - smem);
    [[maybe_unused]] constexpr int last_rows = h - 16 * (NT - 1);  // valid rows of the last tile

    for (int64_t base = (int64_t)blockIdx.x * kPrBoards; base < a.n; base += (int64_t)gridDim.x * kPrBoards) {
        if (base + kBpw * wave >= a.n) continue;  // an empty wave (no barrier below)
        const int64_t i = base + kBpw * wave + lane;
        const bool live = lane < kBpw && i < a.n;  // (kBpw 32: lanes 32..63 carry no board)
        uint4 b = live ? a.boards[(int64_t)a.t0 * a.n + i] : make_uint4(0u, 0u, 0u, 0u);
        uint32_t legal = live ? (uint32_t)(a.flags[(int64_t)a.t0 * a.n + i] & 0xFu) : 0u;
#if PR_CARRY
        BoardCarry carry = board_carry(b);  // the board's statistics, carried (step.hpp step_board_carry)
#endif

        for (int t = a.t0; t < a.t1; t++) {
            // opaque per-step copies of the lane offsets: without them the compiler hoists every
            // (tile, k-step) fragment address out of the step loop and spills them
            int wlane_t = wlane, wlane_xt = wlane_x, glane_t = (col * 48 + 8 * g) * 2, hlane_t = ((col & 3) * KP + 8 * g) * 2;
            asm volatile("" : "+v"(wlane_t), "+v"(wlane_xt), "+v"(glane_t), "+v"(hlane_t));
            // the stem weight fragments through a buffer descriptor (as ppo_fused.hip): rows past h and
            // k past 48 (ks 1, lane groups 2, 3) read out of range = zero, no per-lane branch / zeroing
            const __amdgpu_buffer_rsrc_t w0r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(a.w0), 0, h * 96, 0x00020000);
            const int w0off[2] = {glane_t, g < 2 ? glane_t + 64 : h * 96};
            // the head rows through a buffer descriptor: a lane whose board tile is not the chain's
            // reads out of range (zero) -- one select per tile instead of 8 per k-step
            const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(a.head), 0, 5 * KP * 2, 0x00020000);
            const int hvlane = (4 * KP + 8 * g) * 2;
            // The MLP runs on two board tiles at a time (accumulators of 2 x NT tiles; the weight
            // fragments are read once per pair): stem, blocks and the pair's share of the head
            // chains.  A pair's epilogue overwrites its own layer input (the residual) in place.
            f32x4_t accL = {0.0f, 0.0f, 0.0f, 0.0f}, accV = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 1
            for (int pr = 0; pr < kBpw / 16 / kQ; pr++) {
                uint2 act[kQ][NT];
                // ---------------- stem: obs fragments (to_model_format, natural k order) ------
                uint4 xs[kQ][2];
                // the recipe re-read from LDS per pair (20 registers less across the MLP); an opaque
                // offset keeps the reads inside the loop
                int rco = recoff, lno = 0;
                asm volatile("" : "+v"(rco), "+v"(lno));
                // the LayerNorm affines from an opaque per-pair base: one address register and
                // immediate offsets (else every (layer, tile) address is hoisted and parked in AGPRs)
                const float *sLNr = sLN + lno;
                const uint4 *rec = reinterpret_cast<const uint4 *>(smem + rco);
                const uint4 sc[2] = {rec[0], rec[1]}, ss[2] = {rec[2], rec[3]}, r4 = rec[4];
                const uint32_t sx[2] = {r4.x, r4.y}, sd[2] = {r4.z, r4.w};
#pragma unroll
                for (int q = 0; q < kQ; q++) {
                    const int src = 16 * (kQ * pr + q) + col;
                    const uint32_t B0 = __shfl(b.x, src), B1 = __shfl(b.y, src), B2 = __shfl(b.z, src),
                                   B3 = __shfl(b.w, src);
#pragma unroll
                    for (int ks = 0; ks < 2; ks++) {
                        const uint32_t d = sd[ks];
                        const uint32_t lo = d == 0u ? B0 : d == 1u ? B1 : B2;
                        const uint32_t hi = d == 0u ? B1 : d == 1u ? B2 : B3;
                        const uint32_t X = __builtin_amdgcn_perm(hi, lo, sx[ks]);  // the exponents' bytes
                        const uint32_t e01 = pack_bf2((float)(X & 0xFFu), (float)((X >> 8) & 0xFFu));
                        const uint32_t e2 = pack_bf2((float)((X >> 16) & 0xFFu), 0.0f);
                        xs[q][ks] = make_uint4(__builtin_amdgcn_perm(e01, sc[ks].x, ss[ks].x),
                                               __builtin_amdgcn_perm(e01, sc[ks].y, ss[ks].y),
                                               __builtin_amdgcn_perm(e01, sc[ks].z, ss[ks].z),
                                               __builtin_amdgcn_perm(e2, sc[ks].w, ss[ks].w));
                    }
                }
                f32x4_t acc[kQ][NT];
#pragma unroll
                for (int q = 0; q < kQ; q++)
#pragma unroll
                    for (int n = 0; n < NT; n++) acc[q][n] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int ks = 0; ks < 2; ks++) {
#pragma unroll
                    for (int n = 0; n < NT; n++) {
                        const uint4 fw = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w0r, w0off[ks], 2 * 16 * n * 48, 0));
#pragma unroll
                        for (int q = 0; q < kQ; q++)
                            acc[q][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(fw), as_frag(xs[q][ks]), acc[q][n], 0, 0, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int q = 0; q < kQ; q++) ln_epilogue<NT, H, false>(acc[q], act[q], sLNr, sLNr + 16 * NT, g, inv_n);
                if (a.debug && t == a.t0)
                    for (int q = 0; q < kQ; q++) debug_act<NT>(a, 0, base + kBpw * wave + 16 * (kQ * pr + q) + col, act[q], g);

                // ---------------- residual blocks ---------------------------------------------
#pragma unroll
                for (int l = 0; l < 2; l++) {
#pragma unroll
                    for (int q = 0; q < kQ; q++)
#pragma unroll
                        for (int n = 0; n < NT; n++) acc[q][n] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                    for (int ks = 0; ks < KS; ks++) {
                        uint4 bf[kQ];
#pragma unroll
                        for (int q = 0; q < kQ; q++) bf[q] = act_frag<NT>(act[q], ks);
                        const bool kok = 32 * ks + 8 * g < hp8;
                        // materialised here, per k-step (see wlane_t)
                        int kbase = l * WB + (pr_ks_swz(h, ks) ? wlane_xt : wlane_t) + 64 * ks;
                        asm volatile("" : "+v"(kbase));
#pragma unroll
                        for (int n = 0; n < NT; n++) {
#if PR_NOSEL
                            // no zero redirection: a k-step past h reads the next row's first units
                            // (or the zero gap behind the last image) against a zero B fragment (dG
                            // past h is zero: +-0 products), a row past h reads whatever follows
                            // into an output feature past h, which every epilogue masks by select
                            (void)kok;
                            const int off = kbase + 16 * n * P;
#else
                            const bool rok = n < NT - 1 || col < last_rows;
                            const int off = (kok && rok) ? kbase + 16 * n * P : zoff;
#endif
                            const uint4 fw = *reinterpret_cast<const uint4 *>(smem + off);
#pragma unroll
                            for (int q = 0; q < kQ; q++)
                                acc[q][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(fw), as_frag(bf[q]), acc[q][n], 0, 0, 0);
                        }
                        // keep the scheduler from hoisting the fragment loads of later k-steps
                        // (they would all be live at once)
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    const float *lnp = sLNr + (l + 1) * 32 * NT;
#pragma unroll
                    for (int q = 0; q < kQ; q++) ln_epilogue<NT, H, true>(acc[q], act[q], lnp, lnp + 16 * NT, g, inv_n);
                    if (a.debug && t == a.t0)
                        for (int q = 0; q < kQ; q++)
                            debug_act<NT>(a, l + 1, base + kBpw * wave + 16 * (kQ * pr + q) + col, act[q], g);
                }
                // ---------------- heads: logits of board 16 g + col land in lane (g, col) -------
#pragma unroll
                for (int q = 0; q < kQ; q++) {
                    const int bt = kQ * pr + q;
                    constexpr int kOut = 1 << 30;  // past the 5 head rows
                    const int offl = (col >> 2) == bt ? hlane_t : kOut, offv = col == 4 * bt ? hvlane : kOut;
#pragma unroll
                    for (int ks = 0; ks < KS; ks++) {
                        const uint4 bf = act_frag<NT>(act[q], ks);
                        const uint4 hl = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(hr, offl + 64 * ks, 0, 0));
                        const uint4 hv = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(hr, offv + 64 * ks, 0, 0));
                        accL = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(hl), as_frag(bf), accL, 0, 0, 0);
                        accV = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(hv), as_frag(bf), accV, 0, 0, 0);
                    }
                }
            }

            float lg[4];
#pragma unroll
            for (int r = 0; r < 4; r++) lg[r] = accL[r] + a.ba[r];
            const float val = accV[0] + a.bv[0];
            if (a.debug && t == a.t0 && live) {
                float *d = a.debug + 4 * a.n * (16 * NT) + 5 * i;
                d[0] = lg[0], d[1] = lg[1], d[2] = lg[2], d[3] = lg[3], d[4] = val;
            }

            // ---------------- sample + env step (lane = board) ----------------------------------
            const uint64_t cs = ctr0 + 2ull * (uint64_t)t;
            float lp[4], ent;
#if PR_PHPAIR
            // 32 boards per wave: the board's two Philox draws of the step on the two half-waves at
            // once -- lanes 0..31 the sampler's (counter cs, stream 1), lanes 32..63 the spawn's
            // (cs + 1, stream 0) -- the spawn words then handed down by one permlane32 swap each
            const bool upper = lane >= 32;
            const uint4 d = philox_draw(a.seed, upper ? cs + 1ull : cs, a.env_base + (uint32_t)(upper ? i - 32 : i),
                                        upper ? 0u : 1u);
            const uint32_t sp0 = __builtin_amdgcn_permlane32_swap(d.x, d.x, false, false)[1];
            const uint32_t sp1 = __builtin_amdgcn_permlane32_swap(d.y, d.y, false, false)[1];
            const uint32_t act_a = sample_row(lg, legal, d.x, lp, ent);
#if PR_CARRY
            const StepResult res = step_board_carry(b, carry, act_a, rng, i, cs + 1ull, (uint32_t)a.opts, sp0, sp1);
#else
            const StepResult res =
                step_board<G2048_RNG_PHILOX, true>(b, true, act_a, nullptr, rng, i, cs + 1ull, (uint32_t)a.opts, sp0, sp1);
#endif
#else
            const uint4 d = philox_draw(a.seed, cs, a.env_base + (uint32_t)i, 1u);
            const uint32_t act_a = sample_row(lg, legal, d.x, lp, ent);
            const StepResult res = step_board<G2048_RNG_PHILOX>(b, true, act_a, nullptr, rng, i, cs + 1ull, (uint32_t)a.opts);
#endif
            legal = res.fl & 0xFu;
            if (live) {
                const int64_t o = (int64_t)t * a.n + i;
                a.value[o] = val;
                a.actions[o] = (uint8_t)act_a;
                *reinterpret_cast<float4 *>(a.logp + 4 * o) = make_float4(lp[0], lp[1], lp[2], lp[3]);
                a.entropy[o] = ent;
                a.points[o] = (int32_t)res.pts;
                a.max_tile[o] = (int8_t)res.mx;
                a.pot[o] = res.pot;
                a.boards[o + a.n] = b;
                a.flags[o + a.n] = (uint8_t)res.fl;
            }
        }
    }
}

}  // namespace

extern "C" {

size_t g2048_policy_rollout_lds_bytes(int32_t h) {
    if (h <= 0 || h % 4 != 0) return 0;
    const int nt = (h + 15) / 16;
    const size_t b = (size_t)pr_lds_bytes(h, nt) + kPrRecBytes + kPrGap;
    return b <= (size_t)kPrLdsMax ? b : 0;
}

int g2048_policy_rollout(g2048_stream_t stream, const g2048_policy_rollout_args *p) {
    if (!p) return G2048_EINVAL;
    const int h = p->hidden;
    if (p->num_layers != 2 || h <= 0 || h % 4 != 0 || !g2048_policy_rollout_lds_bytes(h)) return G2048_EINVAL;
    if (p->n < 0 || p->n >= (int64_t(1) << 31) || p->t0 < 0 || p->t1 < p->t0) return G2048_EINVAL;
    if (p->n == 0 || p->t1 == p->t0) return G2048_OK;
    if (!p->boards || !p->flags || !p->actions || !p->logp || !p->entropy || !p->value || !p->points || !p->max_tile ||
        !p->pot || !p->w_stem || !p->w_block[0] || !p->w_block[1] || !p->head_bf16 || !p->head_bias_action ||
        !p->head_bias_value)
        return G2048_EINVAL;
    for (int l = 0; l < 3; l++)
        if (!p->ln_gamma[l] || !p->ln_beta[l]) return G2048_EINVAL;
    if (((uintptr_t)p->boards & 15u) || ((uintptr_t)p->logp & 15u) || ((uintptr_t)p->pot & 3u) ||
        ((uintptr_t)p->w_stem & 15u) || ((uintptr_t)p->w_block[0] & 7u) || ((uintptr_t)p->w_block[1] & 7u) ||
        ((uintptr_t)p->head_bf16 & 15u))
        return G2048_EINVAL;
    if (p->opts & ~(uint32_t)(G2048_OPT_AUTO_RESET | G2048_OPT_SKIP_DONE)) return G2048_EINVAL;
    PrArgs a{};
    a.boards = (uint4 *)p->boards;
    a.flags = p->flags;
    a.actions = p->actions;
    a.logp = p->logp;
    a.entropy = p->entropy;
    a.value = p->value;
    a.points = p->points;
    a.max_tile = p->max_tile;
    a.pot = (uint32_t *)p->pot;
    a.n = p->n;
    a.t0 = (int32_t)p->t0;
    a.t1 = (int32_t)p->t1;
    a.h = h;
    a.opts = (int32_t)p->opts;
    a.w0 = (const uint16_t *)p->w_stem;
    a.w1 = (const uint16_t *)p->w_block[0];
    a.w2 = (const uint16_t *)p->w_block[1];
    for (int l = 0; l < 3; l++) {
        a.gamma[l] = p->ln_gamma[l];
        a.beta[l] = p->ln_beta[l];
    }
    a.head = (const uint16_t *)p->head_bf16;
    a.ba = p->head_bias_action;
    a.bv = p->head_bias_value;
    a.seed = p->seed;
    a.counter_dev = p->counter_dev;
    a.counter = p->counter;
    a.env_base = p->env_base;
    a.debug = p->debug;
    const int nt = (h + 15) / 16;
    const size_t lds = g2048_policy_rollout_lds_bytes(h);
    const int64_t groups = (p->n + kPrBoards - 1) / kPrBoards;
    const unsigned grid = (unsigned)(groups < 256 ? groups : 256);
    hipStream_t s = (hipStream_t)stream;
    (void)nt;
    switch (h) {
    case 196: hipLaunchKernelGGL((policy_rollout_kernel<196>), dim3(grid), dim3(kPrThreads), lds, s, a); break;
    case 192: hipLaunchKernelGGL((policy_rollout_kernel<192>), dim3(grid), dim3(kPrThreads), lds, s, a); break;
    case 128: hipLaunchKernelGGL((policy_rollout_kernel<128>), dim3(grid), dim3(kPrThreads), lds, s, a); break;
    case 64: hipLaunchKernelGGL((policy_rollout_kernel<64>), dim3(grid), dim3(kPrThreads), lds, s, a); break;
    case 32: hipLaunchKernelGGL((policy_rollout_kernel<32>), dim3(grid), dim3(kPrThreads), lds, s, a); break;
    default: return G2048_EINVAL;
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}

int g2048_policy_rollout_supported(int32_t hidden, int32_t num_layers) {
    if (num_layers != 2 || !g2048_policy_rollout_lds_bytes(hidden)) return 0;
    return hidden == 196 || hidden == 192 || hidden == 128 || hidden == 64 || hidden == 32;
}

}  // extern "C"
