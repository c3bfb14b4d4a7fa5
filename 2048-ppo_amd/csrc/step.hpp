// step.hpp -- Game2048.step on a board held in registers (game.py:952-1030), shared by the env
// kernels (g2048.hip) and the fused policy rollout (policy_rollout.hip): flag bits, RNG arguments,
// spawn / reset and the step itself, for the Philox, MT19937-parity and injected-draw RNG modes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "board.hpp"
#include "../../include/g2048.h"

namespace g2048 {
namespace {

enum : uint32_t { FLAG_INVALID = 0x10u, FLAG_RESET = 0x20u, FLAG_INACTIVE = 0x40u, FLAG_DONE = 0x80u };

struct RngArgs {
    uint64_t seed;
    uint64_t counter;
    const uint64_t *counter_dev;
    uint32_t env_base;
    uint32_t *mt;
    const int32_t *inject;
};

__device__ __forceinline__ uint64_t rng_counter(const RngArgs &r) {
    return r.counter + (r.counter_dev ? *r.counter_dev : 0ull);
}

// One spawn on `b` (game.py:923-940).  `slot` selects which pair of the Philox block is used, so a
// reset's two spawns come from one 4-word draw.
template <int Mode>
__device__ __forceinline__ void spawn(uint4 &b, uint32_t u0, uint32_t u1, MT *mt, const RngArgs &r, int64_t i) {
    const uint32_t em = empty_mask16(b);
    const uint32_t cnt = __popc(em);
    if (cnt == 0u) return;
    uint32_t k, v;
    if constexpr (Mode == G2048_RNG_PHILOX) {
        k = (uint32_t)(((uint64_t)u0 * cnt) >> 32);
        v = u1 < kTwoThreshold ? 1u : 2u;
    } else if constexpr (Mode == G2048_RNG_MT19937) {
        k = mt->randbelow(cnt);
        v = mt->below_09() ? 1u : 2u;
    } else {
        k = (uint32_t)r.inject[2 * i];
        v = (uint32_t)r.inject[2 * i + 1];
        k = k < cnt ? k : cnt - 1u;
    }
    set_cell(b, kth_bit16(em, k), v);
}

template <int Mode>
__device__ __forceinline__ uint4 fresh_board(MT *mt, const RngArgs &r, int64_t i, uint64_t ctr) {
    uint4 b = make_uint4(0u, 0u, 0u, 0u);
    uint4 ph = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (Mode == G2048_RNG_PHILOX) ph = philox_draw(r.seed, ctr, r.env_base + (uint32_t)i, 2u);
    spawn<Mode>(b, ph.x, ph.y, mt, r, i);
    spawn<Mode>(b, ph.z, ph.w, mt, r, i);
    return b;
}

struct StepResult {
    uint32_t action, pts, mx, pot, fl;
};

// Game2048.step (game.py:952-1030) on a board held in registers.  has_action == false draws the
// uniform random legal action of the synthetic benchmark policy (Philox stream 1).  kPre: the
// policy-action spawn draw (stream 0 at ctr, words x / y) was made by the caller (pre0, pre1).
template <int Mode, bool kPre = false>
__device__ __forceinline__ StepResult step_board(uint4 &b, bool has_action, uint32_t action_in, MT *mt,
                                                 const RngArgs &rng, int64_t i, uint64_t ctr, uint32_t opts,
                                                 uint32_t pre0 = 0u, uint32_t pre1 = 0u) {
    StepResult res{0u, 0u, 0u, 0u, 0u};
    const uint32_t env = rng.env_base + (uint32_t)i;
    uint32_t legal_in = 0u;
    const bool need_legal = !has_action || (opts & G2048_OPT_SKIP_DONE);
    if (need_legal) legal_in = legal_mask(b);
    if ((opts & G2048_OPT_SKIP_DONE) && legal_in == 0u) {  // episodic mode: this game is already over
        res.action = 0xFFu;
        res.fl = FLAG_INACTIVE | FLAG_DONE;
        return res;
    }
    uint32_t a;
    uint32_t su0 = 0u, su1 = 0u;  // spawn words: one Philox draw per step when the action is drawn here
    if (has_action) {
        a = action_in & 3u;
    } else {
        const uint4 d = philox_draw(rng.seed, ctr, env, 1u);
        const uint32_t nl = __popc(legal_in);
        a = nl ? kth_bit16(legal_in, (uint32_t)(((uint64_t)d.x * nl) >> 32)) : 0u;  // k-th legal action
        su0 = d.y;
        su1 = d.z;
    }
    res.action = a;
    const int mono_b = monotonicity(b);
    const int empt_b = emptiness(b);
    uint32_t pts, mx;
    uint4 moved = apply_move(b, a, pts, mx);
    if (eq4(moved, b)) {
        // illegal action: no-op, zero points and potentials, done = no legal move (game.py:959-978)
        if (!need_legal) legal_in = legal_mask(b);
        res.fl = FLAG_INVALID | legal_in | (legal_in ? 0u : FLAG_DONE);
    } else {
        const int mono_a = monotonicity(moved);
        const int empt_a = emptiness(moved);
        res.pot = (uint32_t)(mono_b & 0xFF) | ((uint32_t)(mono_a & 0xFF) << 8) | ((uint32_t)(empt_b & 0xFF) << 16) |
                  ((uint32_t)(empt_a & 0xFF) << 24);
        res.pts = pts;
        res.mx = mx;
        if constexpr (Mode == G2048_RNG_PHILOX) {
            if (has_action) {  // policy actions: spawn draw from stream 0
                if constexpr (kPre) {
                    su0 = pre0;
                    su1 = pre1;
                } else {
                    const uint4 ph = philox_draw(rng.seed, ctr, env, 0u);
                    su0 = ph.x;
                    su1 = ph.y;
                }
            }
        }
        spawn<Mode>(moved, su0, su1, mt, rng, i);
        b = moved;
        const uint32_t lm = legal_mask(b);
        res.fl = lm | (lm ? 0u : FLAG_DONE);
    }
    if ((res.fl & FLAG_DONE) && (opts & G2048_OPT_AUTO_RESET)) {
        b = fresh_board<Mode>(mt, rng, i, ctr);
        res.fl = (res.fl & ~0xFu) | FLAG_RESET | legal_mask(b);
    }
    return res;
}

// The fused policy rollout's step: step_board<PHILOX, true> with a policy action, bitwise its results
// and board, with the board's monotonicity statistics and emptiness carried from step to step
// (round 5) instead of recomputed from the board: the post-spawn board's statistics come from the
// pre-spawn board's (computed anyway for mono_a) by mono_add_tile -- env_rollout_kernel's rule --,
// its emptiness is empt_a - 1, and a reset board's are computed afresh.  The carry is one packed
// word (bits 0..3 pos, 8..11 L, 12..15 R, 16..19 T, 20..23 B, 24..31 M) and the emptiness.
__device__ __forceinline__ uint32_t carry_pack(const MonoStats &s) {
    return s.pos | ((uint32_t)s.L << 8) | ((uint32_t)s.R << 12) | ((uint32_t)s.T << 16) | ((uint32_t)s.B << 20) |
           (s.M << 24);
}
__device__ __forceinline__ MonoStats carry_unpack(uint32_t w) {
    return MonoStats{(int)((w >> 8) & 15u), (int)((w >> 12) & 15u), (int)((w >> 16) & 15u), (int)((w >> 20) & 15u),
                     w >> 24, w & 15u};
}
struct BoardCarry {
    uint32_t s;  // carry_pack(mono_stats(b))
    int empt;    // emptiness(b)
};
__device__ __forceinline__ BoardCarry board_carry(const uint4 &b) { return BoardCarry{carry_pack(mono_stats(b)), emptiness(b)}; }

__device__ __forceinline__ StepResult step_board_carry(uint4 &b, BoardCarry &cy, uint32_t action_in, const RngArgs &rng,
                                                       int64_t i, uint64_t ctr, uint32_t opts, uint32_t pre0,
                                                       uint32_t pre1) {
    StepResult res{0u, 0u, 0u, 0u, 0u};
    const bool need_legal = (opts & G2048_OPT_SKIP_DONE) != 0u;
    uint32_t legal_in = need_legal ? legal_mask(b) : 0u;
    if (need_legal && legal_in == 0u) {  // episodic mode: this game is already over
        res.action = 0xFFu;
        res.fl = FLAG_INACTIVE | FLAG_DONE;
        return res;
    }
    const uint32_t a = action_in & 3u;
    res.action = a;
    const int mono_b = mono_value(carry_unpack(cy.s));
    const int empt_b = cy.empt;
    uint32_t pts, mx;
    uint4 moved = apply_move(b, a, pts, mx);
    if (eq4(moved, b)) {  // illegal action: board and carry unchanged
        if (!need_legal) legal_in = legal_mask(b);
        res.fl = FLAG_INVALID | legal_in | (legal_in ? 0u : FLAG_DONE);
    } else {
        const MonoStats sa = mono_stats(moved);
        const int mono_a = mono_value(sa);
        const int empt_a = emptiness(moved);
        res.pot = (uint32_t)(mono_b & 0xFF) | ((uint32_t)(mono_a & 0xFF) << 8) | ((uint32_t)(empt_b & 0xFF) << 16) |
                  ((uint32_t)(empt_a & 0xFF) << 24);
        res.pts = pts;
        res.mx = mx;
        // spawn<PHILOX> on the caller's stream-0 words, with its cell and value kept for the carry
        const uint32_t em = empty_mask16(moved);
        const uint32_t cnt = __popc(em);
        MonoStats sn = sa;
        int en = empt_a;
        if (cnt != 0u) {
            const uint32_t k = (uint32_t)(((uint64_t)pre0 * cnt) >> 32);
            const uint32_t v = pre1 < kTwoThreshold ? 1u : 2u;
            const uint32_t p = kth_bit16(em, k);
            sn = mono_add_tile(sa, moved, p, v);
            set_cell(moved, p, v);
            en = empt_a - 1;
        }
        b = moved;
        cy = BoardCarry{carry_pack(sn), en};
        const uint32_t lm = legal_mask(b);
        res.fl = lm | (lm ? 0u : FLAG_DONE);
    }
    if ((res.fl & FLAG_DONE) && (opts & G2048_OPT_AUTO_RESET)) {
        b = fresh_board<G2048_RNG_PHILOX>(nullptr, rng, i, ctr);
        res.fl = (res.fl & ~0xFu) | FLAG_RESET | legal_mask(b);
        cy = board_carry(b);
    }
    return res;
}

}  // namespace
}  // namespace g2048
