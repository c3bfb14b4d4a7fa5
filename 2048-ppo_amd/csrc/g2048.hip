// g2048.hip -- libg2048.so: HIP kernels for gfx950 + the C ABI declared in include/g2048.h.
//
// Kernels (one lane = one env unless stated):
//   env_step_kernel<Rng>   Game2048.step (game.py:952-1030), optional random-legal action and
//                          auto-reset / skip-done.  The hot kernel: 16-B board load, ~40 B out.
//   env_reset_kernel<Rng>  Game2048.reset (game.py:942-950)
//   legal_kernel           current_valid_directions (game.py:295-299)
//   obs_kernel<T>          to_model_format (game.py:92-101); one lane per 4 output values so the
//                          [N,48] stores are contiguous per wave
//   sample_kernel          masked softmax / sample / entropy / log_softmax (train.py:266-326)
//   rtg_kernel             reward + reverse discounted scan + normalisation + advantage
//                          (train.py:699-772), time-major [T][N], float64 arithmetic
//   rtg_reduce / prepare / finalize   batch moments and the EMA update (train.py:731-754, 898-901)
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "board.hpp"
#include "rowtable.hpp"
#include "step.hpp"
#include "launch_util.hpp"
#include "../../include/g2048.h"

using namespace g2048;

namespace {

constexpr int kBlock = 256;

template <int Mode>
__global__ __launch_bounds__(kBlock) void env_step_kernel(const uint4 *__restrict__ bin, uint4 *__restrict__ bout,
                                                          const uint8_t *__restrict__ ain, uint8_t *__restrict__ aout,
                                                          int32_t *__restrict__ points, int8_t *__restrict__ maxt,
                                                          uint32_t *__restrict__ pot, uint8_t *__restrict__ flags,
                                                          int64_t n, RngArgs rng, uint32_t opts) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    uint4 b = bin[i];
    MT mt;
    if constexpr (Mode == G2048_RNG_MT19937) mt.load(rng.mt, n, i);
    const StepResult r = step_board<Mode>(b, ain != nullptr, ain ? ain[i] : 0u, &mt, rng, i, rng_counter(rng), opts);
    if constexpr (Mode == G2048_RNG_MT19937) mt.save();
    bout[i] = b;
    points[i] = (int32_t)r.pts;
    if (maxt) maxt[i] = (int8_t)r.mx;
    if (pot) pot[i] = r.pot;
    if (aout) aout[i] = (uint8_t)r.action;
    flags[i] = (uint8_t)r.fl;
}

template <int Mode>
__global__ __launch_bounds__(kBlock) void env_reset_kernel(uint4 *__restrict__ boards, uint8_t *__restrict__ flags,
                                                           const uint8_t *__restrict__ where, int64_t n, RngArgs rng) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (where && !where[i]) return;
    MT mt;
    if constexpr (Mode == G2048_RNG_MT19937) mt.load(rng.mt, n, i);
    const uint4 b = fresh_board<Mode>(&mt, rng, i, rng_counter(rng));
    if constexpr (Mode == G2048_RNG_MT19937) mt.save();
    boards[i] = b;
    if (flags) flags[i] = (uint8_t)legal_mask(b);
}

// preview_move_rewards (game.py:167-184): merge points of each direction, 0 where illegal.
__global__ __launch_bounds__(kBlock) void preview_kernel(const uint4 *__restrict__ boards, int4 *__restrict__ out,
                                                         int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint4 b = boards[i];
    int r[4];
#pragma unroll
    for (uint32_t a = 0; a < 4u; a++) {
        uint32_t pts, mx;
        const uint4 m = apply_move(b, a, pts, mx);
        r[a] = eq4(m, b) ? 0 : (int)pts;
    }
    out[i] = make_int4(r[0], r[1], r[2], r[3]);
}

__global__ __launch_bounds__(kBlock) void legal_kernel(const uint4 *__restrict__ boards, uint8_t *__restrict__ flags,
                                                       int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t m = legal_mask(boards[i]);
    flags[i] = (uint8_t)(m | (m ? 0u : FLAG_DONE));
}

// CPython random.seed(int) == init_by_array over the 32-bit words of the seed.
__global__ __launch_bounds__(kBlock) void mt_seed_kernel(uint32_t *__restrict__ st, const uint64_t *__restrict__ seeds,
                                                         int64_t n) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    auto W = [&](int k) -> uint32_t & { return st[(int64_t)k * n + e]; };
    const uint64_t s = seeds[e];
    const uint32_t key[2] = {(uint32_t)s, (uint32_t)(s >> 32)};
    const int klen = key[1] ? 2 : 1;
    W(0) = 19650218u;
    for (int k = 1; k < 624; k++) W(k) = 1812433253u * (W(k - 1) ^ (W(k - 1) >> 30)) + (uint32_t)k;
    int i = 1, j = 0;
    for (int k = 624; k; k--) {
        W(i) = (W(i) ^ ((W(i - 1) ^ (W(i - 1) >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= 624) { W(0) = W(623); i = 1; }
        if (j >= klen) j = 0;
    }
    for (int k = 623; k; k--) {
        W(i) = (W(i) ^ ((W(i - 1) ^ (W(i - 1) >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= 624) { W(0) = W(623); i = 1; }
    }
    W(0) = 0x80000000u;
    W(624) = 624u;
}

// to_model_format: value f = 3*cell + k of board i is (e, row/3, col/3)[k].  Lane = 4 values.
__constant__ float kThirds[4] = {0.0f, 1.0f / 3.0f, 2.0f / 3.0f, 1.0f};

template <typename T>
__device__ __forceinline__ T cvt(float x);
template <>
__device__ __forceinline__ float cvt<float>(float x) { return x; }
template <>
__device__ __forceinline__ __hip_bfloat16 cvt<__hip_bfloat16>(float x) { return __float2bfloat16(x); }

template <typename T>
__global__ __launch_bounds__(kBlock) void obs_kernel(const int8_t *__restrict__ boards, T *__restrict__ obs, int64_t n) {
    const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // chunk of 4 values
    if (q >= n * 12) return;
    const int64_t i = q / 12;
    const int f0 = (int)(q - i * 12) * 4;
    T v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int f = f0 + u, cell = f / 3, k = f - cell * 3;
        const float x = k == 0 ? (float)boards[i * 16 + cell] : kThirds[k == 1 ? (cell >> 2) : (cell & 3)];
        v[u] = cvt<T>(x);
    }
    T *dst = obs + q * 4;
#pragma unroll
    for (int u = 0; u < 4; u++) dst[u] = v[u];
}

__global__ __launch_bounds__(kBlock) void sample_kernel(const float *__restrict__ logits, int64_t stride,
                                                        const uint8_t *__restrict__ flags, uint8_t *__restrict__ actions,
                                                        float *__restrict__ logp, float *__restrict__ entropy, int64_t n,
                                                        RngArgs rng) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t legal = flags[i] & 0xFu;
    const uint4 d = philox_draw(rng.seed, rng_counter(rng), rng.env_base + (uint32_t)i, 1u);
    float l[4];
#pragma unroll
    for (int a = 0; a < 4; a++) l[a] = logits ? logits[i * stride + a] : 0.0f;
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
    const float u = (float)(d.x >> 8) * (1.0f / 16777216.0f);
    float cum = 0.0f, h = 0.0f;
    uint32_t act = 0xFFu;
#pragma unroll
    for (int a = 0; a < 4; a++) {
        const bool ok = (legal >> a) & 1u;
        const float p = e[a] * inv, lp = (l[a] - m) - ls;
        if (ok) {
            cum += p;
            if (act == 0xFFu && u < cum) act = (uint32_t)a;
            if (p > 0.0f) h -= p * lp;
        }
        if (logp) logp[i * 4 + a] = ok ? lp : -INFINITY;
    }
    if (act == 0xFFu) {  // rounding left u >= cum: take the last legal action
#pragma unroll
        for (int a = 0; a < 4; a++)
            if ((legal >> a) & 1u) act = (uint32_t)a;
        if (!legal) act = 0u;
    }
    actions[i] = (uint8_t)act;
    if (entropy) entropy[i] = legal ? h : 0.0f;
}

// ---------------------------------------------------------------- info heuristics ----------
// The info-only heuristics Game2048.step computes around every move (game.py:981-1002): smoothness
// (:339-357), corner bonus (:359-399), adjacency bonus (:401-442), monotonic chain (:444-506, a DFS
// with a visited set), topological score with the pre-move anchor corner (:610-668, :802-921),
// before the move and after it (pre-spawn).  They never reach the reward (train.py:702-719) but
// fill the EpisodeData records, the episode breakdown tables and the viz export.  float64 in the
// reference's operation order (this file is built -ffp-contract=off): bit-identical deltas.
namespace info {
__device__ __forceinline__ int at(const int8_t *b, int i, int j) { return b[4 * i + j]; }
__device__ __forceinline__ int bmax(const int8_t *b) {
    int m = 0;
    for (int p = 0; p < 16; p++) m = b[p] > m ? b[p] : m;
    return m;
}
__device__ double smoothness(const int8_t *b) {
    double s = 0.0;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            const int x = at(b, i, j);
            if (x == 0) continue;
            if (j < 3 && at(b, i, j + 1) != 0) s -= abs(x - at(b, i, j + 1));
            if (i < 3 && at(b, i + 1, j) != 0) s -= abs(x - at(b, i + 1, j));
        }
    return s;
}
__device__ double corner(const int8_t *b) {
    const int m = bmax(b);
    if (m == 0) return 0.0;
    return (b[0] == m || b[3] == m || b[12] == m || b[15] == m) ? (double)m : -(double)m;
}
__device__ double adjacency(const int8_t *b) {
    int m = 0, mi = 0, mj = 0;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            if (at(b, i, j) > m) m = at(b, i, j), mi = i, mj = j;
    double bonus = 0.0;
    const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
    for (int d = 0; d < 4; d++) {
        const int ni = mi + di[d], nj = mj + dj[d];
        if (ni >= 0 && ni < 4 && nj >= 0 && nj < 4 && at(b, ni, nj) > 0) bonus += at(b, ni, nj) * 0.5;
    }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            const int x = at(b, i, j);
            if (x < 5) continue;
            if (j < 3 && at(b, i, j + 1) >= 5) bonus += (x + at(b, i, j + 1)) * 0.25;
            if (i < 3 && at(b, i + 1, j) >= 5) bonus += (x + at(b, i + 1, j)) * 0.25;
        }
    return bonus;
}
// the best chain from cell p: cells of values m, m-1, m-2, ... along orthogonal steps without
// revisiting, score = sum of the values; an explicit stack replaces the reference's recursion
// (depth <= 18: the value drops by one per step and 0 matches only as the last cell)
__device__ double chain_from(const int8_t *b, int p0, int m) {
    int cell[20], dir[20];
    uint32_t visited = 1u << p0;
    double sum[20], best[20];
    int depth = 0;
    cell[0] = p0, dir[0] = 0, sum[0] = (double)m, best[0] = 0.0;
    const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
    for (;;) {
        if (dir[depth] < 4) {
            const int d = dir[depth]++;
            const int i = cell[depth] / 4 + di[d], j = cell[depth] % 4 + dj[d];
            const int expected = m - 1 - depth;
            if (i < 0 || i > 3 || j < 0 || j > 3) continue;
            const int q = 4 * i + j;
            if ((visited >> q) & 1u) continue;
            if (b[q] != expected || depth + 1 >= 20) continue;
            visited |= 1u << q;
            depth++;
            cell[depth] = q, dir[depth] = 0, sum[depth] = (double)expected, best[depth] = 0.0;
        } else {  // all children tried: this node's chain = its value + the best child chain
            const double c = sum[depth] + best[depth];
            visited &= ~(1u << cell[depth]);
            if (depth == 0) return c;
            depth--;
            if (c > best[depth]) best[depth] = c;
        }
    }
}
__device__ double chain(const int8_t *b) {
    const int m = bmax(b);
    if (m == 0) return 0.0;
    double best = 0.0;
    for (int p = 0; p < 16; p++)
        if (b[p] == m) {
            const double c = chain_from(b, p, m);
            if (c > best) best = c;
        }
    return best;
}
__device__ int anchor(const int8_t *b) {  // the corner (packed 4 row + col) holding or nearest the max
    const int corners[4] = {0, 3, 12, 15};
    int m = 0, first = -1;
    uint32_t maxpos = 0;
    for (int p = 0; p < 16; p++) {
        if (b[p] > m) m = b[p], maxpos = 1u << p, first = p;
        else if (b[p] == m && m > 0) maxpos |= 1u << p;
    }
    if (first < 0) return 0;
    for (int p = 0; p < 16; p++)
        if ((maxpos >> p) & 1u)
            for (int c = 0; c < 4; c++)
                if (corners[c] == p) return p;
    const int ti = first / 4, tj = first % 4;
    int best = corners[0], bd = 1 << 30;
    for (int c = 0; c < 4; c++) {
        const int d = abs(corners[c] / 4 - ti) + abs(corners[c] % 4 - tj);
        if (d < bd) bd = d, best = corners[c];
    }
    return best;
}
__device__ double topological(const int8_t *b, int corner_p) {
    const int m = bmax(b);
    if (m == 0) return 0.0;
    int order[16], idx_of[16];
    const int cr = corner_p / 4, cc = corner_p % 4, rd = cr == 0 ? 1 : -1, cd = cc == 0 ? 1 : -1;
    for (int i = 0, k = 0; i < 4; i++)
        for (int s = 0; s < 4; s++, k++) order[k] = 4 * (cr + i * rd) + ((i % 2 == 0) ? cc + s * cd : cc + (3 - s) * cd);
    for (int k = 0; k < 16; k++) idx_of[order[k]] = k;
    double score = 0.0;
    for (int p = 0; p < 16; p++)
        if (b[p] > 0) score += (double)((16 - idx_of[p]) * b[p]) * 0.1;
    double prev = INFINITY, mono = 0.0, inv = 0.0;
    for (int k = 0; k < 16; k++) {
        const int v = b[order[k]];
        if (v == 0) continue;
        if ((double)v <= prev) mono += v * 0.2;
        else inv += ((double)v - prev) * 0.5;
        prev = (double)v;
    }
    score += mono - inv;
    if (b[corner_p] == m) score += m * 2.0;
    const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
    for (int p = 0; p < 16; p++) {
        const int v = b[p];
        if (v < 4) continue;
        int lower = 0, tot = 0;
        const int i = p / 4, j = p % 4;
        for (int d = 0; d < 4; d++) {
            const int ni = i + di[d], nj = j + dj[d];
            if (ni >= 0 && ni < 4 && nj >= 0 && nj < 4 && at(b, ni, nj) > 0) {
                tot++;
                if (at(b, ni, nj) < v - 2) lower++;
            }
        }
        if (tot >= 2 && lower >= tot - 1 && idx_of[p] > 4) score -= v * 1.0;
    }
    return score;
}
}  // namespace info

// out[i] = {smoothness, corner, adjacency, chain, topological} deltas of action a[i] on board i
// (zeros for an illegal action: game.py:959-978 returns no deltas), anchor[i] = the anchor corner.
__global__ __launch_bounds__(kBlock) void info_kernel(const uint4 *__restrict__ boards, const uint8_t *__restrict__ acts,
                                                      double *__restrict__ out, int8_t *__restrict__ anchor_out,
                                                      int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint4 w = boards[i];
    uint32_t pts, mx;
    const uint4 mw = apply_move(w, acts[i] & 3u, pts, mx);
    double d[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    int anc = 0;
    if (!eq4(mw, w)) {
        int8_t b[16], m[16];
        const uint32_t bw[4] = {w.x, w.y, w.z, w.w}, mm[4] = {mw.x, mw.y, mw.z, mw.w};
        for (int r = 0; r < 4; r++)
            for (int c = 0; c < 4; c++) {
                b[4 * r + c] = (int8_t)((bw[r] >> (8 * c)) & 0xFFu);
                m[4 * r + c] = (int8_t)((mm[r] >> (8 * c)) & 0xFFu);
            }
        anc = info::anchor(b);
        d[0] = info::smoothness(m) - info::smoothness(b);
        d[1] = info::corner(m) - info::corner(b);
        d[2] = info::adjacency(m) - info::adjacency(b);
        d[3] = info::chain(m) - info::chain(b);
        d[4] = info::topological(m, anc) - info::topological(b, anc);
    }
    for (int k = 0; k < 5; k++) out[5 * i + k] = d[k];
    if (anchor_out) anchor_out[i] = (int8_t)anc;
}

// ---------------------------------------------------------------- reward / return-to-go ------
struct RewardArgs {
    double gamma, wp, wm, we;
};

template <int NW>
__device__ __forceinline__ double block_sum(double v, double *sh) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) sh[w] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int k = 0; k < NW; k++) t += sh[k];
    return t;  // valid on thread 0
}

// One lane per env walks t = T-1 .. 0.  The recurrence is serial, but its inputs are not: the loads
// of kRtgU consecutive steps are issued together before the arithmetic of that group, so a lane
// waits for one memory round trip per kRtgU steps instead of one per step (at 65 536 envs there
// is one wave per SIMD and nothing else hides the latency).
constexpr int kRtgU = 16;

__global__ __launch_bounds__(kBlock) void rtg_kernel(const int32_t *__restrict__ points, const uint32_t *__restrict__ pot,
                                                     const uint8_t *__restrict__ flags, const float *__restrict__ value,
                                                     int64_t T, int64_t n, RewardArgs ra, const double *__restrict__ state,
                                                     float *__restrict__ g_raw, float *__restrict__ g_norm,
                                                     float *__restrict__ adv, double *__restrict__ reward,
                                                     double *__restrict__ partial) {
    __shared__ double sh[kBlock / 64];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const double mu_c = state[4], inv = 1.0 / (state[5] + 1e-8);
    double s1 = 0.0, s2 = 0.0, cnt = 0.0;
    if (i < n) {
        double G = 0.0;
        for (int64_t t1 = T; t1 > 0; t1 -= kRtgU) {
            const int64_t t0 = t1 - kRtgU > 0 ? t1 - kRtgU : 0;
            int32_t P[kRtgU];
            uint32_t W[kRtgU], F[kRtgU];
            float V[kRtgU];
#pragma unroll
            for (int u = 0; u < kRtgU; u++) {
                const int64_t t = t1 - 1 - u;
                if (t >= t0) {
                    const int64_t o = t * n + i;
                    P[u] = points[o];
                    W[u] = pot[o];
                    F[u] = flags[o];
                    V[u] = value[o];
                }
            }
#pragma unroll
            for (int u = 0; u < kRtgU; u++) {
                const int64_t t = t1 - 1 - u;
                if (t < t0) break;
                const int64_t o = t * n + i;
                const uint32_t fl = F[u];
                if (fl & FLAG_INACTIVE) {
                    G = 0.0;
                    g_raw[o] = 0.0f;
                    g_norm[o] = 0.0f;
                    adv[o] = 0.0f;
                    if (reward) reward[o] = 0.0;
                    continue;
                }
                const uint32_t pw = W[u];
                const bool done = (fl & FLAG_DONE) != 0u;
                const double mb = (double)(int8_t)(pw & 0xFFu), ma = done ? 0.0 : (double)(int8_t)((pw >> 8) & 0xFFu);
                const double eb = (double)(int8_t)((pw >> 16) & 0xFFu), ea = done ? 0.0 : (double)(int8_t)(pw >> 24);
                // same operation order as train.py:702-719 (float64, no contraction: built -ffp-contract=off)
                double shaped = ra.wm * (ra.gamma * ma - mb);
                shaped = shaped + ra.we * (ra.gamma * ea - eb);
                const double r = (double)P[u] * ra.wp + shaped;
                if (done) G = 0.0;  // the episode ended on this step: nothing flows back across it
                G = r + ra.gamma * G;
                const double gn = (G - mu_c) * inv;  // train.py:751 divides; the reciprocal is within 1 ulp
                g_raw[o] = (float)G;
                g_norm[o] = (float)gn;
                adv[o] = (float)(gn - (double)V[u]);
                if (reward) reward[o] = r;
                const double dv = G - mu_c;
                s1 += dv;
                s2 += dv * dv;
                cnt += 1.0;
            }
        }
    }
    const double b1 = block_sum<kBlock / 64>(s1, sh);
    const double b2 = block_sum<kBlock / 64>(s2, sh);
    const double b3 = block_sum<kBlock / 64>(cnt, sh);
    if (threadIdx.x == 0) {
        partial[3 * blockIdx.x + 0] = b1;
        partial[3 * blockIdx.x + 1] = b2;
        partial[3 * blockIdx.x + 2] = b3;
    }
}

__global__ __launch_bounds__(kBlock) void rtg_reduce_kernel(const double *__restrict__ part, int nb, double *__restrict__ out) {
    __shared__ double sh[kBlock / 64];
    double a = 0.0, b = 0.0, c = 0.0;
    for (int k = threadIdx.x; k < nb; k += kBlock) {
        a += part[3 * k];
        b += part[3 * k + 1];
        c += part[3 * k + 2];
    }
    a = block_sum<kBlock / 64>(a, sh);
    b = block_sum<kBlock / 64>(b, sh);
    c = block_sum<kBlock / 64>(c, sh);
    if (threadIdx.x == 0) {
        out[0] = a;
        out[1] = b;
        out[2] = c;
    }
}

__global__ void rtg_prepare_kernel(double *state, double beta) {
    const double eps = 1e-8;
    const double step = state[3] < 1.0 ? 1.0 : state[3];
    const double bc = fmax(1.0 - pow(beta, step), eps);  // train.py:746
    const double mu_c = state[0] / bc, m2_c = state[1] / bc;
    state[4] = mu_c;
    state[5] = sqrt(fmax(m2_c - mu_c * mu_c, eps));
}

__global__ void rtg_finalize_kernel(double *state, const double *part, double beta) {
    const double n = part[2];
    if (n <= 0.0) return;
    const double m1 = part[0] / n;
    const double mean = state[4] + m1;
    const double var = n <= 1.0 ? 0.0 : fmax(part[1] / n - m1 * m1, 0.0);
    state[6] = mean;
    state[7] = var;
    const double mu = beta * state[0] + (1.0 - beta) * mean;       // train.py:900
    state[1] = beta * state[1] + (1.0 - beta) * (var + mean * mean);  // train.py:899
    state[0] = mu;
    state[2] = mu;  // train.py:901
    state[3] = state[3] + 1.0;
}


// Episode bookkeeping of a fixed-horizon rollout (the score / max-tile statistics of
// compute_batch_stats, train.py:1040-1120): per env, walk t = 0..T-1 carrying the running score and
// max tile of the current game across rollouts; where step t ends a game, emit (score, max tile
// exponent), else -1.  One thread per env, time-major reads.
__global__ __launch_bounds__(kBlock) void episode_scan_kernel(const int32_t *__restrict__ points,
                                                              const uint4 *__restrict__ boards,
                                                              const int8_t *__restrict__ max_tile,
                                                              const uint8_t *__restrict__ step_flags, int64_t T,
                                                              int64_t n, int64_t *__restrict__ run_score,
                                                              int32_t *__restrict__ run_max,
                                                              int64_t *__restrict__ scores, int32_t *__restrict__ tiles) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    int64_t rs = run_score[e];
    int32_t rm = run_max[e];
    for (int64_t t = 0; t < T; t++) {
        const int64_t k = t * n + e;
        rs += points[k];
        uint4 b = boards[k];
        uint32_t m = bytemax(bytemax(b.x, b.y), bytemax(b.z, b.w));
        m = bytemax(m, m >> 8);
        m = bytemax(m, m >> 16);
        rm = max(rm, max((int32_t)(m & 0xFFu), (int32_t)max_tile[k]));
        const uint8_t f = step_flags[k];
        const bool done = (f & FLAG_DONE) && !(f & FLAG_INACTIVE);
        scores[k] = done ? rs : -1;
        tiles[k] = done ? rm : -1;
        if (done) {
            rs = 0;
            rm = 0;
        }
    }
    run_score[e] = rs;
    run_max[e] = rm;
}

// ------------------------------------------------------------------ rollout statistics ------
// The rollout half of the train step's metrics (the reward / advantage / return summaries and
// compute_batch_stats' finished-game statistics, train.py:1040-1120 and :1700-1760) in two launches
// instead of ~60 torch ops: rollout_stats_kernel walks each env's T steps once (the episode scan
// of episode_scan_kernel plus every row statistic, float64 per-thread sums, a fixed-order block
// reduction into per-block partials; finished scores are appended to a key list at a range each
// block reserves with one atomic), rollout_stats_final_kernel sums the partials in block order and finds the lower median
// of the finished scores by a three-pass radix select.  Deterministic: the atomics only decide
// the order of the key list, which the selection does not see.
namespace rstat {
enum : int { N, R, R2, RZ, A, A2, GN, GN2, GR, GR2, V, V2, G0, G0N, CNT, SSUM, T9, T10, T11, AMIN, AMAX, GNMIN,
             GNMAX, SMAX, K };
constexpr size_t kHead = 256;  // the key counter, then the partials, then the keys
__device__ __forceinline__ bool is_min(int j) { return j == AMIN || j == GNMIN; }
__device__ __forceinline__ bool is_max(int j) { return j == AMAX || j == GNMAX || j == SMAX; }
__device__ __forceinline__ double combine(int j, double a, double b) {
    return is_min(j) ? fmin(a, b) : is_max(j) ? fmax(a, b) : a + b;
}
}  // namespace rstat

// kEpi: episodic mode.  The walk is latency-bound at one wave per SIMD (n / 64 waves), so the
// loads of kChunk steps are issued before any of them is used.
template <bool kEpi>
__global__ __launch_bounds__(kBlock) void rollout_stats_kernel(
    const int32_t *__restrict__ points, const uint32_t *__restrict__ pot, const uint8_t *__restrict__ sf,
    const float *__restrict__ value, const float *__restrict__ g_raw, const float *__restrict__ g_norm,
    const float *__restrict__ adv, const uint4 *__restrict__ boards, const int8_t *__restrict__ max_tile, int64_t T,
    int64_t n, float wp, float wm, float we, float gamma, int64_t *__restrict__ run_score,
    int32_t *__restrict__ run_max, uint32_t *__restrict__ counter, double *__restrict__ part,
    uint32_t *__restrict__ keys) {
    using namespace rstat;
    constexpr int kChunk = 8;
    const int64_t e0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool act = e0 < n;
    const int64_t e = act ? e0 : n - 1;  // every lane walks (the ballots), only act lanes count
    double acc[K];
#pragma unroll
    for (int j = 0; j < K; j++) acc[j] = is_min(j) ? INFINITY : is_max(j) ? -INFINITY : 0.0;
    acc[SMAX] = -1.0;
    const int64_t rsc0 = kEpi ? 0 : run_score[e];
    int64_t rsc = rsc0;
    int32_t rmx = kEpi ? 0 : run_max[e];
    uint32_t prev = 0;
    for (int64_t t0 = 0; t0 < T; t0 += kChunk) {
        uint32_t fl[kChunk], pw[kChunk], bm[kChunk];
        int32_t pt[kChunk], mt[kChunk];
        float av[kChunk], gnv[kChunk], grv[kChunk], vv[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int64_t k = min(t0 + u, T - 1) * n + e;
            fl[u] = sf[k];
            pw[u] = pot[k];
            pt[u] = points[k];
            av[u] = adv[k];
            gnv[u] = g_norm[k];
            grv[u] = g_raw[k];
            vv[u] = value[k];
            if (!kEpi) {
                const uint4 b = boards[k];
                uint32_t m = bytemax(bytemax(b.x, b.y), bytemax(b.z, b.w));
                m = bytemax(m, m >> 8);
                bm[u] = bytemax(m, m >> 16) & 0xFFu;
                mt[u] = max_tile[k];
            }
        }
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            if (t0 + u >= T) break;  // wave-uniform
            const uint32_t f = fl[u];
            const bool inactive = (f & FLAG_INACTIVE) != 0;
            const bool start = kEpi ? t0 + u == 0 : (prev & FLAG_RESET) != 0;
            prev = f;
            if (act && start) {
                acc[G0] += (double)grv[u];
                acc[G0N] += 1.0;
            }
            if (act && (!kEpi || !inactive)) {
                // the metric's reward in float32, operation for operation as the torch expression
                // points * w_p + w_m * (gamma * pot1 * (1 - done) - pot0) + w_e * (gamma * pot3 * (1 - done) - pot2)
                const uint32_t q = pw[u];
                const float p0 = (float)(int8_t)(q & 0xFFu), p1 = (float)(int8_t)((q >> 8) & 0xFFu);
                const float p2 = (float)(int8_t)((q >> 16) & 0xFFu), p3 = (float)(int8_t)(q >> 24);
                const float nd = (f & FLAG_DONE) ? 0.0f : 1.0f;
                const float x1 = __fsub_rn(__fmul_rn(__fmul_rn(gamma, p1), nd), p0);
                const float x2 = __fsub_rn(__fmul_rn(__fmul_rn(gamma, p3), nd), p2);
                const float r = __fadd_rn(__fadd_rn(__fmul_rn((float)pt[u], wp), __fmul_rn(wm, x1)), __fmul_rn(we, x2));
                const double rd = r, a = av[u], gn = gnv[u], gr = grv[u], v = vv[u];
                acc[N] += 1.0;
                acc[R] += rd;
                acc[R2] += rd * rd;
                acc[RZ] += r == 0.0f ? 1.0 : 0.0;
                acc[A] += a;
                acc[A2] += a * a;
                acc[AMIN] = fmin(acc[AMIN], a);
                acc[AMAX] = fmax(acc[AMAX], a);
                acc[GN] += gn;
                acc[GN2] += gn * gn;
                acc[GNMIN] = fmin(acc[GNMIN], gn);
                acc[GNMAX] = fmax(acc[GNMAX], gn);
                acc[GR] += gr;
                acc[GR2] += gr * gr;
                acc[V] += v;
                acc[V2] += v * v;
            }
            if (kEpi) {
                if (!inactive) rsc += pt[u];
                continue;
            }
            // fixed horizon: episode_scan_kernel's running score / max tile of the current game
            rsc += pt[u];
            rmx = max(rmx, max((int32_t)bm[u], mt[u]));
            const bool ends = (f & FLAG_DONE) && !inactive;
            if (act && ends) {
                acc[CNT] += 1.0;
                acc[SSUM] += (double)rsc;
                acc[SMAX] = fmax(acc[SMAX], (double)(int32_t)rsc);
                acc[T9] += rmx >= 9 ? 1.0 : 0.0;
                acc[T10] += rmx >= 10 ? 1.0 : 0.0;
                acc[T11] += rmx >= 11 ? 1.0 : 0.0;
            }
            if (ends) {
                rsc = 0;
                rmx = 0;
            }
        }
    }
    if (kEpi) {  // every env's game is finished: its score and the max tile of its final board
        const uint4 b = boards[T * n + e];
        uint32_t m = bytemax(bytemax(b.x, b.y), bytemax(b.z, b.w));
        m = bytemax(m, m >> 8);
        m = bytemax(m, m >> 16);
        const int32_t mx = (int32_t)(m & 0xFFu);
        if (act) {
            acc[CNT] = 1.0;
            acc[SSUM] = (double)rsc;
            acc[SMAX] = (double)(int32_t)rsc;
            acc[T9] = mx >= 9 ? 1.0 : 0.0;
            acc[T10] = mx >= 10 ? 1.0 : 0.0;
            acc[T11] = mx >= 11 ? 1.0 : 0.0;
        }
    } else if (act) {
        run_score[e] = rsc;
        run_max[e] = rmx;
    }
    // the finished scores into keys[]: the block reserves its range with ONE atomic (a per-step
    // atomic per wave serialises on the counter), lanes take block-exclusive-scan offsets, and the
    // fixed-horizon walk is replayed over points / flags to emit its keys in place
    __shared__ uint32_t wsum[kBlock / 64 + 1];
    {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        const uint32_t mine = act ? (uint32_t)acc[CNT] : 0u;
        uint32_t incl = mine;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
            for (int q = 0; q < kBlock / 64; q++) {
                const uint32_t c = wsum[q];
                wsum[q] = tot;
                tot += c;
            }
            wsum[kBlock / 64] = tot ? atomicAdd(counter, tot) : 0u;
        }
        __syncthreads();
        uint32_t at = wsum[kBlock / 64] + wsum[w] + incl - mine;
        if (kEpi) {
            if (act) keys[at] = (uint32_t)(int32_t)rsc;
        } else if (mine) {
            int64_t r2 = rsc0;
            for (int64_t t0 = 0; t0 < T; t0 += kChunk) {
                uint32_t fl[kChunk];
                int32_t pt[kChunk];
#pragma unroll
                for (int u = 0; u < kChunk; u++) {
                    const int64_t k = min(t0 + u, T - 1) * n + e;
                    fl[u] = sf[k];
                    pt[u] = points[k];
                }
#pragma unroll
                for (int u = 0; u < kChunk; u++) {
                    if (t0 + u >= T) break;
                    r2 += pt[u];
                    if ((fl[u] & FLAG_DONE) && !(fl[u] & FLAG_INACTIVE)) {
                        keys[at++] = (uint32_t)(int32_t)r2;
                        r2 = 0;
                    }
                }
            }
        }
    }
    // block reduction: wave butterflies, then the block's waves in order
    __shared__ double red[kBlock / 64][K];
#pragma unroll
    for (int j = 0; j < K; j++) {
        double x = acc[j];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x = combine(j, x, __shfl_xor(x, o));
        acc[j] = x;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < K; j++) red[w][j] = acc[j];
    __syncthreads();
    if (threadIdx.x < K) {
        const int j = threadIdx.x;
        double x = red[0][j];
        for (int q = 1; q < kBlock / 64; q++) x = combine(j, x, red[q][j]);
        part[(int64_t)blockIdx.x * K + j] = x;
    }
}

__global__ __launch_bounds__(1024) void rollout_stats_final_kernel(const double *__restrict__ part, int nb,
                                                                   uint32_t *__restrict__ counter,
                                                                   const uint32_t *__restrict__ keys,
                                                                   float *__restrict__ out) {
    using namespace rstat;
    __shared__ double tot[K];
    __shared__ uint32_t hist[2048];
    __shared__ uint32_t sel[2];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int j = w; j < K; j += 16) {  // column j: lanes stride the blocks in order, then a butterfly
        double x = is_min(j) ? INFINITY : is_max(j) ? -INFINITY : 0.0;
        if (j == SMAX) x = -1.0;
        for (int b = lane; b < nb; b += 64) x = combine(j, x, part[(int64_t)b * K + j]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x = combine(j, x, __shfl_xor(x, o));
        if (lane == 0) tot[j] = x;
    }
    const uint32_t cnt = counter[0];
    // lower median = the key of rank (cnt - 1) / 2: radix select, digits of at most 11 bits from the
    // highest bit any key has set (the OR of the keys) down
    __shared__ uint32_t kor;
    if (tid == 0) kor = 0;
    __syncthreads();
    {
        uint32_t o = 0;
        for (uint32_t i = tid; i < cnt; i += 1024) o |= keys[i];
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) o |= __shfl_xor(o, d);
        if (lane == 0 && o) atomicOr(&kor, o);
    }
    __syncthreads();
    uint32_t prefix = 0, pmask = 0, rank = cnt > 0 ? (cnt - 1) / 2 : 0;
    for (int hb = kor ? 32 - __clz((int)kor) : 0; hb > 0 && cnt > 0;) {
        const int sh = hb > 11 ? hb - 11 : 0;
        const uint32_t bm = (1u << (hb - sh)) - 1u;
        for (int i = tid; i < 2048; i += 1024) hist[i] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < cnt; i += 1024) {
            const uint32_t key = keys[i];
            if ((key & pmask) == prefix) atomicAdd(&hist[(key >> sh) & bm], 1u);
        }
        __syncthreads();
        if (w == 0) {  // lane owns bins [32 lane, 32 lane + 32)
            uint32_t s = 0;
            for (int j = 0; j < 32; j++) s += hist[lane * 32 + j];
            uint32_t incl = s;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            const uint32_t excl = incl - s;
            if (excl <= rank && rank < incl) {
                uint32_t c = excl;
                for (int j = 0; j < 32; j++) {
                    const uint32_t h = hist[lane * 32 + j];
                    if (rank < c + h) {
                        sel[0] = (uint32_t)(lane * 32 + j);
                        sel[1] = rank - c;
                        break;
                    }
                    c += h;
                }
            }
        }
        __syncthreads();
        prefix |= sel[0] << sh;
        pmask |= bm << sh;
        rank = sel[1];
        hb = sh;
        __syncthreads();
    }
    __syncthreads();
    if (tid == 0) {
        const double nr = tot[N], cf = fmax(tot[CNT], 1.0);
        const double rm = tot[R] / nr, am = tot[A] / nr, gnm = tot[GN] / nr, grm = tot[GR] / nr, vm = tot[V] / nr;
        const double o[23] = {
            nr, rm, fmax(tot[R2] / nr - rm * rm, 0.0), tot[RZ] / nr * 100.0,
            am, fmax(tot[A2] / nr - am * am, 0.0), sqrt(tot[A2]), tot[AMIN], tot[AMAX],
            gnm, sqrt(fmax(tot[GN2] / nr - gnm * gnm, 0.0)), tot[GNMIN], tot[GNMAX],
            sqrt(fmax(tot[GR2] / nr - grm * grm, 0.0)), sqrt(fmax(tot[V2] / nr - vm * vm, 0.0)),
            tot[G0] / fmax(tot[G0N], 1.0),
            tot[SSUM] / cf, cnt > 0 ? (double)(int32_t)prefix : -1.0, tot[SMAX],
            tot[T9] / cf * 100.0, tot[T10] / cf * 100.0, tot[T11] / cf * 100.0, tot[CNT]};
        for (int j = 0; j < 23; j++) out[j] = (float)o[j];
        counter[0] = 0;  // every thread has read it (the barrier above): the workspace is left zeroed
    }
}

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }


inline bool rng_ok(const g2048_rng *r) {
    if (!r) return false;
    if (r->mode == G2048_RNG_MT19937) return r->mt_state != nullptr;
    if (r->mode == G2048_RNG_INJECT) return r->inject != nullptr;
    return r->mode == G2048_RNG_PHILOX;
}


// ------------------------------------------------------------------ D4 up-sampling ------------
// calculate_advantage's augmentation (train.py:774-881): k distinct source samples, each with an
// independent 1/2 chance of a mirror copy (game.py:509-535, axis 1/2 each) and of a rotation copy
// (game.py:537-590, 90/180/270 degrees clockwise, 1/3 each).  Transform codes: 0 mirror horizontal
// (flip columns), 1 mirror vertical (flip rows), 2/3/4 rotation by 90/180/270 degrees.
struct AugPlan {
    uint32_t src;    // source row
    uint32_t mirror; // 0 none, else 1 + code
    uint32_t rot;    // 0 none, else 1 + code
};

__device__ __forceinline__ uint32_t lowbias32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    h *= 0x846CA68Bu;
    h ^= h >> 16;
    return h;
}

// Sample j -> source row: a 4-round Feistel permutation of [0, 2^bits) (bits even, 2^bits >= n),
// cycle-walked into [0, n), so k < n samples are k DISTINCT rows (random.sample without replacement).
__device__ __forceinline__ uint32_t feistel_row(uint32_t j, uint32_t n, uint32_t half, const uint4 &key) {
    const uint32_t mask = (1u << half) - 1u;
    const uint32_t rk[4] = {key.x, key.y, key.z, key.w};
    uint32_t x = j;
    do {
        uint32_t l = x >> half, r = x & mask;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t f = lowbias32(r ^ rk[q]) & mask;
            const uint32_t t = l ^ f;
            l = r;
            r = t;
        }
        x = (l << half) | r;
    } while (x >= n);
    return x;
}

__device__ __forceinline__ AugPlan aug_plan(uint32_t j, uint32_t n, uint32_t half, const uint4 &key, uint64_t seed,
                                            uint64_t counter) {
    const uint4 u = philox_draw(seed, counter, j, 3u);
    AugPlan p;
    p.src = feistel_row(j, n, half, key);
    p.mirror = u.x < 0x80000000u ? 1u + (u.y >> 31) : 0u;
    p.rot = u.z < 0x80000000u ? 3u + (uint32_t)(((uint64_t)u.w * 3u) >> 32) : 0u;
    return p;
}

// direction remap of each transform (UP, DOWN, LEFT, RIGHT = 0..3), 2 bits per direction:
// mirror h swaps LEFT/RIGHT, mirror v swaps UP/DOWN; 90 degrees: UP->RIGHT->DOWN->LEFT->UP
__device__ __forceinline__ uint32_t aug_dir(uint32_t code, uint32_t d) {
    constexpr uint32_t kMap[5] = {0u | 1u << 2 | 3u << 4 | 2u << 6, 1u | 0u << 2 | 2u << 4 | 3u << 6,
                                  3u | 2u << 2 | 0u << 4 | 1u << 6, 1u | 0u << 2 | 3u << 4 | 2u << 6,
                                  2u | 3u << 2 | 1u << 4 | 0u << 6};
    const uint32_t m = code == 0u ? kMap[0] : code == 1u ? kMap[1] : code == 2u ? kMap[2] : code == 3u ? kMap[3] : kMap[4];
    return (m >> (2u * d)) & 3u;
}

__device__ __forceinline__ uint4 aug_board(uint32_t code, const uint4 &b) {
    switch (code) {
        case 0u: return bswap4(b);                                        // new[i][3-j] = old[i][j]
        case 1u: return make_uint4(b.w, b.z, b.y, b.x);                   // new[3-i][j] = old[i][j]
        case 2u: return bswap4(transpose(b));                             // new[j][3-i] = old[i][j]
        case 3u: { const uint4 r = bswap4(b); return make_uint4(r.w, r.z, r.y, r.x); }
        default: { const uint4 t = transpose(b); return make_uint4(t.w, t.z, t.y, t.x); }  // new[3-j][i]
    }
}

struct AugArgs {
    uint4 *boards;
    uint8_t *actions, *legal;
    float4 *logp;
    float *adv, *ret;
    uint32_t n, k, half;
    uint4 key;
    uint64_t seed, counter;
};

__device__ __forceinline__ void aug_write(const AugArgs &a, uint32_t code, uint32_t src, int64_t dst) {
    a.boards[dst] = aug_board(code, a.boards[src]);
    a.actions[dst] = (uint8_t)aug_dir(code, a.actions[src] & 3u);
    const uint32_t lg = a.legal[src];
    uint32_t nl = lg & ~0xFu;
    const float4 lp = a.logp[src];
    const float o[4] = {lp.x, lp.y, lp.z, lp.w};
    float np[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (uint32_t d = 0; d < 4u; d++) {
        const uint32_t e = aug_dir(code, d);
        nl |= ((lg >> d) & 1u) << e;
        np[e] = o[d];  // new[remap(d)] = old[d] (train.py:810-824)
    }
    a.legal[dst] = (uint8_t)nl;
    a.logp[dst] = make_float4(np[0], np[1], np[2], np[3]);
    a.adv[dst] = a.adv[src];
    a.ret[dst] = a.ret[src];
}

constexpr int kAugBlock = 256;

// pass 1: copies emitted per block of samples
__global__ __launch_bounds__(kAugBlock) void aug_count_kernel(AugArgs a, uint32_t *__restrict__ counts) {
    __shared__ uint32_t red[kAugBlock / 64];
    const uint32_t j = blockIdx.x * kAugBlock + threadIdx.x;
    uint32_t c = 0u;
    if (j < a.k) {
        const uint4 u = philox_draw(a.seed, a.counter, j, 3u);
        c = (u.x < 0x80000000u ? 1u : 0u) + (u.z < 0x80000000u ? 1u : 0u);
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0u;
        for (int w = 0; w < kAugBlock / 64; w++) t += red[w];
        counts[blockIdx.x] = t;
    }
}

// pass 2 (one block): exclusive scan of the block counts in place; *count = n + total
__global__ __launch_bounds__(1024) void aug_scan_kernel(uint32_t *__restrict__ counts, int nblk, uint32_t n,
                                                        int64_t *__restrict__ count) {
    __shared__ uint32_t sh[1024];
    const int per = (nblk + 1023) / 1024, b0 = threadIdx.x * per;
    uint32_t loc = 0u;
    for (int q = 0; q < per && b0 + q < nblk; q++) loc += counts[b0 + q];
    sh[threadIdx.x] = loc;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
        const uint32_t v = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0u;
        __syncthreads();
        sh[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = sh[threadIdx.x] - loc;
    for (int q = 0; q < per && b0 + q < nblk; q++) {
        const uint32_t c = counts[b0 + q];
        counts[b0 + q] = run;
        run += c;
    }
    if (threadIdx.x == 1023) *count = (int64_t)n + (int64_t)sh[1023];
}

// pass 3: the copies, sample by sample (mirror before rotation), after the n real rows
__global__ __launch_bounds__(kAugBlock) void aug_emit_kernel(AugArgs a, const uint32_t *__restrict__ offsets) {
    __shared__ uint32_t sh[kAugBlock];
    const uint32_t j = blockIdx.x * kAugBlock + threadIdx.x;
    AugPlan p{0u, 0u, 0u};
    if (j < a.k) p = aug_plan(j, a.n, a.half, a.key, a.seed, a.counter);
    const uint32_t c = (p.mirror ? 1u : 0u) + (p.rot ? 1u : 0u);
    sh[threadIdx.x] = c;
    __syncthreads();
    for (int o = 1; o < kAugBlock; o <<= 1) {
        const uint32_t v = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0u;
        __syncthreads();
        sh[threadIdx.x] += v;
        __syncthreads();
    }
    int64_t dst = (int64_t)a.n + offsets[blockIdx.x] + (sh[threadIdx.x] - c);
    if (p.mirror) aug_write(a, p.mirror - 1u, p.src, dst++);
    if (p.rot) aug_write(a, p.rot - 1u, p.src, dst);
}

}  // namespace

extern "C" {

size_t g2048_mt_state_words(void) { return 625; }

int g2048_mt_seed(g2048_stream_t stream, uint32_t *mt_state, const uint64_t *seeds, int64_t n) {
    if (n < 0 || (n > 0 && (!mt_state || !seeds))) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    hipLaunchKernelGGL(mt_seed_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, (hipStream_t)stream, mt_state, seeds, n);
    return launch_status();
}

int g2048_env_reset(g2048_stream_t stream, int8_t *boards, uint8_t *flags, const uint8_t *where, int64_t n,
                    const g2048_rng *rng) {
    if (n < 0 || !rng_ok(rng) || (n > 0 && (!boards || !aligned16(boards)))) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    const RngArgs a = rng_args(rng);
    const dim3 g(blocks_for(n)), b(kBlock);
    hipStream_t s = (hipStream_t)stream;
    uint4 *bd = (uint4 *)boards;
    switch (rng->mode) {
        case G2048_RNG_PHILOX: hipLaunchKernelGGL(env_reset_kernel<G2048_RNG_PHILOX>, g, b, 0, s, bd, flags, where, n, a); break;
        case G2048_RNG_MT19937: hipLaunchKernelGGL(env_reset_kernel<G2048_RNG_MT19937>, g, b, 0, s, bd, flags, where, n, a); break;
        default: hipLaunchKernelGGL(env_reset_kernel<G2048_RNG_INJECT>, g, b, 0, s, bd, flags, where, n, a); break;
    }
    return launch_status();
}

int g2048_env_step(g2048_stream_t stream, const int8_t *boards_in, int8_t *boards_out, const uint8_t *actions_in,
                   uint8_t *actions_out, int32_t *points, int8_t *max_tile, int8_t *pot, uint8_t *flags, int64_t n,
                   const g2048_rng *rng, uint32_t options) {
    if (n < 0 || !rng_ok(rng)) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!boards_in || !boards_out || !points || !flags || !aligned16(boards_in) || !aligned16(boards_out)) return G2048_EINVAL;
    if (pot && ((uintptr_t)pot & 3u)) return G2048_EINVAL;
    if (options & ~(uint32_t)(G2048_OPT_AUTO_RESET | G2048_OPT_SKIP_DONE)) return G2048_EINVAL;
    const RngArgs a = rng_args(rng);
    const dim3 g(blocks_for(n)), b(kBlock);
    hipStream_t s = (hipStream_t)stream;
    const uint4 *bi = (const uint4 *)boards_in;
    uint4 *bo = (uint4 *)boards_out;
    uint32_t *pw = (uint32_t *)pot;
    switch (rng->mode) {
        case G2048_RNG_PHILOX:
            hipLaunchKernelGGL(env_step_kernel<G2048_RNG_PHILOX>, g, b, 0, s, bi, bo, actions_in, actions_out, points,
                               max_tile, pw, flags, n, a, options);
            break;
        case G2048_RNG_MT19937:
            hipLaunchKernelGGL(env_step_kernel<G2048_RNG_MT19937>, g, b, 0, s, bi, bo, actions_in, actions_out, points,
                               max_tile, pw, flags, n, a, options);
            break;
        default:
            hipLaunchKernelGGL(env_step_kernel<G2048_RNG_INJECT>, g, b, 0, s, bi, bo, actions_in, actions_out, points,
                               max_tile, pw, flags, n, a, options);
            break;
    }
    return launch_status();
}

int g2048_preview_points(g2048_stream_t stream, const int8_t *boards, int32_t *points4, int64_t n) {
    if (n < 0 || (n > 0 && (!boards || !points4 || !aligned16(boards) || !aligned16(points4)))) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    hipLaunchKernelGGL(preview_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, (hipStream_t)stream, (const uint4 *)boards,
                       (int4 *)points4, n);
    return launch_status();
}

int g2048_legal_mask(g2048_stream_t stream, const int8_t *boards, uint8_t *flags, int64_t n) {
    if (n < 0 || (n > 0 && (!boards || !flags || !aligned16(boards)))) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    hipLaunchKernelGGL(legal_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, (hipStream_t)stream, (const uint4 *)boards,
                       flags, n);
    return launch_status();
}

int g2048_info_deltas(g2048_stream_t stream, const int8_t *boards, const uint8_t *actions, double *deltas,
                      int8_t *anchor, int64_t n) {
    if (n < 0) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!boards || !actions || !deltas || !aligned16(boards)) return G2048_EINVAL;
    hipLaunchKernelGGL(info_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, (hipStream_t)stream, (const uint4 *)boards,
                       actions, deltas, anchor, n);
    return launch_status();
}

int g2048_obs_encode(g2048_stream_t stream, const int8_t *boards, void *obs, int32_t dtype, int64_t n) {
    if (n < 0 || (n > 0 && (!boards || !obs)) || (dtype != G2048_DTYPE_F32 && dtype != G2048_DTYPE_BF16))
        return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    const dim3 g(blocks_for(n * 12)), b(kBlock);
    if (dtype == G2048_DTYPE_F32)
        hipLaunchKernelGGL(obs_kernel<float>, g, b, 0, (hipStream_t)stream, boards, (float *)obs, n);
    else
        hipLaunchKernelGGL(obs_kernel<__hip_bfloat16>, g, b, 0, (hipStream_t)stream, boards, (__hip_bfloat16 *)obs, n);
    return launch_status();
}

int g2048_sample_actions(g2048_stream_t stream, const float *logits, int64_t logits_stride, const uint8_t *flags,
                         uint8_t *actions, float *logp, float *entropy, int64_t n, const g2048_rng *rng) {
    if (n < 0 || !rng || rng->mode != G2048_RNG_PHILOX) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!flags || !actions || (logits && logits_stride < 4)) return G2048_EINVAL;
    hipLaunchKernelGGL(sample_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, (hipStream_t)stream, logits,
                       logits_stride, flags, actions, logp, entropy, n, rng_args(rng));
    return launch_status();
}

size_t g2048_reward_rtg_workspace_bytes(int64_t n) { return (size_t)blocks_for(n > 0 ? n : 1) * 3 * sizeof(double); }

int g2048_rtg_prepare(g2048_stream_t stream, double *state, const g2048_reward_cfg *cfg) {
    if (!state || !cfg) return G2048_EINVAL;
    hipLaunchKernelGGL(rtg_prepare_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, state, cfg->beta);
    return launch_status();
}

int g2048_reward_rtg(g2048_stream_t stream, const int32_t *points, const int8_t *pot, const uint8_t *flags,
                     const float *value, int64_t T, int64_t n, const g2048_reward_cfg *cfg, const double *state,
                     float *g_raw, float *g_norm, float *adv, double *partials, void *workspace,
                     size_t workspace_bytes) {
    return g2048_reward_rtg_ex(stream, points, pot, flags, value, T, n, cfg, state, g_raw, g_norm, adv, nullptr,
                               partials, workspace, workspace_bytes);
}

int g2048_reward_rtg_ex(g2048_stream_t stream, const int32_t *points, const int8_t *pot, const uint8_t *flags,
                        const float *value, int64_t T, int64_t n, const g2048_reward_cfg *cfg, const double *state,
                        float *g_raw, float *g_norm, float *adv, double *reward, double *partials, void *workspace,
                        size_t workspace_bytes) {
    if (T < 0 || n < 0 || !cfg || !state || !partials) return G2048_EINVAL;
    if (workspace_bytes < g2048_reward_rtg_workspace_bytes(n) || !workspace) return G2048_EINVAL;
    if (T > 0 && n > 0 && (!points || !pot || !flags || !value || !g_raw || !g_norm || !adv)) return G2048_EINVAL;
    if (pot && ((uintptr_t)pot & 3u)) return G2048_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const unsigned nb = blocks_for(n > 0 ? n : 1);
    const RewardArgs ra{cfg->gamma, cfg->w_points, cfg->w_mono, cfg->w_empt};
    hipLaunchKernelGGL(rtg_kernel, dim3(nb), dim3(kBlock), 0, s, points, (const uint32_t *)pot, flags, value,
                       (n > 0 ? T : 0), n, ra, state, g_raw, g_norm, adv, reward, (double *)workspace);
    hipLaunchKernelGGL(rtg_reduce_kernel, dim3(1), dim3(kBlock), 0, s, (const double *)workspace, (int)nb, partials);
    return launch_status();
}

int g2048_rtg_finalize(g2048_stream_t stream, double *state, const double *partials, const g2048_reward_cfg *cfg) {
    if (!state || !partials || !cfg) return G2048_EINVAL;
    hipLaunchKernelGGL(rtg_finalize_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, state, partials, cfg->beta);
    return launch_status();
}

int g2048_episode_scan(g2048_stream_t stream, const int32_t *points, const int8_t *boards, const int8_t *max_tile,
                       const uint8_t *step_flags, int64_t T, int64_t n, int64_t *run_score, int32_t *run_max,
                       int64_t *scores, int32_t *tiles) {
    if (T < 0 || n < 0 || !points || !boards || !max_tile || !step_flags || !run_score || !run_max || !scores || !tiles)
        return G2048_EINVAL;
    if (!aligned16(boards)) return G2048_EINVAL;
    if (n == 0 || T == 0) return G2048_OK;
    hipLaunchKernelGGL(episode_scan_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, (hipStream_t)stream, points,
                       (const uint4 *)boards, max_tile, step_flags, T, n, run_score, run_max, scores, tiles);
    return launch_status();
}

size_t g2048_rollout_stats_workspace_bytes(int64_t T, int64_t n) {
    if (T < 1 || n < 1) return rstat::kHead;
    return rstat::kHead + (size_t)blocks_for(n) * rstat::K * sizeof(double) + (size_t)T * (size_t)n * sizeof(uint32_t);
}

int g2048_rollout_stats(g2048_stream_t stream, const int32_t *points, const int8_t *pot, const uint8_t *step_flags,
                        const float *value, const float *g_raw, const float *g_norm, const float *adv,
                        const int8_t *boards, const int8_t *max_tile, int64_t T, int64_t n, int32_t episodic,
                        const g2048_reward_cfg *cfg, int64_t *run_score, int32_t *run_max, void *workspace,
                        size_t workspace_bytes, float *out) {
    if (T < 1 || n < 1 || n > (int64_t)UINT32_MAX || T * n > (int64_t)UINT32_MAX || !points || !pot || !step_flags ||
        !value || !g_raw || !g_norm || !adv || !boards || !cfg || !workspace || !out)
        return G2048_EINVAL;
    if (!episodic && (!max_tile || !run_score || !run_max)) return G2048_EINVAL;
    if (!aligned16(boards) || ((uintptr_t)pot & 3u) || ((uintptr_t)workspace & 15u)) return G2048_EINVAL;
    if (workspace_bytes < g2048_rollout_stats_workspace_bytes(T, n)) return G2048_EINVAL;
    const unsigned nb = blocks_for(n);
    char *ws = (char *)workspace;
    uint32_t *counter = (uint32_t *)ws;
    double *part = (double *)(ws + rstat::kHead);
    uint32_t *keys = (uint32_t *)(ws + rstat::kHead + (size_t)nb * rstat::K * sizeof(double));
    const hipStream_t s = (hipStream_t)stream;
    const float wp = (float)cfg->w_points, wm = (float)cfg->w_mono, we = (float)cfg->w_empt, gm = (float)cfg->gamma;
    if (episodic)
        hipLaunchKernelGGL(rollout_stats_kernel<true>, dim3(nb), dim3(kBlock), 0, s, points, (const uint32_t *)pot,
                           step_flags, value, g_raw, g_norm, adv, (const uint4 *)boards, max_tile, T, n, wp, wm, we, gm,
                           run_score, run_max, counter, part, keys);
    else
        hipLaunchKernelGGL(rollout_stats_kernel<false>, dim3(nb), dim3(kBlock), 0, s, points, (const uint32_t *)pot,
                           step_flags, value, g_raw, g_norm, adv, (const uint4 *)boards, max_tile, T, n, wp, wm, we, gm,
                           run_score, run_max, counter, part, keys);
    hipLaunchKernelGGL(rollout_stats_final_kernel, dim3(1), dim3(1024), 0, s, (const double *)part, (int)nb, counter,
                       (const uint32_t *)keys, out);
    return launch_status();
}

// The epoch's minibatch order (DataLoader(shuffle=True), train.py:470): out[i] = a keyed Feistel
// bijection of [0, n) (feistel_row: 4 rounds over [0, 4^k), cycle-walked), round keys Philox-drawn
// in the kernel from *key_dev (a device draw of the update's generator: no host read) or `seed`.
__global__ __launch_bounds__(kBlock) void permutation_kernel(int64_t *__restrict__ out, uint32_t n, uint32_t half,
                                                             const int64_t *__restrict__ key_dev, uint64_t seed,
                                                             uint64_t counter) {
    const uint64_t sd = key_dev ? (uint64_t)key_dev[0] : seed;
    const uint4 key = philox_draw(sd, counter, 0xFFFFFFFEu, 5u);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
        out[i] = (int64_t)feistel_row(i, n, half, key);
}

int g2048_permutation(g2048_stream_t stream, int64_t *out, int64_t n, const int64_t *key_dev, uint64_t seed,
                      uint64_t counter) {
    if (n < 0 || n >= (int64_t(1) << 31) || (n > 0 && !out)) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    uint32_t bits = 2u;
    while ((1ull << bits) < (uint64_t)n) bits += 2u;
    const unsigned blocks = blocks_for(n) < 2048u ? blocks_for(n) : 2048u;
    hipLaunchKernelGGL(permutation_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, out, (uint32_t)n,
                       bits / 2u, key_dev, seed, counter);
    return launch_status();
}

// Philox4x32-10 on the host (the Feistel round keys of g2048_augment)
static uint4 philox_host(uint64_t seed, uint64_t step, uint32_t env, uint32_t stream) {
    uint32_t c0 = (uint32_t)step, c1 = (uint32_t)(step >> 32), c2 = env, c3 = stream;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        c0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        c1 = (uint32_t)p1;
        c2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

size_t g2048_augment_workspace_bytes(int64_t k) {
    return (size_t)((k > 0 ? k : 1) + kAugBlock - 1) / kAugBlock * sizeof(uint32_t);
}

int g2048_augment(g2048_stream_t stream, int8_t *boards, uint8_t *actions, uint8_t *legal, float *logp, float *adv,
                  float *ret, int64_t n, int64_t k, uint64_t seed, uint64_t counter, void *workspace,
                  size_t workspace_bytes, int64_t *count) {
    if (n < 0 || n >= (int64_t(1) << 31) || k < 0 || k > n || !count) return G2048_EINVAL;
    if (k > 0 && (!boards || !actions || !legal || !logp || !adv || !ret || !workspace || !aligned16(boards) ||
                  !aligned16(logp) || workspace_bytes < g2048_augment_workspace_bytes(k)))
        return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    if (k == 0) {  // no copies: *count = n
        hipLaunchKernelGGL(aug_scan_kernel, dim3(1), dim3(1024), 0, s, (uint32_t *)nullptr, 0, (uint32_t)n, count);
        return launch_status();
    }
    uint32_t bits = 2u;
    while ((1ull << bits) < (uint64_t)n) bits += 2u;
    const uint4 key = philox_host(seed, counter, 0xFFFFFFFFu, 4u);
    AugArgs a{(uint4 *)boards, actions, legal, (float4 *)logp, adv, ret, (uint32_t)n, (uint32_t)k, bits / 2u, key,
              seed, counter};
    const int nblk = (int)((k + kAugBlock - 1) / kAugBlock);
    uint32_t *counts = (uint32_t *)workspace;
    hipLaunchKernelGGL(aug_count_kernel, dim3(nblk), dim3(kAugBlock), 0, s, a, counts);
    hipLaunchKernelGGL(aug_scan_kernel, dim3(1), dim3(1024), 0, s, counts, nblk, (uint32_t)n, count);
    hipLaunchKernelGGL(aug_emit_kernel, dim3(nblk), dim3(kAugBlock), 0, s, a, (const uint32_t *)counts);
    return launch_status();
}

const char *g2048_build_info(void) { return "libg2048 gfx950 v0.1"; }

}  // extern "C"
