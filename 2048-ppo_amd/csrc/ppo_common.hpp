// ppo_common.hpp -- pieces shared by the PPO-update kernels (ppo_update.hip: the per-layer kernels;
// ppo_fused.hip: the fused per-row-tile forward / KL kernels): the dropout keep masks of
// GameMLP's ResidualBlocks (Philox draws regenerated from (row, column group, layer, pass,
// counter), never stored) and the per-row PPO-clip / entropy / smooth-L1 loss with its gradient
// (model_optimize_step, train.py:497-546) and the KL diagnostic of one row (train.py:578-601).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "board.hpp"
#include "../../include/g2048_ppo.h"

namespace g2048 {
namespace ppo {

struct DropArgs {
    uint32_t thr;       // keep iff 16-bit draw >= thr  (thr = round(p 2^16))
    float scale;        // 1 / (1 - p)
    uint32_t c1base;    // layer << 12 | pass << 20
    uint32_t k0, k1;    // seed
    uint64_t counter;
    const uint64_t *counter_dev;
};

struct Drop {
    uint32_t thr, c1base, c2, c3, k0, k1;
    float scale;
};

__device__ __forceinline__ Drop make_drop(const DropArgs &a) {
    const uint64_t c = a.counter + (a.counter_dev ? *a.counter_dev : 0ull);
    return Drop{a.thr, a.c1base, (uint32_t)c, (uint32_t)(c >> 32), a.k0, a.k1, a.scale};
}

// One Philox4x32-10 call gives 8 16-bit uniforms: the keep draws of column groups cg and cg ^ 4
// (cg = 8a + 4h + b shares the call (a, b); h picks the half), so a lane that owns both -- the
// fused forward's layout -- draws once per two groups.
__device__ __forceinline__ uint4 drop_draw4(const Drop &d, uint32_t row, uint32_t cg) {
    const uint32_t pair = ((cg >> 3) << 2) | (cg & 3u);
    return philox(row, pair | d.c1base, d.c2, d.c3, d.k0, d.k1);
}

__device__ __forceinline__ uint2 drop_half(const uint4 &r, uint32_t cg) {
    return (cg & 4u) ? make_uint2(r.z, r.w) : make_uint2(r.x, r.y);
}

__device__ __forceinline__ uint2 drop_draw(const Drop &d, uint32_t row, uint32_t cg) {
    return drop_half(drop_draw4(d, row, cg), cg);
}

__device__ __forceinline__ void drop_mult_bits(const Drop &d, uint2 w, float k[4]) {
    k[0] = (w.x & 0xFFFFu) >= d.thr ? d.scale : 0.0f;
    k[1] = (w.x >> 16) >= d.thr ? d.scale : 0.0f;
    k[2] = (w.y & 0xFFFFu) >= d.thr ? d.scale : 0.0f;
    k[3] = (w.y >> 16) >= d.thr ? d.scale : 0.0f;
}

// The same draw as 8 keep bits: bits 0-3 = columns 4 cg .. + 3 (cg & 4 == 0: the x, y words, as
// drop_mult_bits on drop_half), bits 4-7 = columns of cg ^ 4 (z, w) -- so a kernel can draw a row's
// masks ahead (between its MFMAs) and hold them in a register instead of 4 Philox words.
__device__ __forceinline__ uint32_t drop_keep8(const Drop &d, uint32_t row, uint32_t cg) {
    const uint4 r = drop_draw4(d, row, cg);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
    uint32_t b = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        b |= ((w[j] & 0xFFFFu) >= d.thr ? 1u : 0u) << (2 * j);
        b |= ((w[j] >> 16) >= d.thr ? 1u : 0u) << (2 * j + 1);
    }
    return b;
}

// The multipliers (0 or scale) of feature tile n from keep bits 4 n .. 4 n + 3 of kb[0] | kb[1] << 32:
// a sign-extended one-bit field masks the bits of `scale` (two VALU per feature).
__device__ __forceinline__ void keep_mult(const uint32_t (&kb)[2], int n, float scale, float k[4]) {
    const uint32_t w = kb[n >> 3];
    const int s = 4 * (n & 7);
    const int sc = __float_as_int(scale);
#pragma unroll
    for (int j = 0; j < 4; j++) k[j] = __int_as_float(((int)(w << (31 - s - j)) >> 31) & sc);
}

// keep multipliers (0 or 1/(1-p)) of columns 4cg .. 4cg+3 of `row`
__device__ __forceinline__ void drop_mult(const Drop &d, uint32_t row, uint32_t cg, float k[4]) {
    drop_mult_bits(d, drop_draw(d, row, cg), k);
}

// ------------------------------------------------------------------ minibatch statistics -------
struct StatsArgs {
    const float *sums, *gn, *beta;
    const int64_t *rows;
    float *stats;
    uint64_t *counter;
    uint32_t *sync;
    float critic, m;
    int64_t *idx_off;  // nullable: += idx_step (the next minibatch's rows in the epoch's permutation)
    int64_t idx_step;
};

// g2048_ppo_stats' arithmetic by the threads of one block (>= 256; LDS scratch of 2 KiB + 4): the KL
// partial rows [kl_rows][2] summed / maxed in ppo_stats_kernel's fixed order, then the stats update
// by thread 0, which also puts the ticket word back to zero
__device__ __forceinline__ void stats_block(const StatsArgs &a, const float *kl, int kl_rows, char *lds, int tid) {
    float(*red)[256] = reinterpret_cast<float(*)[256]>(lds);
    float ks = 0.0f, km = -INFINITY;
    if (tid < 256) {
        // sc1 loads (L2-served, past this CU's L1): the partials were handed off by other workgroups
        // (MI355X_MICROARCH.md hand-off table, row 1); the same bits as plain loads after an acquire
        float *klw = const_cast<float *>(kl);
        for (int b = tid; b < kl_rows; b += 256) {
            ks += __hip_atomic_load(klw + 2 * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            km = fmaxf(km, __hip_atomic_load(klw + 2 * b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
        red[0][tid] = ks;
        red[1][tid] = km;
    }
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (tid < w) {
            red[0][tid] += red[0][tid + w];
            red[1][tid] = fmaxf(red[1][tid], red[1][tid + w]);
        }
        __syncthreads();
    }
    if (tid != 0) return;
    ks = red[0][0];
    km = red[1][0];
    const float m = a.rows ? (float)max(*a.rows, (int64_t)1) : a.m;
    const float s_ppo = a.sums[0] / m, s_ent = a.sums[1] / m, s_v = a.sums[2] / m, b = *a.beta;
    a.stats[0] += -(s_ppo - a.critic * s_v + b * s_ent);
    a.stats[1] += -s_ppo;
    a.stats[2] += -b * s_ent;
    a.stats[3] += a.critic * s_v;
    a.stats[4] += *a.gn;
    a.stats[5] += s_ent;
    a.stats[6] += ks;
    a.stats[7] += ks / m;
    a.stats[8] = fmaxf(a.stats[8], km);
    if (a.counter) *a.counter += 1ull;
    if (a.idx_off) *a.idx_off += a.idx_step;
    __hip_atomic_store((__attribute__((address_space(1))) uint32_t *)a.sync, 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ heads + PPO loss ---------
struct HeadLossArgs {
    const int64_t *idx;
    const uint8_t *action;
    const uint8_t *legal;
    const float *old_logp;
    const float *adv;
    const float *ret;
    const float *beta_dev;
    const int64_t *rows;  // nullable: valid-row count of a padded minibatch
    float critic, clip_lo, clip_hi, inv_m;
    int decouple;
};

// The PPO-clip / entropy / smooth-L1 loss of one row and its gradient w.r.t. the 5 head outputs
// (train.py:497-546, with torch's backward conventions: minimum splits ties, clamp passes its
// bounds); z = {4 logits, value}, i = the row's index in the flat trajectory.
struct RowIn {
    uint32_t act, legal;
    float olp[4], adv, ret;
};

// The per-row inputs of trajectory row i (independent loads, issued together).
__device__ __forceinline__ RowIn load_row_in(const HeadLossArgs &a, int64_t i) {
    RowIn in;
    in.act = a.action[i] & 3u;
    in.legal = a.legal[i] & 0xFu;
    const float4 o = *reinterpret_cast<const float4 *>(a.old_logp + i * 4);
    in.olp[0] = o.x;
    in.olp[1] = o.y;
    in.olp[2] = o.z;
    in.olp[3] = o.w;
    in.adv = a.adv[i];
    in.ret = a.ret[i];
    return in;
}

__device__ __forceinline__ void row_loss(const float z[5], const RowIn &in, const HeadLossArgs &a, float beta_c,
                                         float dz[5], float mk[4], float &ppo_out, float &ent_out, float &vl_out) {
    const int act = (int)in.act;
    const uint32_t legal = in.legal;
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        mk[k] = (legal >> k) & 1u ? z[k] : -INFINITY;
        mx = fmaxf(mx, mk[k]);
    }
    float se = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; k++) se += (legal >> k) & 1u ? expf(mk[k] - mx) : 0.0f;
    const float lse = mx + logf(se);
    float sm[4];
#pragma unroll
    for (int k = 0; k < 4; k++) sm[k] = (legal >> k) & 1u ? expf(mk[k] - lse) : 0.0f;
    const float lp_a = mk[act] - lse;
    const float olp_a = act == 0 ? in.olp[0] : act == 1 ? in.olp[1] : act == 2 ? in.olp[2] : in.olp[3];
    const float dlt = lp_a - olp_a;
    const float ratio = expf(fminf(fmaxf(dlt, -20.0f), 20.0f));
    const bool in20 = dlt >= -20.0f && dlt <= 20.0f;
    const float A = in.adv;
    const float rc = fminf(fmaxf(ratio, a.clip_lo), a.clip_hi);
    const bool inr = ratio >= a.clip_lo && ratio <= a.clip_hi;
    const float t1 = A * ratio, t2 = A * rc;
    const float ppo = fminf(t1, t2);
    // torch.minimum backward: the smaller side takes the gradient, a tie splits it in halves
    float dp;
    if (t1 < t2) dp = A;
    else if (t1 > t2) dp = inr ? A : 0.0f;
    else dp = 0.5f * A + (inr ? 0.5f * A : 0.0f);
    const float dd = in20 ? dp * ratio : 0.0f;  // d ppo / d (logpi(a) - old)

    // entropy of softmax(clamp(masked, -20, 20)) summed over the legal actions
    float ck[4], cmx = -INFINITY;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        ck[k] = fminf(fmaxf(mk[k], -20.0f), 20.0f);
        cmx = fmaxf(cmx, ck[k]);
    }
    float se2 = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; k++) se2 += expf(ck[k] - cmx);
    const float lse2 = cmx + logf(se2);
    float lp2[4], p2[4], ent = 0.0f, S = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        lp2[k] = ck[k] - lse2;
        p2[k] = expf(lp2[k]);
        if ((legal >> k) & 1u) {
            ent -= p2[k] * lp2[k];
            S += p2[k] * (lp2[k] + 1.0f);
        }
    }
    const float dv0 = z[4] - in.ret;
    const float adv0 = fabsf(dv0);
    const float vl = adv0 < 1.0f ? 0.5f * dv0 * dv0 : adv0 - 0.5f;
    const float dvl = fminf(fmaxf(dv0, -1.0f), 1.0f);

#pragma unroll
    for (int k = 0; k < 4; k++) {
        const bool valid = (legal >> k) & 1u;
        const bool cpass = valid && mk[k] >= -20.0f && mk[k] <= 20.0f;
        const float dent = -(p2[k] * (lp2[k] + 1.0f) - p2[k] * S);
        const float g = dd * ((k == act ? 1.0f : 0.0f) - sm[k]) + (cpass ? beta_c * dent : 0.0f);
        dz[k] = valid ? -a.inv_m * g : 0.0f;
    }
    dz[4] = a.inv_m * a.critic * dvl;

    ppo_out = ppo;
    ent_out = ent;
    vl_out = vl;
}

// KL(old || new) of one row over its legal actions (old illegal = -inf), train.py:594-601
__device__ __forceinline__ float kl_row(const float o[4], const float z[4]) {
    bool ok[4];
    float mo = -INFINITY, mn = -INFINITY, nz[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        ok[k] = o[k] != -INFINITY;
        nz[k] = ok[k] ? z[k] : -INFINITY;
        mo = fmaxf(mo, o[k]);
        mn = fmaxf(mn, nz[k]);
    }
    float so = 0.0f, sn = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        so += ok[k] ? expf(o[k] - mo) : 0.0f;
        sn += ok[k] ? expf(nz[k] - mn) : 0.0f;
    }
    const float lso = mo + logf(so), lsn = mn + logf(sn);
    float kl = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (!ok[k]) continue;
        const float lo = o[k] - lso, ln = nz[k] - lsn;
        kl += expf(lo) * (lo - ln);
    }
    return kl;
}

// ------------------------------------------------------------------ host helpers -------------
inline DropArgs drop_args(const g2048_dropout *d) {
    DropArgs a{};
    a.thr = 0;
    a.scale = 1.0f;
    if (d && d->p > 0.0f) {
        const double t = (double)d->p * 65536.0;
        a.thr = t >= 65536.0 ? 0x10000u : (uint32_t)(t + 0.5);
        a.scale = 1.0f / (1.0f - d->p);
        a.c1base = (d->layer << 12) | (d->pass << 20);
        a.k0 = (uint32_t)d->seed;
        a.k1 = (uint32_t)(d->seed >> 32);
        a.counter = d->counter;
        a.counter_dev = d->counter_dev;
    }
    return a;
}

inline bool drop_on(const g2048_dropout *d) { return d && d->p > 0.0f; }


}  // namespace ppo
}  // namespace g2048
