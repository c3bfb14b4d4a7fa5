// urm_loss.hip -- the PPO minibatch loss of GameURM and its KL diagnostic as three device kernels
// (model_optimize_step, train.py:491-601, on GameURM's pooled features, game.py:1451-1456):
//
//   g2048_urm_head_loss      heads (action_head / value_head under bf16 autocast: bf16 operands,
//                            fp32 accumulation, the bf16 bias added before ONE bf16 rounding) + the
//                            PPO-clip / entropy / smooth-L1 loss of every row and its gradient dz
//                            w.r.t. the 5 head outputs (ppo_common.hpp row_loss, shared with GameMLP's
//                            fused passes), the masked logits for the KL, and the minibatch sums
//   g2048_urm_head_loss_bwd  dpooled = bf16(g dz) W (autocast's bf16 input-gradient GEMM, 5 terms) and
//                            the head weight / bias gradients (fixed-order block partials)
//   g2048_urm_kl_stats       KL(old || new) of every row on the re-forward's logits + the minibatch
//                            statistics (ppo_common.hpp stats_block, as GameMLP's fused KL pass)
//
// replacing ~50 small torch kernels per minibatch (gathers of the trajectory columns, masked_fill,
// log_softmax, clamp, exp, minimum, smooth_l1, the means, their autograd backward, the heads' cast /
// copy / pad kernels, the KL's masked softmaxes and the statistics stack).  One thread per board row;
// every reduction is a fixed-order tree plus a last-block pass over the block partials (the counter
// form of cdna_hip_programming.md Guideline 16: plain partial stores, drain, one release + ticket;
// the last arriver acquires and puts the ticket back to zero): deterministic, one launch each.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/g2048_ppo.h"
#include "../../include/g2048_urm.h"
#include "ppo_common.hpp"

namespace {

namespace P = g2048::ppo;

constexpr int kT = 256;  // rows (threads) per block

__device__ __forceinline__ float bfr(float f) { return (float)(__bf16)f; }

// 4 consecutive pooled features from element i (i % 4 == 0), rounded to bf16 like autocast's operand
__device__ __forceinline__ void ld_pooled4(const void *p, int pb, int64_t i, float (&x)[4]) {
    if (pb) {
        const uint2 u = *reinterpret_cast<const uint2 *>(reinterpret_cast<const uint16_t *>(p) + i);
        x[0] = __builtin_bit_cast(float, u.x << 16);
        x[1] = __builtin_bit_cast(float, u.x & 0xFFFF0000u);
        x[2] = __builtin_bit_cast(float, u.y << 16);
        x[3] = __builtin_bit_cast(float, u.y & 0xFFFF0000u);
    } else {
        const float4 v = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + i);
        x[0] = bfr(v.x);
        x[1] = bfr(v.y);
        x[2] = bfr(v.z);
        x[3] = bfr(v.w);
    }
}

// true in every thread of the last block to finish (its partial stores visible to it); the ticket
// word is put back to zero by the caller's last block once it is done
__device__ bool arrive_last(uint32_t *sync, int *flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t k = __hip_atomic_fetch_add((__attribute__((address_space(1))) uint32_t *)sync, 1u,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = k == gridDim.x - 1u;
    }
    __syncthreads();
    if (!*flag) return false;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    return true;
}

__device__ __forceinline__ void reset_ticket(uint32_t *sync) {
    __hip_atomic_store((__attribute__((address_space(1))) uint32_t *)sync, 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// sum (or max) of v over the block's 256 threads in a fixed tree order; result in thread 0
__device__ __forceinline__ float block_tree(float v, float *red, bool mx) {
    const int t = threadIdx.x;
    red[t] = v;
    __syncthreads();
    for (int w = kT / 2; w > 0; w >>= 1) {
        if (t < w) red[t] = mx ? fmaxf(red[t], red[t + w]) : red[t] + red[t + w];
        __syncthreads();
    }
    const float r = red[0];
    __syncthreads();
    return r;
}

// the 5 head rows (action 0-3, value 4) as autocast's bf16 operands, their bf16 biases
template <int H>
__device__ __forceinline__ void stage_heads(const float *wa, const float *ba, const float *wv, const float *bv,
                                            float (*sw)[H], float *sb) {
    for (int e = threadIdx.x; e < 5 * H; e += kT) sw[e / H][e % H] = bfr(e < 4 * H ? wa[e] : wv[e - 4 * H]);
    if (threadIdx.x < 5) sb[threadIdx.x] = bfr(threadIdx.x < 4 ? ba[threadIdx.x] : bv[0]);
    __syncthreads();
}

struct LossArgs {
    const void *pooled;
    int pb;  // pooled is bf16 (else fp32)
    const float *wa, *ba, *wv, *bv;
    P::HeadLossArgs la;
    int64_t m;
    float *dz, *masked, *part, *sums, *loss;
    uint32_t *sync;
};

template <int H>
__global__ __launch_bounds__(kT) void urm_head_loss_kernel(LossArgs a) {
    __shared__ float sw[5][H];
    __shared__ float sb[5];
    __shared__ float red[kT];
    __shared__ int flag;
    stage_heads<H>(a.wa, a.ba, a.wv, a.bv, sw, sb);
    const int64_t r = (int64_t)blockIdx.x * kT + threadIdx.x;
    const float beta = *a.la.beta_dev;
    float ppo = 0.0f, ent = 0.0f, vl = 0.0f;
    if (r < a.m) {
        const P::RowIn in = P::load_row_in(a.la, a.la.idx[r]);
        float z[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 4
        for (int j = 0; j < H; j += 4) {
            float x[4];
            ld_pooled4(a.pooled, a.pb, r * H + j, x);
#pragma unroll
            for (int u = 0; u < 4; u++)
#pragma unroll
                for (int k = 0; k < 5; k++) z[k] = __builtin_fmaf(x[u], sw[k][j + u], z[k]);
        }
#pragma unroll
        for (int k = 0; k < 5; k++) z[k] = bfr(z[k] + sb[k]);  // autocast: bf16(x W^T + b)
        float dz[5], mk[4];
        P::row_loss(z, in, a.la, beta, dz, mk, ppo, ent, vl);
        float4 *d = reinterpret_cast<float4 *>(a.dz + r * 8);
        d[0] = make_float4(dz[0], dz[1], dz[2], dz[3]);
        d[1] = make_float4(dz[4], 0.0f, 0.0f, 0.0f);
        *reinterpret_cast<float4 *>(a.masked + r * 4) = make_float4(mk[0], mk[1], mk[2], mk[3]);
    }
    const float s0 = block_tree(ppo, red, false), s1 = block_tree(ent, red, false), s2 = block_tree(vl, red, false);
    if (threadIdx.x == 0)
        *reinterpret_cast<float4 *>(a.part + (int64_t)blockIdx.x * 4) = make_float4(s0, s1, s2, 0.0f);
    if (!arrive_last(a.sync, &flag)) return;
    float t[3] = {0.0f, 0.0f, 0.0f};
    for (int b = threadIdx.x; b < (int)gridDim.x; b += kT) {
        const float4 p = *reinterpret_cast<const float4 *>(a.part + (int64_t)b * 4);
        t[0] += p.x;
        t[1] += p.y;
        t[2] += p.z;
    }
    const float u0 = block_tree(t[0], red, false), u1 = block_tree(t[1], red, false), u2 = block_tree(t[2], red, false);
    if (threadIdx.x == 0) {
        a.sums[0] = u0;
        a.sums[1] = u1;
        a.sums[2] = u2;
        const float im = a.la.inv_m;
        a.loss[0] = -(u0 * im - a.la.critic * (u2 * im) + beta * (u1 * im));
        reset_ticket(a.sync);
    }
}

struct BwdArgs {
    const void *pooled;
    int pb;
    const float *wa, *wv, *dz, *grad_out;
    void *dpooled;  // pooled's dtype
    float *part;
    uint32_t *sync;
    float *dwa, *dba, *dwv, *dbv;
    int acc;
    int64_t m;
};

template <int H>
__global__ __launch_bounds__(kT) void urm_head_loss_bwd_kernel(BwdArgs a) {
    constexpr int NO = 5 * H + 5;  // outputs: dW [5][H] then db [5]
    __shared__ float sw[5][H];
    __shared__ float sb[5];
    __shared__ __bf16 xs[kT][H + 2];  // this block's bf16 pooled rows (33-dword pitch: conflict-free row stores)
    __shared__ float ys[kT][5];      // ... and their bf16 output gradients dy
    __shared__ int flag;
    stage_heads<H>(a.wa, a.wa, a.wv, a.wv, sw, sb);  // (the biases are not used here)
    const int tid = threadIdx.x;
    const int64_t r = (int64_t)blockIdx.x * kT + tid;
    const float go = *a.grad_out;
    float dy[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if (r < a.m) {
        const float4 d0 = *reinterpret_cast<const float4 *>(a.dz + r * 8);
        const float d4 = a.dz[r * 8 + 4];
        // the heads' output gradient as autocast hands it to the bf16 GEMMs
        dy[0] = bfr(go * d0.x);
        dy[1] = bfr(go * d0.y);
        dy[2] = bfr(go * d0.z);
        dy[3] = bfr(go * d0.w);
        dy[4] = bfr(go * d4);
    }
#pragma unroll
    for (int k = 0; k < 5; k++) ys[tid][k] = dy[k];
#pragma unroll 4
    for (int j = 0; j < H; j += 4) {
        float x[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (r < a.m) ld_pooled4(a.pooled, a.pb, r * H + j, x);
        float dp[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            xs[tid][j + u] = (__bf16)x[u];
            float s = 0.0f;
#pragma unroll
            for (int k = 0; k < 5; k++) s = __builtin_fmaf(dy[k], sw[k][j + u], s);
            dp[u] = bfr(s);  // dpooled = bf16(dy W), in pooled's dtype
        }
        if (r < a.m) {
            if (a.pb)
                *reinterpret_cast<uint2 *>(reinterpret_cast<uint16_t *>(a.dpooled) + r * H + j) =
                    make_uint2((__builtin_bit_cast(uint32_t, dp[0]) >> 16) | (__builtin_bit_cast(uint32_t, dp[1]) & 0xFFFF0000u),
                               (__builtin_bit_cast(uint32_t, dp[2]) >> 16) | (__builtin_bit_cast(uint32_t, dp[3]) & 0xFFFF0000u));
            else
                *reinterpret_cast<float4 *>(reinterpret_cast<float *>(a.dpooled) + r * H + j) =
                    make_float4(dp[0], dp[1], dp[2], dp[3]);
        }
    }
    __syncthreads();
    // block partials of dW = dy^T x and db = sum dy over its rows, rows in order
    for (int o = tid; o < NO; o += kT) {
        float s = 0.0f;
        if (o < 5 * H) {
            const int k = o / H, j = o - k * H;
            for (int t = 0; t < kT; t++) s = __builtin_fmaf(ys[t][k], (float)xs[t][j], s);
        } else {
            const int k = o - 5 * H;
            for (int t = 0; t < kT; t++) s += ys[t][k];
        }
        a.part[(int64_t)blockIdx.x * NO + o] = s;
    }
    if (!arrive_last(a.sync, &flag)) return;
    const int nb = (int)gridDim.x;
    for (int o = tid; o < NO; o += kT) {
        float s = 0.0f;
        int b = 0;
        for (; b + 8 <= nb; b += 8) {  // 8 loads in flight, added in block order
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = a.part[(int64_t)(b + u) * NO + o];
#pragma unroll
            for (int u = 0; u < 8; u++) s += v[u];
        }
        for (; b < nb; b++) s += a.part[(int64_t)b * NO + o];
        float *dst = o < 4 * H ? a.dwa + o : o < 5 * H ? a.dwv + (o - 4 * H) : o < 5 * H + 4 ? a.dba + (o - 5 * H) : a.dbv;
        *dst = a.acc ? *dst + s : s;
    }
    __syncthreads();
    if (tid == 0) reset_ticket(a.sync);
}

struct KlArgs {
    const float *old_masked, *logits;
    int64_t m;
    float *part;
    P::StatsArgs st;
};

__global__ __launch_bounds__(kT) void urm_kl_stats_kernel(KlArgs a) {
    __shared__ float red[kT];
    __shared__ __attribute__((aligned(16))) char lds[2 * 256 * 4 + 16];
    __shared__ int flag;
    const int64_t r = (int64_t)blockIdx.x * kT + threadIdx.x;
    float kl = 0.0f, km = -INFINITY;
    if (r < a.m) {
        const float4 o4 = *reinterpret_cast<const float4 *>(a.old_masked + r * 4);
        const float4 z4 = *reinterpret_cast<const float4 *>(a.logits + r * 4);
        const float o[4] = {o4.x, o4.y, o4.z, o4.w}, z[4] = {z4.x, z4.y, z4.z, z4.w};
        kl = P::kl_row(o, z);
        km = kl;
    }
    const float s = block_tree(kl, red, false), mx = block_tree(km, red, true);
    if (threadIdx.x == 0) *reinterpret_cast<float2 *>(a.part + (int64_t)blockIdx.x * 2) = make_float2(s, mx);
    if (!arrive_last(a.st.sync, &flag)) return;
    P::stats_block(a.st, a.part, (int)gridDim.x, lds, threadIdx.x);  // (thread 0 resets the ticket)
}

inline int nblocks(int64_t m) { return (int)((m + kT - 1) / kT); }

bool h_ok(int h) { return h == 64 || h == 32; }

}  // namespace

extern "C" {

size_t g2048_urm_head_loss_partials(int64_t m, int32_t h) {
    if (m <= 0 || !h_ok(h)) return 0;
    return (size_t)nblocks(m) * (size_t)(5 * h + 5 > 4 ? 5 * h + 5 : 4);
}

int g2048_urm_head_loss(g2048_stream_t stream, const void *pooled, int32_t pooled_dtype, const float *wa,
                        const float *ba, const float *wv, const float *bv, int64_t m, int32_t h,
                        const struct g2048_ppo_batch *batch, const float *beta_dev, float critic, float clip_eps,
                        float *dz, float *masked, float *partials, uint32_t *sync, float *sums, float *loss) {
    if (m <= 0 || !h_ok(h) || (pooled_dtype != 0 && pooled_dtype != 1) || !batch) return G2048_EINVAL;
    if (!pooled || !wa || !ba || !wv || !bv || !beta_dev || !dz || !masked || !partials || !sync || !sums || !loss)
        return G2048_EINVAL;
    if (!batch->idx || !batch->action || !batch->legal || !batch->old_logp || !batch->adv || !batch->ret || batch->rows)
        return G2048_EINVAL;  // (no padded rows: the URM update runs a ragged minibatch at its own size)
    if (((uintptr_t)dz | (uintptr_t)masked | (uintptr_t)partials | (uintptr_t)batch->old_logp | (uintptr_t)pooled) % 16)
        return G2048_EINVAL;
    LossArgs a{};
    a.pooled = pooled;
    a.pb = pooled_dtype;
    a.wa = wa;
    a.ba = ba;
    a.wv = wv;
    a.bv = bv;
    a.la.idx = batch->idx;
    a.la.action = batch->action;
    a.la.legal = batch->legal;
    a.la.old_logp = batch->old_logp;
    a.la.adv = batch->adv;
    a.la.ret = batch->ret;
    a.la.beta_dev = beta_dev;
    a.la.rows = nullptr;
    a.la.critic = critic;
    a.la.clip_lo = 1.0f - clip_eps;
    a.la.clip_hi = 1.0f + clip_eps;
    a.la.inv_m = 1.0f / (float)m;
    a.la.decouple = 0;
    a.m = m;
    a.dz = dz;
    a.masked = masked;
    a.part = partials;
    a.sums = sums;
    a.loss = loss;
    a.sync = sync;
    const hipStream_t s = (hipStream_t)stream;
    if (h == 64) hipLaunchKernelGGL(urm_head_loss_kernel<64>, dim3(nblocks(m)), dim3(kT), 0, s, a);
    else hipLaunchKernelGGL(urm_head_loss_kernel<32>, dim3(nblocks(m)), dim3(kT), 0, s, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}

int g2048_urm_head_loss_bwd(g2048_stream_t stream, const void *pooled, int32_t pooled_dtype, const float *wa,
                            const float *wv, const float *dz, const float *grad_out, void *dpooled, float *partials,
                            uint32_t *sync, float *dwa, float *dba, float *dwv, float *dbv, int32_t accumulate,
                            int64_t m, int32_t h) {
    if (m <= 0 || !h_ok(h) || (pooled_dtype != 0 && pooled_dtype != 1)) return G2048_EINVAL;
    if (!pooled || !wa || !wv || !dz || !grad_out || !dpooled || !partials || !sync || !dwa || !dba || !dwv || !dbv)
        return G2048_EINVAL;
    if (((uintptr_t)dz | (uintptr_t)pooled | (uintptr_t)dpooled) % 16) return G2048_EINVAL;
    BwdArgs a{};
    a.pooled = pooled;
    a.pb = pooled_dtype;
    a.wa = wa;
    a.wv = wv;
    a.dz = dz;
    a.grad_out = grad_out;
    a.dpooled = dpooled;
    a.part = partials;
    a.sync = sync;
    a.dwa = dwa;
    a.dba = dba;
    a.dwv = dwv;
    a.dbv = dbv;
    a.acc = accumulate ? 1 : 0;
    a.m = m;
    const hipStream_t s = (hipStream_t)stream;
    if (h == 64) hipLaunchKernelGGL(urm_head_loss_bwd_kernel<64>, dim3(nblocks(m)), dim3(kT), 0, s, a);
    else hipLaunchKernelGGL(urm_head_loss_bwd_kernel<32>, dim3(nblocks(m)), dim3(kT), 0, s, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}

int g2048_urm_kl_stats(g2048_stream_t stream, const float *old_masked, const float *logits, int64_t m,
                       const float *sums, const float *gn, const float *beta_dev, float critic, float *stats,
                       float *partials, uint32_t *sync) {
    if (m <= 0 || !old_masked || !logits || !sums || !gn || !beta_dev || !stats || !partials || !sync)
        return G2048_EINVAL;
    if (((uintptr_t)old_masked | (uintptr_t)logits | (uintptr_t)partials) % 16) return G2048_EINVAL;
    KlArgs a{};
    a.old_masked = old_masked;
    a.logits = logits;
    a.m = m;
    a.part = partials;
    a.st.sums = sums;
    a.st.gn = gn;
    a.st.beta = beta_dev;
    a.st.rows = nullptr;
    a.st.stats = stats;
    a.st.counter = nullptr;
    a.st.sync = sync;
    a.st.critic = critic;
    a.st.m = (float)m;
    a.st.idx_off = nullptr;
    a.st.idx_step = 0;
    hipLaunchKernelGGL(urm_kl_stats_kernel, dim3(nblocks(m)), dim3(kT), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}

}  // extern "C"
