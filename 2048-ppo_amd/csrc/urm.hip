// GameURM policy forward (game.py:1223-1458) for gfx950: the fused kernels between the block's four
// projections (include/g2048_urm.h).  A board is 16 consecutive token rows of every activation.
//
//   stem             one wave per token row: Linear(3 -> h) + LayerNorm + SiLU, + init_hidden
//   attention        one wave per (board, head) on v_mfma_f32_16x16x16_bf16:
//                      S^T = K Q^T  -> lane (i, g) = (l & 15, l >> 4) holds S[i][4g .. 4g+3],
//                      i.e. query i's scores of keys 4g..4g+3: the row softmax is 4 values in
//                      registers + two cross-lane steps (xor 16, xor 32);
//                      O^T = V^T P^T -> the P fragment a lane holds is exactly its B operand
//                      (B[k = key][n = query]), no shuffles; lane (i, g) gets O[i][4g .. 4g+3].
//   residual_rms     x = rms_norm(x + y) [+ emb], bf16 copy for the next GEMM: h / 4 lanes per
//                    row (rounded to a power of two), 4 columns per lane, 64 / P rows per wave
//   swiglu_conv      one thread per (board, channel pair): SiLU(gate)*up, the kernel-2 depthwise
//                    conv along the board's 16 tokens carried in registers, SiLU
//   pool_heads       one wave per board: mean over the 16 tokens, action / value heads
//
// fp32 arithmetic throughout (bf16 only as GEMM operands / attention probabilities, like torch's
// bf16 autocast of the same module); parity vs the fp32 module in tests/test_gpu_urm.py.
#include <hip/hip_runtime.h>
#include <algorithm>

#include <cstdint>

#include "../../include/g2048_urm.h"
#include "board.hpp"
#include "wgrad_ring.hpp"

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kMaxPerLane = 8;  // h <= 512 over 64 lanes

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }
// round to nearest even on the hardware converter (v_cvt_pk_bf16_f32: one instruction per pair)
typedef __bf16 bf16x2_hw __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t pk2bf(float a, float b) {
    const bf16x2_hw v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}
// x * sigmoid(x) with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of an IEEE division
// sequence: exp overflow for x << 0 gives rcp(inf) = 0, i.e. -0
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// silu of a feature pair with the multiplies / adds packed (v_pk_mul_f32 / v_pk_add_f32) around the
// per-element v_exp_f32 / v_rcp_f32: per element the operations of silu() (__expf(-x) is
// exp2(x * -log2 e)), so the same bits
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 silu2(f32x2 x) {
    const f32x2 t = x * f32x2{-1.44269504088896341f, -1.44269504088896341f};
    const f32x2 d = f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + f32x2{1.0f, 1.0f};
    return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// butterfly steps across the 16-lane rows on the VALU lane swaps (v_permlane16/32_swap) instead of
// ds_bpermute round trips through LDS: x op x[lane ^ 16], x op x[lane ^ 32]
__device__ __forceinline__ float xsum16(float x) {
    const uint32_t u = __float_as_uint(x);
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float x) {
    const uint32_t u = __float_as_uint(x);
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xmax16(float x) {
    const uint32_t u = __float_as_uint(x);
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xmax32(float x) {
    const uint32_t u = __float_as_uint(x);
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

inline int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}
inline unsigned blocks(int64_t items, int per_block) { return (unsigned)((items + per_block - 1) / per_block); }
inline bool h_ok(int32_t h) { return h > 0 && h % 4 == 0 && h <= 64 * kMaxPerLane; }

template <bool kBf16Obs>
__global__ __launch_bounds__(kThreads) void urm_stem_kernel(const void *__restrict__ obs, const float *__restrict__ w,
                                                            const float *__restrict__ lnw,
                                                            const float *__restrict__ lnb,
                                                            const float *__restrict__ init,
                                                            float *__restrict__ emb, float *__restrict__ x,
                                                            uint16_t *__restrict__ xb, int64_t rows, int h) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int64_t b = row >> 4;
    const int t = (int)(row & 15);
    float f[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const int64_t o = b * 48 + 3 * t + k;
        f[k] = kBf16Obs ? bf2f(static_cast<const uint16_t *>(obs)[o]) : static_cast<const float *>(obs)[o];
    }
    float y[kMaxPerLane];
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < kMaxPerLane; j++) {
        const int c = lane + 64 * j;
        y[j] = 0.0f;
        if (c < h) y[j] = fmaf(w[3 * c + 2], f[2], fmaf(w[3 * c + 1], f[1], w[3 * c] * f[0]));
        s += y[j];
    }
    const float mean = wave_sum(s) / (float)h;
    float v = 0.0f;
#pragma unroll
    for (int j = 0; j < kMaxPerLane; j++) {
        const float d = y[j] - mean;
        v += (lane + 64 * j < h) ? d * d : 0.0f;
    }
    const float rstd = rsqrtf(wave_sum(v) / (float)h + 1e-5f);
#pragma unroll
    for (int j = 0; j < kMaxPerLane; j++) {
        const int c = lane + 64 * j;
        if (c >= h) continue;
        const float e = silu((y[j] - mean) * rstd * lnw[c] + lnb[c]);
        const float xv = init[t * h + c] + e;
        emb[row * h + c] = e;
        x[row * h + c] = xv;
        xb[row * h + c] = f2bf(xv);
    }
}

// Attention dropout (training mode, game.py:1314 dropout_p): keep multipliers (0 or 1/(1-p)) of
// P[query i][keys 4g .. 4g+3] of (board b, head hh) -- one Philox4x32-10 draw (words x, y: four
// 16-bit uniforms, keep iff u >= thr = round(p 2^16)), counter {b, hh|i|g, call counter}, key = the
// seed.  The forward and backward lane layouts both hold 4 consecutive keys of one query, so both
// regenerate the same mask from the same draw; nothing is stored.
struct AttnDrop {
    uint32_t thr;
    float scale;
    uint32_t k0, k1;
    const uint64_t *counter;  // device call counter (graph-replay safe)
    uint64_t offset;          // this application's offset from *counter (round 5: one counter bump per forward)
};
__device__ __forceinline__ void attn_keep_c(const AttnDrop &d, uint64_t c, int64_t b, int hh, int i, int g, float km[4]) {
    const uint4 r = g2048::philox((uint32_t)b, ((uint32_t)hh << 8) | ((uint32_t)i << 2) | (uint32_t)g, (uint32_t)c,
                                  (uint32_t)(c >> 32), d.k0, d.k1);
    km[0] = (r.x & 0xFFFFu) >= d.thr ? d.scale : 0.0f;
    km[1] = (r.x >> 16) >= d.thr ? d.scale : 0.0f;
    km[2] = (r.y & 0xFFFFu) >= d.thr ? d.scale : 0.0f;
    km[3] = (r.y >> 16) >= d.thr ? d.scale : 0.0f;
}
__device__ __forceinline__ void attn_keep(const AttnDrop &d, int64_t b, int hh, int i, int g, float km[4]) {
    attn_keep_c(d, *d.counter + d.offset, b, hh, i, g, km);
}

template <bool kAligned, bool kDrop>
__global__ __launch_bounds__(kThreads) void urm_attn_kernel(const uint16_t *__restrict__ qkv,
                                                            uint16_t *__restrict__ out, int64_t tasks, int h,
                                                            int heads, AttnDrop drop) {
    const int lane = threadIdx.x & 63;
    const int64_t task = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (task >= tasks) return;  // wave-uniform
    const int64_t b = task / heads;
    const int hh = (int)(task - b * heads);
    const int hd = h / heads;
    const int i = lane & 15, g = lane >> 4;
    const uint16_t *base = qkv + b * 16 * (int64_t)(3 * h);
    const uint16_t *qrow = base + (int64_t)i * (3 * h) + hh * hd;  // query / key row i of this head
    const uint16_t *krow = qrow + h;
    // S^T = K Q^T over head_dim in steps of 16 (zero-padded)
    f32x4 st = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int d0 = 0; d0 < hd; d0 += 16) {
        s16x4 ka, qb;
        const int dq = d0 + 4 * g;
        if (kAligned) {  // 4 | head_dim: a fragment is one 8-byte load (or entirely padding)
            const uint2 kv = dq < hd ? *reinterpret_cast<const uint2 *>(krow + dq) : make_uint2(0u, 0u);
            const uint2 qv = dq < hd ? *reinterpret_cast<const uint2 *>(qrow + dq) : make_uint2(0u, 0u);
            ka = __builtin_bit_cast(s16x4, kv);
            qb = __builtin_bit_cast(s16x4, qv);
        } else {
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const int d = dq + jj;
                ka[jj] = d < hd ? (short)krow[d] : (short)0;
                qb[jj] = d < hd ? (short)qrow[d] : (short)0;
            }
        }
        st = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ka, qb, st, 0, 0, 0);
    }
    // lane (i, g): st[r] = S[i][4g + r]; softmax over the 16 keys of query i
    const float scale = 1.0f / sqrtf((float)hd);
    float p[4];
    float m = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        p[r] = st[r] * scale;
        m = fmaxf(m, p[r]);
    }
    m = xmax32(xmax16(m));
    float sum = 0.0f;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        p[r] = __expf(p[r] - m);
        sum += p[r];
    }
    sum = xsum32(xsum16(sum));
    const float inv = 1.0f / sum;
    float km[4] = {1.0f, 1.0f, 1.0f, 1.0f};
    if (kDrop) attn_keep(drop, b, hh, i, g, km);
    s16x4 pb;  // B operand of O^T = V^T P^T: B[k = key 4g + jj][n = query i]
#pragma unroll
    for (int r = 0; r < 4; r++) pb[r] = (short)f2bf(kDrop ? p[r] * inv * km[r] : p[r] * inv);
    // A operand: V^T[row = dim d0 + i][k = key 4g + jj] = V[4g + jj][d0 + i]
    const uint16_t *vcol = base + 2 * h + hh * hd;
    uint16_t *orow = out + (b * 16 + i) * (int64_t)h + hh * hd;
    if (kAligned && hd == 16) {
        // V^T from V's row fragments (lane (i, g): V[i][4g..4g+3], one 8-byte load) by one MFMA
        // against the identity (exact) instead of four strided 2-byte loads per lane
        s16x4 eye;
#pragma unroll
        for (int r = 0; r < 4; r++) eye[r] = (short)(4 * g + r == i ? 0x3F80 : 0);
        const s16x4 vrow = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(vcol + (int64_t)i * (3 * h) + 4 * g));
        const f32x4 vt = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vrow, eye, f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
        const s16x4 va = __builtin_bit_cast(s16x4, make_uint2(pk2bf(vt[0], vt[1]), pk2bf(vt[2], vt[3])));
        const f32x4 o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, pb, f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
        *reinterpret_cast<uint2 *>(orow + 4 * g) = make_uint2(pk2bf(o[0], o[1]), pk2bf(o[2], o[3]));
        return;
    }
    for (int d0 = 0; d0 < hd; d0 += 16) {
        s16x4 va;
        const int d = d0 + i;
#pragma unroll
        for (int jj = 0; jj < 4; jj++)
            va[jj] = d < hd ? (short)vcol[(int64_t)(4 * g + jj) * (3 * h) + d] : (short)0;
        f32x4 o = {0.0f, 0.0f, 0.0f, 0.0f};
        o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, pb, o, 0, 0, 0);
        // lane (i, g): o[r] = O^T[d0 + 4g + r][i] = O[i][d0 + 4g + r]
        const int dd = d0 + 4 * g;
        if (kAligned) {
            if (dd < hd)
                *reinterpret_cast<uint2 *>(orow + dd) = make_uint2(pk2bf(o[0], o[1]),
                                                                   pk2bf(o[2], o[3]));
        } else {
#pragma unroll
            for (int r = 0; r < 4; r++)
                if (dd + r < hd) orow[dd + r] = f2bf(o[r]);
        }
    }
}

__global__ __launch_bounds__(kThreads) void urm_residual_rms_kernel(float *__restrict__ x,
                                                                    const uint16_t *__restrict__ y,
                                                                    const float *__restrict__ emb,
                                                                    uint16_t *__restrict__ xb, int64_t rows, int h,
                                                                    float eps) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (row >= rows) return;
    float v[kMaxPerLane];
    float ss = 0.0f;
#pragma unroll
    for (int j = 0; j < kMaxPerLane; j++) {
        const int c = lane + 64 * j;
        v[j] = 0.0f;
        if (c < h) v[j] = x[row * h + c] + bf2f(y[row * h + c]);
        ss += v[j] * v[j];
    }
    const float r = rsqrtf(wave_sum(ss) / (float)h + eps);
#pragma unroll
    for (int j = 0; j < kMaxPerLane; j++) {
        const int c = lane + 64 * j;
        if (c >= h) continue;
        float o = v[j] * r;
        if (emb) o += emb[row * h + c];
        x[row * h + c] = o;
        xb[row * h + c] = f2bf(o);
    }
}

// h <= 256: P = pow2 >= h / 4 lanes per row (4 consecutive columns each, 16-byte fp32 / 8-byte
// bf16 accesses), 64 / P rows per wave, the row reduction a P-lane butterfly
template <int P>
__global__ __launch_bounds__(kThreads) void urm_residual_rms_vec_kernel(float *__restrict__ x,
                                                                        const uint16_t *__restrict__ y,
                                                                        const float *__restrict__ emb,
                                                                        uint16_t *__restrict__ xb, int64_t rows, int h,
                                                                        float eps) {
    const int lane = threadIdx.x & 63, sub = lane & (P - 1);
    const int64_t row = ((int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6)) * (64 / P) + lane / P;
    const int c = 4 * sub;
    const bool on = row < rows && c < h;
    const int64_t o = row * h + c;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (on) {
        const float4 a = *reinterpret_cast<const float4 *>(x + o);
        const uint2 b = *reinterpret_cast<const uint2 *>(y + o);
        v = make_float4(a.x + bf2f(b.x & 0xFFFFu), a.y + bf2f(b.x >> 16), a.z + bf2f(b.y & 0xFFFFu), a.w + bf2f(b.y >> 16));
    }
    float ss = (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
#pragma unroll
    for (int s = P / 2; s > 0; s >>= 1) ss += __shfl_xor(ss, s, 64);
    const float r = rsqrtf(ss / (float)h + eps);
    if (!on) return;
    float4 out = make_float4(v.x * r, v.y * r, v.z * r, v.w * r);
    if (emb) {
        const float4 e = *reinterpret_cast<const float4 *>(emb + o);
        out = make_float4(out.x + e.x, out.y + e.y, out.z + e.z, out.w + e.w);
    }
    *reinterpret_cast<float4 *>(x + o) = out;
    *reinterpret_cast<uint2 *>(xb + o) = make_uint2(pk2bf(out.x, out.y),
                                                    pk2bf(out.z, out.w));
}

// two channels per thread (inter % 8 == 0): 4-byte bf16 pairs
__global__ __launch_bounds__(kThreads) void urm_swiglu_conv2_kernel(const uint16_t *__restrict__ gu,
                                                                    const float *__restrict__ w,
                                                                    const float *__restrict__ bias,
                                                                    uint16_t *__restrict__ out, int64_t n, int inter) {
    const int half = inter >> 1;
    const int64_t idx = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (idx >= n * half) return;
    const int64_t b = idx / half;
    const int c = 2 * (int)(idx - b * half);
    const float4 wc = *reinterpret_cast<const float4 *>(w + 2 * c);  // w[c][0], w[c][1], w[c+1][0], w[c+1][1]
    const float b0 = bias[c], b1 = bias[c + 1];
    float p0 = 0.0f, p1 = 0.0f;
    for (int t = 0; t < 16; t++) {
        const int64_t row = b * 16 + t;
        const uint32_t g2 = *reinterpret_cast<const uint32_t *>(gu + row * (2 * inter) + c);
        const uint32_t u2 = *reinterpret_cast<const uint32_t *>(gu + row * (2 * inter) + inter + c);
        const float a0 = silu(bf2f(g2 & 0xFFFFu)) * bf2f(u2 & 0xFFFFu);
        const float a1 = silu(bf2f(g2 >> 16)) * bf2f(u2 >> 16);
        const float c0 = fmaf(wc.y, a0, fmaf(wc.x, p0, b0)), c1 = fmaf(wc.w, a1, fmaf(wc.z, p1, b1));
        *reinterpret_cast<uint32_t *>(out + row * inter + c) = pk2bf(silu(c0), silu(c1));
        p0 = a0;
        p1 = a1;
    }
}

__global__ __launch_bounds__(kThreads) void urm_swiglu_conv_kernel(const uint16_t *__restrict__ gu,
                                                                   const float *__restrict__ w,
                                                                   const float *__restrict__ bias,
                                                                   uint16_t *__restrict__ out, int64_t n, int inter) {
    const int64_t idx = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (idx >= n * inter) return;
    const int64_t b = idx / inter;
    const int c = (int)(idx - b * inter);
    const float w0 = w[2 * c], w1 = w[2 * c + 1], bb = bias[c];
    float prev = 0.0f;
    for (int t = 0; t < 16; t++) {
        const int64_t row = b * 16 + t;
        const float gt = bf2f(gu[row * (2 * inter) + c]), ut = bf2f(gu[row * (2 * inter) + inter + c]);
        const float a = silu(gt) * ut;
        const float cv = fmaf(w1, a, fmaf(w0, prev, bb));
        out[row * inter + c] = f2bf(silu(cv));
        prev = a;
    }
}

__global__ __launch_bounds__(kThreads) void urm_pool_heads_kernel(const float *__restrict__ x,
                                                                  const float *__restrict__ wa,
                                                                  const float *__restrict__ ba,
                                                                  const float *__restrict__ wv,
                                                                  const float *__restrict__ bv,
                                                                  float *__restrict__ logits,
                                                                  float *__restrict__ value, int64_t n, int h) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (b >= n) return;
    float acc[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    for (int c = lane; c < h; c += 64) {
        float s = 0.0f;
        for (int t = 0; t < 16; t++) s += x[(b * 16 + t) * h + c];
        const float p = s / 16.0f;
#pragma unroll
        for (int k = 0; k < 4; k++) acc[k] = fmaf(p, wa[k * h + c], acc[k]);
        acc[4] = fmaf(p, wv[c], acc[4]);
    }
#pragma unroll
    for (int k = 0; k < 5; k++) acc[k] = wave_sum(acc[k]);
    if (lane < 4) logits[b * 4 + lane] = (lane == 0 ? acc[0] : lane == 1 ? acc[1] : lane == 2 ? acc[2] : acc[3]) + ba[lane];
    if (lane == 4) value[b] = acc[4] + bv[0];
}


// ---------------------------------------------------------------------------------------------
// Projections with their epilogues fused (h <= 64, the default GameURMConfig): Y^T = W X^T on
// v_mfma_f32_16x16x32_bf16 in the orientation of the MLP kernels -- a wave takes ONE board (its 16
// token rows are the 16 MFMA columns; B fragment = 16 contiguous bytes of a token row), W [N, K]
// is staged once per block in LDS (row pitch 16 KS + 4 dwords: conflict-free fragment reads), and
// the lane holding token t gets 4 consecutive output features of it per column tile:
//   EPI_STORE  qkv_proj:                    y bf16 [rows, N]
//   EPI_RMS    o_proj / down_proj:          x = rms_norm(x + y) [+ emb], xb = bf16(x) -- the row's
//              N features sit in the 4 lanes (g = 0..3) of token t: two cross-lane steps
//   EPI_SWIGLU gate_up_proj:                W's rows staged so gate feature c and up feature c land
//              in the same lane and register (tiles ct and ct + CT/2); a = SiLU(gate) * up, the
//              token t-1 value of the same channel from the lane one to the left within its
//              16-lane DPP row (row_shr:1; token 0 gets the conv's zero padding), then
//              SiLU(w0 a_{t-1} + w1 a_t + b) -> act bf16 [rows, inter]
// The projection outputs stay fp32 into the epilogue (no bf16 round trip through HBM).
//   EPI_SWIGLU_T the training variant (autograd GateUpSwiGLUFn): the gate / up accumulators are
//              rounded to bf16 and stored as gu [rows, 2 inter] (the backward's input, autocast's
//              gate_up output) and act follows urm_swiglu_conv_fwd's arithmetic on those rounded
//              values (y = bf16(bf16(silu(g)) u), act = bf16(silu(y_{t-1} w0 + y_t w1 + b))): the
//              gu round trip through HBM of the unfused path (GEMM write + SwiGLU read) is gone.
//   EPI_RMS_T  the training variant of EPI_RMS (autograd LinResRMSFn): a = bf16(x W^T) (autocast's
//              projection output), s = h + a with h read from `emb` (not written: autograd keeps it),
//              out = s rsqrt(mean(s^2) + eps) -> x (fp32), xb (bf16), rstd [rows] -- the projection's
//              bf16 output never round-trips through HBM.
enum { EPI_STORE = 0, EPI_RMS = 1, EPI_SWIGLU = 2, EPI_SWIGLU_T = 3, EPI_RMS_T = 4 };

__device__ __forceinline__ float dpp_prev_token(float v) {  // lane t-1 of the 16-lane row, 0 for t = 0
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xF, 0xF, false));
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// The staged W image of a projection with K <= 32 KS (round 5): rows unpadded with their 16-byte
// chunks XOR-swizzled by the row (mask SW) where that makes the fragment reads (lane (t, g): row
// 16 ct + t, chunk 4 s + g) conflict-free in every ds_read_b128 lane group (KS 2 / 6: mask 7, KS 4 /
// 8: mask 15); the other K keep the padded pitch 32 KS + 8.  Values unchanged: bitwise the same MFMAs.
template <int KS>
struct LinW {
    static constexpr int SW = (KS == 2 || KS == 6) ? 7 : (KS == 4 || KS == 8) ? 15 : 0;
    static constexpr int PITCH = SW ? 32 * KS : 32 * KS + 8;  // bf16 per staged row
    // byte offset of the 8-byte piece c4 (bf16 4 c4 .. + 3) of staged row q
    static __device__ __forceinline__ int piece(int q, int c4) {
        return q * PITCH * 2 + ((((c4 >> 1) ^ (q & SW)) << 4) | ((c4 & 1) << 3));
    }
    // byte offset of lane (t, g)'s A fragment of k-step s in the row block of tile 0
    static __device__ __forceinline__ int frag(int t, int g, int s) { return t * PITCH * 2 + (((4 * s + g) ^ (t & SW)) << 4); }
};

template <int KS, int CT, int EPI>
__global__ __launch_bounds__(kThreads) void urm_linear_kernel(const uint16_t *__restrict__ in,
                                                              const uint16_t *__restrict__ w, int64_t rows, int K,
                                                              int N, int inter, uint16_t *__restrict__ y,
                                                              float *__restrict__ x, const float *__restrict__ emb,
                                                              uint16_t *__restrict__ xb, float eps,
                                                              const float *__restrict__ cw_g,
                                                              const float *__restrict__ cb_g,
                                                              float *__restrict__ rstd, int wt) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int kPitch = LinW<KS>::PITCH;  // bf16 per staged row
    constexpr int kRowsW = 16 * CT;
    constexpr int kLinWBytes = kRowsW * kPitch * 2;
    // per-wave LDS tile of EPI_STORE: the 16-row bf16 output (staging the fp32 residual stream of
    // EPI_RMS the same way measured slower: 194 -> 213 us for o_proj)
    constexpr int kLinTileBytes = EPI == EPI_STORE ? 16 * (2 * 16 * CT + 8) : 0;
    constexpr bool kSwi = EPI == EPI_SWIGLU || EPI == EPI_SWIGLU_T;
    const int tid = threadIdx.x;
    for (int e = tid; e < kRowsW * kPitch / 8; e += kThreads) reinterpret_cast<uint4 *>(smem)[e] = make_uint4(0u, 0u, 0u, 0u);
    // the SwiGLU epilogues' conv taps w [inter][2] and biases [inter], staged once per block (zero past
    // inter): 16-byte LDS reads whatever the parameters' alignment in global memory (an optimizer may
    // re-home them into a flat buffer at any 4-byte offset)
    float *s_cw = reinterpret_cast<float *>(smem + kLinWBytes), *s_cb = s_cw + kRowsW;
    if constexpr (kSwi) {
        for (int e = tid; e < kRowsW / 2; e += kThreads) {
            const bool ok = e < inter;
            s_cw[2 * e] = ok ? cw_g[2 * e] : 0.0f;
            s_cw[2 * e + 1] = ok ? cw_g[2 * e + 1] : 0.0f;
            s_cb[e] = ok ? cb_g[e] : 0.0f;
        }
    }
    const float *cw = kSwi ? s_cw : cw_g, *cb = kSwi ? s_cb : cb_g;
    __syncthreads();
    if (wt) {  // w given as the [K, N] row-major matrix whose transpose is staged (dX = dY W, no W^T copy)
        for (int e = tid; e < N * (K >> 2); e += kThreads) {
            const int q = e % N, c4 = e / N;  // 4 consecutive k of output row q: 2-byte gathers of column q
            const uint16_t *src = w + (int64_t)(4 * c4) * N + q;
            const uint32_t lo = (uint32_t)src[0] | ((uint32_t)src[N] << 16);
            const uint32_t hi = (uint32_t)src[2 * N] | ((uint32_t)src[3 * N] << 16);
            *reinterpret_cast<uint2 *>(smem + LinW<KS>::piece(q, c4)) = make_uint2(lo, hi);
        }
    } else {   // staged row q <- W row src(q) (EPI_SWIGLU: gate rows at q < kRowsW / 2, up rows above)
        const int k4 = K >> 2;
        for (int e = tid; e < kRowsW * k4; e += kThreads) {
            const int q = e / k4, c4 = e - q * k4;
            int src = q;
            if (kSwi) {
                const int hq = q - kRowsW / 2;
                src = q < kRowsW / 2 ? (q < inter ? q : -1) : (hq < inter ? inter + hq : -1);
            } else if (q >= N) {
                src = -1;
            }
            if (src >= 0)
                *reinterpret_cast<uint2 *>(smem + LinW<KS>::piece(q, c4)) =
                    *reinterpret_cast<const uint2 *>(w + (int64_t)src * K + 4 * c4);
        }
    }
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6, t = lane & 15, g = lane >> 4;
    const int64_t boards = rows >> 4;
    int wo[KS];
#pragma unroll
    for (int s = 0; s < KS; s++) wo[s] = LinW<KS>::frag(t, g, s);
    // the board's B fragments (its 16 token rows of `in`), K % 4 == 0 with a 4-element tail
    auto load_b = [&](int64_t board, bf16x8 (&f)[KS]) {
        const uint16_t *xr = in + (board * 16 + t) * K;
#pragma unroll
        for (int s = 0; s < KS; s++) {
            const int kk = 32 * s + 8 * g;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (kk + 8 <= K) {
                v = *reinterpret_cast<const uint4 *>(xr + kk);
            } else if (kk < K) {
                const uint2 tl = *reinterpret_cast<const uint2 *>(xr + kk);
                v = make_uint4(tl.x, tl.y, 0u, 0u);
            }
            f[s] = __builtin_bit_cast(bf16x8, v);
        }
    };
    const int64_t bstride = (int64_t)gridDim.x * (kThreads / 64);
    int64_t bd = (int64_t)blockIdx.x * (kThreads / 64) + wave;
    bf16x8 fb[KS];
    if (bd < boards) load_b(bd, fb);
    for (; bd < boards; bd += bstride) {
        const int64_t r = bd * 16 + t;
        if constexpr (EPI == EPI_STORE) {
            if (bd != (int64_t)blockIdx.x * (kThreads / 64) + wave) load_b(bd, fb);  // (the first: above)
        }
        f32x4 acc[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ct++) acc[ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        bf16x8 fa[2][KS];
#pragma unroll
        for (int s = 0; s < KS; s++) fa[0][s] = *reinterpret_cast<const bf16x8 *>(smem + wo[s]);
#pragma unroll
        for (int ct = 0; ct < CT; ct++) {
            if (ct + 1 < CT) {
#pragma unroll
                for (int s = 0; s < KS; s++)
                    fa[(ct + 1) & 1][s] = *reinterpret_cast<const bf16x8 *>(smem + 16 * (ct + 1) * kPitch * 2 + wo[s]);
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int s = 0; s < KS; s++) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ct & 1][s], fb[s], acc[ct], 0, 0, 0);
        }
        // round 6: the next board's fragments are requested now, so their HBM latency runs under this
        // board's epilogue (each wave used to wait for its loads at the top of every board).  The
        // RMSNorm / SwiGLU epilogues gain (gate_up + SwiGLU-conv training 184.7 -> 170.9 us, o_proj /
        // down_proj -1.5 %); the plain store epilogue -- its LDS output tile, short epilogue -- lost 4 %
        // and keeps the loads at the top (profiles/r06j/ab_urm_linear.log)
        constexpr bool kPrefetch = EPI != EPI_STORE;
        if (kPrefetch && bd + bstride < boards) load_b(bd + bstride, fb);
        // lane (t, g), tile ct: acc[ct][i] = Y[r][16 ct + 4 g + i]
        if constexpr (EPI == EPI_STORE) {
            // the board's 16 x N outputs are one contiguous span of y: stage them in this wave's LDS
            // tile (row pitch N + 4 bf16) and write the span with 16-byte stores, instead of 16 rows
            // x 32-byte pieces per store instruction
            char *tile = smem + kLinWBytes + wave * kLinTileBytes;
            const int tp = 2 * N + 8;
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                const int c = 16 * ct + 4 * g;
                if (c < N) {
                    if (cw) {  // g2048_urm_linear_bias: the fp32 bias added before the single rounding
                        const float4 bv = *reinterpret_cast<const float4 *>(cw + c);
                        acc[ct][0] += bv.x;
                        acc[ct][1] += bv.y;
                        acc[ct][2] += bv.z;
                        acc[ct][3] += bv.w;
                    }
                    *reinterpret_cast<uint2 *>(tile + t * tp + 2 * c) =
                        make_uint2(pk2bf(acc[ct][0], acc[ct][1]),
                                   pk2bf(acc[ct][2], acc[ct][3]));
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            const int per_row = N >> 3;  // 16-byte chunks per row (N % 8 == 0)
            uint16_t *dst = y + bd * 16 * (int64_t)N;
            for (int q = lane; q < 16 * per_row; q += 64) {
                const int row = q / per_row, c8 = q - row * per_row;
                *reinterpret_cast<uint4 *>(dst + row * N + 8 * c8) = *reinterpret_cast<const uint4 *>(tile + row * tp + 16 * c8);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();  // the tile is rewritten by the next board
        } else if constexpr (EPI == EPI_RMS) {
            float ss = 0.0f;
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                const int c = 16 * ct + 4 * g;
                if (c < N) {
                    const float4 a = *reinterpret_cast<const float4 *>(x + r * N + c);
                    acc[ct][0] += a.x;
                    acc[ct][1] += a.y;
                    acc[ct][2] += a.z;
                    acc[ct][3] += a.w;
                    ss += (acc[ct][0] * acc[ct][0] + acc[ct][1] * acc[ct][1]) +
                          (acc[ct][2] * acc[ct][2] + acc[ct][3] * acc[ct][3]);
                }
            }
            ss += __shfl_xor(ss, 16, 64);
            ss += __shfl_xor(ss, 32, 64);
            const float rr = rsqrtf(ss / (float)N + eps);
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                const int c = 16 * ct + 4 * g;
                if (c < N) {
                    float4 o = make_float4(acc[ct][0] * rr, acc[ct][1] * rr, acc[ct][2] * rr, acc[ct][3] * rr);
                    if (emb) {
                        const float4 e = *reinterpret_cast<const float4 *>(emb + r * N + c);
                        o = make_float4(o.x + e.x, o.y + e.y, o.z + e.z, o.w + e.w);
                    }
                    *reinterpret_cast<float4 *>(x + r * N + c) = o;
                    *reinterpret_cast<uint2 *>(xb + r * N + c) =
                        make_uint2(pk2bf(o.x, o.y),
                                   pk2bf(o.z, o.w));
                }
            }
        } else if constexpr (EPI == EPI_RMS_T) {
            f32x4 sv[CT];
            float ss = 0.0f;
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                const int c = 16 * ct + 4 * g;
                sv[ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                if (c < N) {
                    const float4 hv = *reinterpret_cast<const float4 *>(emb + r * N + c);
                    sv[ct][0] = hv.x + (float)(__bf16)acc[ct][0];
                    sv[ct][1] = hv.y + (float)(__bf16)acc[ct][1];
                    sv[ct][2] = hv.z + (float)(__bf16)acc[ct][2];
                    sv[ct][3] = hv.w + (float)(__bf16)acc[ct][3];
                    ss += (sv[ct][0] * sv[ct][0] + sv[ct][1] * sv[ct][1]) + (sv[ct][2] * sv[ct][2] + sv[ct][3] * sv[ct][3]);
                }
            }
            ss = xsum32(xsum16(ss));
            const float rs = rsqrtf(ss * (1.0f / (float)N) + eps);
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                const int c = 16 * ct + 4 * g;
                if (c < N) {
                    const float4 o = make_float4(sv[ct][0] * rs, sv[ct][1] * rs, sv[ct][2] * rs, sv[ct][3] * rs);
                    *reinterpret_cast<float4 *>(x + r * N + c) = o;
                    if (xb) *reinterpret_cast<uint2 *>(xb + r * N + c) = make_uint2(pk2bf(o.x, o.y), pk2bf(o.z, o.w));
                }
            }
            if (g == 0) rstd[r] = rs;
        } else if constexpr (EPI == EPI_SWIGLU_T) {
            constexpr int CH = CT / 2;
            static_assert(CH % 2 == 0, "column tiles are stored in pairs");
            auto sg = [](float v) { return __builtin_amdgcn_rcpf(1.0f + __expf(-v)); };  // = sigm below
            auto rb = [](float v) { return (float)(__bf16)v; };
            auto pk = [](float a0, float a1, float a2, float a3) {
                const __attribute__((ext_vector_type(2))) __bf16 p0 = {(__bf16)a0, (__bf16)a1}, p1 = {(__bf16)a2, (__bf16)a3};
                return make_uint2(__builtin_bit_cast(uint32_t, p0), __builtin_bit_cast(uint32_t, p1));
            };
            // tiles ct, ct + 1 are stored together: lane (t, g) holds 4 features of each; one
            // v_permlane16_swap per dword between the lane rows g, g ^ 1 gives every lane 8
            // consecutive features (even g: 16 ct + 4 g .. + 7, odd g: 16 ct + 16 + 4 (g - 1) .. + 7),
            // so each output is written with 16-byte stores (half the store instructions)
            const int cb8 = (g & 1) ? 16 + 4 * (g - 1) : 4 * g;
#pragma unroll
            for (int cp = 0; cp < CH; cp += 2) {
                uint2 og[2], ou[2], oo[2];
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    const int ct = cp + j;
                    const int c = 16 * ct + 4 * g;
                    const int cc = c < inter ? c : 0;
                    const float4 w01 = *reinterpret_cast<const float4 *>(cw + 2 * cc);
                    const float4 w23 = *reinterpret_cast<const float4 *>(cw + 2 * cc + 4);
                    const float4 bb = *reinterpret_cast<const float4 *>(cb + cc);
                    const float wk0[4] = {w01.x, w01.z, w23.x, w23.z}, wk1[4] = {w01.y, w01.w, w23.y, w23.w};
                    const float bk[4] = {bb.x, bb.y, bb.z, bb.w};
                    float gq[4], uq[4], o[4];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        gq[i] = rb(acc[ct][i]);
                        uq[i] = rb(acc[ct + CH][i]);
                        const float yv = rb(rb(gq[i] * sg(gq[i])) * uq[i]);
                        const float prev = dpp_prev_token(yv);
                        const float z = prev * wk0[i] + yv * wk1[i] + bk[i];
                        o[i] = z * sg(z);
                    }
                    og[j] = pk(gq[0], gq[1], gq[2], gq[3]);
                    ou[j] = pk(uq[0], uq[1], uq[2], uq[3]);
                    oo[j] = pk(o[0], o[1], o[2], o[3]);
                }
                auto pair16 = [](const uint2 (&v)[2]) {
                    const auto sx = __builtin_amdgcn_permlane16_swap(v[0].x, v[1].x, false, false);
                    const auto sy = __builtin_amdgcn_permlane16_swap(v[0].y, v[1].y, false, false);
                    return make_uint4(sx[0], sy[0], sx[1], sy[1]);
                };
                const uint4 vg = pair16(og), vu = pair16(ou), vo = pair16(oo);
                const int c8 = 16 * cp + cb8;
                if (c8 < inter) {  // inter % 8 == 0: a lane's 8 features are all valid or all past inter
                    if (xb) {  // gu output (xb carries it; null: the no-grad loops, act only)
                        uint16_t *gr = xb + r * 2 * inter;
                        *reinterpret_cast<uint4 *>(gr + c8) = vg;
                        *reinterpret_cast<uint4 *>(gr + inter + c8) = vu;
                    }
                    *reinterpret_cast<uint4 *>(y + r * inter + c8) = vo;
                }
            }
        } else {
            constexpr int CH = CT / 2;
#pragma unroll
            for (int ct = 0; ct < CH; ct++) {
                const int c = 16 * ct + 4 * g;
                // the 4 channels' conv taps and biases: three 16-byte loads (inter % 4 == 0)
                const int cc = c < inter ? c : 0;
                const float4 w01 = *reinterpret_cast<const float4 *>(cw + 2 * cc);      // w[c][0..1], w[c+1][0..1]
                const float4 w23 = *reinterpret_cast<const float4 *>(cw + 2 * cc + 4);  // w[c+2][..], w[c+3][..]
                const float4 bb = *reinterpret_cast<const float4 *>(cb + cc);
                const float wk0[4] = {w01.x, w01.z, w23.x, w23.z}, wk1[4] = {w01.y, w01.w, w23.y, w23.w};
                const float bk[4] = {bb.x, bb.y, bb.z, bb.w};
                float o[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const float a = silu(acc[ct][i]) * acc[ct + CH][i];
                    const float prev = dpp_prev_token(a);
                    o[i] = silu(fmaf(wk1[i], a, fmaf(wk0[i], prev, bk[i])));
                }
                if (c < inter)
                    *reinterpret_cast<uint2 *>(y + r * inter + c) =
                        make_uint2(pk2bf(o[0], o[1]),
                                   pk2bf(o[2], o[3]));
            }
        }
    }
}

// (KS, CT) of a projection: K <= 32 KS, N (EPI_SWIGLU: 2 x 16 ceil(inter / 16)) <= 16 CT
struct LinShape {
    int ks, ct;
};
inline LinShape lin_shape(int K, int N, int inter, int epi) {
    const int ks = (K + 31) / 32;
    const int ct = (epi == EPI_SWIGLU || epi == EPI_SWIGLU_T) ? 2 * ((inter + 15) / 16) : (N + 15) / 16;
    return {ks, ct};
}

template <int KS, int CT, int EPI>
int launch_lin(hipStream_t s, const uint16_t *in, const uint16_t *w, int64_t rows, int K, int N, int inter,
               uint16_t *y, float *x, const float *emb, uint16_t *xb, float eps, const float *cw, const float *cb,
               float *rstd, int wt) {
    const size_t tile = EPI == EPI_STORE ? 16 * (2 * 16 * CT + 8) : 0;
    const size_t conv = (EPI == EPI_SWIGLU || EPI == EPI_SWIGLU_T) ? (size_t)16 * CT * 2 * 4 : 0;  // w + b per channel
    const size_t lds = (size_t)16 * CT * LinW<KS>::PITCH * 2 + std::max((size_t)(kThreads / 64) * tile, conv);
    int64_t grid = ((rows >> 4) + (kThreads / 64) - 1) / (kThreads / 64);
    // persistent over boards, W staged once per block.  The cap is per instance, from a sweep of
    // 512..3072 blocks at 65 536 boards (profiles/r06j/grid_sweep.log): the h 64 qkv forward is 17 %
    // faster at 768 (115.6 vs 138.6 us), the SwiGLU training epilogue that also stores gu 15 % faster
    // at 3072 (265.7 vs 313.0 us: more waves in flight for its two output streams); every other
    // instance is within noise of 1024.
    const int64_t cap = (EPI == EPI_STORE && CT == 12) ? 768 : (EPI == EPI_SWIGLU_T && xb) ? 3072 : 1024;
    grid = grid > cap ? cap : grid;
    hipLaunchKernelGGL((urm_linear_kernel<KS, CT, EPI>), dim3((unsigned)grid), dim3(kThreads), lds, s, in, w, rows, K, N,
                       inter, y, x, emb, xb, eps, cw, cb, rstd, wt);
    return launch_status();
}

// the instantiated shapes: GameURMConfig h = 64 (inter 120) and h = 32 (inter 64, the golden config)
int dispatch_lin(hipStream_t s, int epi, const uint16_t *in, const uint16_t *w, int64_t rows, int K, int N, int inter,
                 uint16_t *y, float *x, const float *emb, uint16_t *xb, float eps, const float *cw, const float *cb,
                 bool dry, float *rstd = nullptr, int wt = 0) {
    const LinShape sh = lin_shape(K, N, inter, epi);
#define G2048_LIN(EPI_, KS_, CT_)                                                                              \
    if (epi == EPI_ && sh.ks == KS_ && sh.ct == CT_)                                                            \
        return dry ? G2048_OK : launch_lin<KS_, CT_, EPI_>(s, in, w, rows, K, N, inter, y, x, emb, xb, eps, cw, cb, rstd, wt);
    G2048_LIN(EPI_STORE, 2, 12)   // h 64 qkv
    G2048_LIN(EPI_STORE, 1, 6)    // h 32 qkv
    // the training Functions' plain projections (URMLinearFn / GateUpSwiGLUFn): the forwards of
    // o_proj / down_proj and every input gradient dX = dY W, run as dY (W^T)^T with W^T staged
    G2048_LIN(EPI_STORE, 2, 4)    // h 64: o_proj fwd and dX (K 64, N 64)
    G2048_LIN(EPI_STORE, 4, 4)    // h 64: down_proj fwd (K 120, N 64)
    G2048_LIN(EPI_STORE, 6, 4)    // h 64: qkv dX (K 192, N 64)
    G2048_LIN(EPI_STORE, 2, 8)    // h 64: down_proj dX (K 64, N 120)
    G2048_LIN(EPI_STORE, 8, 4)    // h 64: gate_up dX (K 240, N 64)
    G2048_LIN(EPI_STORE, 1, 2)    // h 32: o_proj fwd and dX (K 32, N 32)
    G2048_LIN(EPI_STORE, 2, 2)    // h 32: down_proj fwd (K 64, N 32)
    G2048_LIN(EPI_STORE, 3, 2)    // h 32: qkv dX (K 96, N 32)
    G2048_LIN(EPI_STORE, 1, 4)    // h 32: down_proj dX (K 32, N 64)
    G2048_LIN(EPI_STORE, 4, 2)    // h 32: gate_up dX (K 128, N 32)
    G2048_LIN(EPI_STORE, 2, 1)    // h 64: the two heads [action | value | 0 pad] forward (K 64, N 8)
    G2048_LIN(EPI_STORE, 1, 1)    // h 32 heads forward (K 32, N 8)
    G2048_LIN(EPI_RMS, 2, 4)      // h 64 o_proj
    G2048_LIN(EPI_RMS, 4, 4)      // h 64 down_proj (K = inter = 120)
    G2048_LIN(EPI_RMS, 1, 2)      // h 32 o_proj
    G2048_LIN(EPI_RMS, 2, 2)      // h 32 down_proj (K = 64)
    G2048_LIN(EPI_RMS_T, 2, 4)    // h 64 o_proj, training (LinResRMSFn)
    G2048_LIN(EPI_RMS_T, 4, 4)    // h 64 down_proj, training
    G2048_LIN(EPI_RMS_T, 1, 2)    // h 32 o_proj, training
    G2048_LIN(EPI_RMS_T, 2, 2)    // h 32 down_proj, training
    G2048_LIN(EPI_SWIGLU, 2, 16)  // h 64 gate_up (inter 120 -> 2 x 8 tiles)
    G2048_LIN(EPI_SWIGLU, 1, 8)   // h 32 gate_up (inter 64)
    G2048_LIN(EPI_SWIGLU_T, 2, 16)  // training variants of the two
    G2048_LIN(EPI_SWIGLU_T, 1, 8)
#undef G2048_LIN
    return G2048_EINVAL;
}

// ---------------------------------------------------------------------------------------------
// The whole GameURM forward in ONE persistent kernel (the default config: h 64, 4 heads of 16,
// inter 120, conv kernel 2, 1 or 2 layers, any number of loops).  Nothing but obs in and
// logits / value out touches HBM: a wave carries one board (16 token lanes x 4 feature groups)
// through every block with the residual stream x and the stem output emb in registers (acc
// layout: lane (t, g) holds features 16 ct + 4 g + i of token t), and the workgroup streams the
// weights of the layer being applied through LDS:
//   per block application: __syncthreads, stage layer l's four bf16 matrices + conv taps (92 KB,
//   every weight row padded to a conflict-free pitch), __syncthreads, then per board:
//     qkv    12 tiles x 2 k-steps of v_mfma_f32_16x16x32_bf16 -> bf16 into the wave's LDS tile
//     attn   per head: S^T = K Q^T and O^T = V^T P^T on v_mfma_f32_16x16x16_bf16, K / Q / V read
//            from the tile (V transposed by the read), O written over its head's Q columns
//     o_proj 4 x 2 MFMAs + x, RMSNorm across the token's 4 lanes      -> x (registers), xb (tile)
//     gateup 16 x 2 MFMAs (gate / up of a channel in the same lane), SiLU * up, the token t-1
//            value by a DPP row shift, conv, SiLU                      -> act (tile)
//     down   4 x 4 MFMAs + x, RMSNorm [+ emb at the end of a loop]     -> x, xb
// The tile is the hand-off between the MFMA result layout and the next product's operand layout
// (16-byte fragment reads); wave-local s_waitcnt + wave barrier order the lanes' LDS accesses.
namespace mk {
constexpr int H = 64, QKV = 192, INTER = 120, GU = 256, KD = 128;
// Weight rows padded to 40 / 72 dwords = 10 / 18 16-byte units.  Round 5: a unit pitch of 2 x odd
// puts the 16 lanes of every ds_read_b128 lane group (rows {0-3, 12-15} of one column unit with rows
// 4-11 of the next, MI355X_MICROARCH.md's LDS table) on 16 distinct units, where round 4's 9 / 17
// units met two by two (SQ_LDS_BANK_CONFLICT 2.8 -> 1.0 cycles per LDS instruction, 2.31 -> 2.26 ms
// in tools/time_urm.py, profiles/r05al).  (Round 5 also measured the alternative: unpadded rows with their
// 16-byte chunks XOR-swizzled by the row, conflict-free fragment reads in every ds_read_b128 lane
// group by the bank model -- the forward got SLOWER, 2.23 -> 2.36 ms per 65 536 boards: the LDS
// conflicts are not what bounds it at two waves per SIMD, the extra addressing registers spilled.)
#ifndef G2048_URM_WPAD
#define G2048_URM_WPAD 16
#endif
#ifndef G2048_URM_TPAD
#define G2048_URM_TPAD 8
#endif
constexpr int P64 = H + G2048_URM_WPAD;     // bf16 pitch of K = 64 weight rows
constexpr int PD = KD + G2048_URM_WPAD;     // bf16 pitch of the down-proj rows
constexpr int OFF_QKV = 0;
constexpr int OFF_O = OFF_QKV + QKV * P64 * 2;
constexpr int OFF_GU = OFF_O + H * P64 * 2;
constexpr int OFF_D = OFF_GU + GU * P64 * 2;
constexpr int OFF_CW = OFF_D + H * PD * 2;       // conv taps fp32 [128][2]
constexpr int OFF_CB = OFF_CW + KD * 2 * 4;      // conv bias fp32 [128]
constexpr int W_BYTES = OFF_CB + KD * 4;         // 92 672
constexpr int TP = QKV + G2048_URM_TPAD;         // bf16 pitch of a wave's tile (100 dwords)
constexpr int TILE_BYTES = 16 * TP * 2;          // 6 400
constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;
// small fp32 parameters staged once per kernel (lane-relative LDS offsets instead of dozens of
// per-lane 64-bit global addresses held in registers)
constexpr int PS_STEM = 0, PS_LNW = PS_STEM + 3 * H, PS_LNB = PS_LNW + H, PS_INIT = PS_LNB + H,
              PS_WA = PS_INIT + 16 * H, PS_WV = PS_WA + 4 * H, PS_BA = PS_WV + H, PS_BV = PS_BA + 4,
              PS_ALL = PS_BV + 4;
static_assert(W_BYTES + WAVES * TILE_BYTES + PS_ALL * 4 <= 163840, "one workgroup's LDS");
#ifndef G2048_URM_RCP
#define G2048_URM_RCP 1
#endif
#ifndef G2048_URM_PK
#define G2048_URM_PK 1
#endif
#ifndef G2048_URM_PK_RMS
#define G2048_URM_PK_RMS G2048_URM_PK
#endif
#ifndef G2048_URM_STAGE_OPAQUE
#define G2048_URM_STAGE_OPAQUE 1
#endif
#ifndef G2048_URM_NB
#define G2048_URM_NB 2
#endif
constexpr int NB = G2048_URM_NB;                 // boards per wave per batch (unrolled)
}  // namespace mk

struct UrmW {  // device pointers (see g2048_urm_weights)
    const float *stem_w, *ln_w, *ln_b, *init, *wa, *ba, *wv, *bv;
    const uint16_t *qkv[2], *o[2], *gu[2], *dn[2];
    const float *cw[2], *cb[2];
    int layers, loops;
    float eps;
    AttnDrop drop;  // thr == 0: no attention dropout; else block application `app` uses counter *counter + app
};

__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// 16 B (8 bf16) from LDS
__device__ __forceinline__ bf16x8 lds16(const char *p) { return *reinterpret_cast<const bf16x8 *>(p); }

// acc-layout values (4 per tile) -> bf16 in the tile at [t][16 ct + 4 g].  Round 5: 16-byte stores,
// tiles ct, ct + 1 paired by one v_permlane16_swap per dword between the lane rows g, g ^ 1 (lane g
// even then holds columns 16 ct + 4 g .. + 7, lane g odd 16 (ct + 1) + 4 (g - 1) .. + 7; mlp_tile.hpp
// store_row16): half the store instructions, and the 8 lanes of a ds_write_b128 group (8 rows, one
// column unit) fall on distinct banks at the 100-dword tile pitch, where the 16 same-column lanes
// of a ds_write_b64 group met two by two (the forward's LDS conflict cycles 1.0 -> 0.4 per LDS
// instruction)
template <int CT>
__device__ __forceinline__ void tile_put(char *tile, const f32x4 (&v)[CT], int t, int g, int col0 = 0) {
    static_assert(CT % 2 == 0, "column tiles are stored in pairs");
    char *p = tile + (t * mk::TP + col0) * 2;
    const int cb = (g & 1) ? 16 + 4 * (g - 1) : 4 * g;
#pragma unroll
    for (int ct = 0; ct < CT; ct += 2) {
        const auto sx = __builtin_amdgcn_permlane16_swap(pk2bf(v[ct][0], v[ct][1]), pk2bf(v[ct + 1][0], v[ct + 1][1]), false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(pk2bf(v[ct][2], v[ct][3]), pk2bf(v[ct + 1][2], v[ct + 1][3]), false, false);
        *reinterpret_cast<uint4 *>(p + 2 * (16 * ct + cb)) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
    }
}

// acc[CT] = W X^T for the board in `tile` (B fragments [t][32 s + 8 g]); W rows at `w` with pitch
// `pitch` bf16 (A fragments [16 ct + t][32 s + 8 g])
template <int CT, int KS>
__device__ __forceinline__ void tile_gemm(f32x4 (&acc)[CT], const char *w, int pitch, const char *tile, int t, int g) {
    bf16x8 fb[KS], fa[2][KS];
#pragma unroll
    for (int s = 0; s < KS; s++) fb[s] = lds16(tile + (t * mk::TP + 32 * s + 8 * g) * 2);
    const char *wb = w + (t * pitch + 8 * g) * 2;
#pragma unroll
    for (int s = 0; s < KS; s++) fa[0][s] = lds16(wb + 64 * s);
    // W fragments one tile ahead; the empty asm keeps the compiler from hoisting every tile's
    // reads (the register file would spill)
#pragma unroll
    for (int ct = 0; ct < CT; ct++) {
        if (ct + 1 < CT) {
#pragma unroll
            for (int s = 0; s < KS; s++) fa[(ct + 1) & 1][s] = lds16(wb + 16 * (ct + 1) * pitch * 2 + 64 * s);
        }
        asm volatile("" ::: "memory");
        acc[ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < KS; s++) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ct & 1][s], fb[s], acc[ct], 0, 0, 0);
    }
}

// the same with the B fragments already in registers
template <int CT, int KS>
__device__ __forceinline__ void frag_gemm(f32x4 (&acc)[CT], const char *w, int pitch, const bf16x8 (&fb)[KS], int t,
                                          int g) {
    bf16x8 fa[2][KS];
    const char *wb = w + (t * pitch + 8 * g) * 2;
#pragma unroll
    for (int s = 0; s < KS; s++) fa[0][s] = lds16(wb + 64 * s);
#pragma unroll
    for (int ct = 0; ct < CT; ct++) {
        if (ct + 1 < CT) {
#pragma unroll
            for (int s = 0; s < KS; s++) fa[(ct + 1) & 1][s] = lds16(wb + 16 * (ct + 1) * pitch * 2 + 64 * s);
        }
        asm volatile("" ::: "memory");
        acc[ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < KS; s++) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ct & 1][s], fb[s], acc[ct], 0, 0, 0);
    }
}

// x = rms_norm(x + y) [+ emb]  (the token's 64 features in 4 lanes x 16 values)
__device__ __forceinline__ void rms_update(f32x4 (&x)[4], const f32x4 (&y)[4], const f32x4 (&emb)[4], bool add_emb,
                                           float eps) {
#if G2048_URM_PK_RMS
    // round 5: feature pairs on packed adds / fmas (the sum of squares as two interleaved partial sums)
    f32x2 s2 = {0.0f, 0.0f};
#pragma unroll
    for (int ct = 0; ct < 4; ct++)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
            const f32x2 v = f32x2{x[ct][i], x[ct][i + 1]} + f32x2{y[ct][i], y[ct][i + 1]};
            x[ct][i] = v.x;
            x[ct][i + 1] = v.y;
            s2 = __builtin_elementwise_fma(v, v, s2);
        }
    const float ss = xsum32(xsum16(s2.x + s2.y));
    const float r = rsqrtf(ss * (1.0f / mk::H) + eps);
#pragma unroll
    for (int ct = 0; ct < 4; ct++)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
            const f32x2 e = add_emb ? f32x2{emb[ct][i], emb[ct][i + 1]} : f32x2{0.0f, 0.0f};
            const f32x2 v = __builtin_elementwise_fma(f32x2{x[ct][i], x[ct][i + 1]}, f32x2{r, r}, e);
            x[ct][i] = v.x;
            x[ct][i + 1] = v.y;
        }
#else
    float ss = 0.0f;
#pragma unroll
    for (int ct = 0; ct < 4; ct++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            x[ct][i] += y[ct][i];
            ss += x[ct][i] * x[ct][i];
        }
    ss = xsum32(xsum16(ss));
    const float r = rsqrtf(ss * (1.0f / mk::H) + eps);
#pragma unroll
    for (int ct = 0; ct < 4; ct++)
#pragma unroll
        for (int i = 0; i < 4; i++) x[ct][i] = x[ct][i] * r + (add_emb ? emb[ct][i] : 0.0f);
#endif
}

template <bool kBf16Obs, bool kDrop>
__global__ __launch_bounds__(mk::THREADS) void urm_forward_kernel(const void *__restrict__ obs, UrmW W,
                                                                  float *__restrict__ logits,
                                                                  float *__restrict__ value, int64_t n) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, t = lane & 15, g = lane >> 4;
    char *tile = smem + mk::W_BYTES + wave * mk::TILE_BYTES;
    float *par = reinterpret_cast<float *>(smem + mk::W_BYTES + mk::WAVES * mk::TILE_BYTES);
    {
        auto put = [&](int off, const float *src, int cnt) {
            for (int e = tid; e < cnt; e += mk::THREADS) par[off + e] = src[e];
        };
        put(mk::PS_STEM, W.stem_w, 3 * mk::H);
        put(mk::PS_LNW, W.ln_w, mk::H);
        put(mk::PS_LNB, W.ln_b, mk::H);
        put(mk::PS_INIT, W.init, 16 * mk::H);
        put(mk::PS_WA, W.wa, 4 * mk::H);
        put(mk::PS_WV, W.wv, mk::H);
        put(mk::PS_BA, W.ba, 4);
        put(mk::PS_BV, W.bv, 1);
    }
    const float *cwl = reinterpret_cast<const float *>(smem + mk::OFF_CW);
    const float *cbl = reinterpret_cast<const float *>(smem + mk::OFF_CB);
    const int64_t per_batch = (int64_t)mk::WAVES * mk::NB;
    const int64_t batches = (n + per_batch - 1) / per_batch;
    const int apps = W.layers * W.loops;
    const uint64_t drop_c0 = kDrop ? *W.drop.counter : 0ull;  // attention dropout (training-mode forward)
    for (int e = tid; e < mk::W_BYTES / 16; e += mk::THREADS) reinterpret_cast<uint4 *>(smem)[e] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();  // the parameters and the zeroed padding are read by every wave
    for (int64_t bt = blockIdx.x; bt < batches; bt += gridDim.x) {
        f32x4 x[mk::NB][4], emb[mk::NB][4];
        // ---- stem: emb = SiLU(LayerNorm(Linear(3 -> 64)(cells))), x = init_hidden + emb
#pragma unroll
        for (int nb = 0; nb < mk::NB; nb++) {
            int64_t b = bt * per_batch + wave * mk::NB + nb;
            b = b < n ? b : n - 1;
            float c[3];
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const int64_t o = b * 48 + 3 * t + k;
                c[k] = kBf16Obs ? bf2f(static_cast<const uint16_t *>(obs)[o]) : static_cast<const float *>(obs)[o];
            }
            float s = 0.0f;
#pragma unroll
            for (int ct = 0; ct < 4; ct++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int f = 16 * ct + 4 * g + i;
                    const float *sw = par + mk::PS_STEM + 3 * f;
                    const float y = fmaf(sw[2], c[2], fmaf(sw[1], c[1], sw[0] * c[0]));
                    emb[nb][ct][i] = y;
                    s += y;
                }
            s = xsum32(xsum16(s));
            const float mean = s * (1.0f / mk::H);
            float v = 0.0f;
#pragma unroll
            for (int ct = 0; ct < 4; ct++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const float d = emb[nb][ct][i] - mean;
                    v += d * d;
                }
            v = xsum32(xsum16(v));
            const float rstd = rsqrtf(v * (1.0f / mk::H) + 1e-5f);
#pragma unroll
            for (int ct = 0; ct < 4; ct++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int f = 16 * ct + 4 * g + i;
                    const float e = silu((emb[nb][ct][i] - mean) * rstd * par[mk::PS_LNW + f] + par[mk::PS_LNB + f]);
                    emb[nb][ct][i] = e;
                    x[nb][ct][i] = par[mk::PS_INIT + t * mk::H + f] + e;
                }
        }
        for (int app = 0; app < apps; app++) {
            const int l = app % W.layers;
            const bool loop_end = (l == W.layers - 1) && (app < apps - 1);
            if (app < W.layers || W.layers > 1) {  // (re)stage layer l's weights
                __syncthreads();
                // one flat list of 16-byte chunks (4 matrices + conv taps / bias), every load of a
                // thread in flight before its LDS writes: one L2 round trip per staging.  Padding
                // rows / columns were zeroed once and are never written.
                constexpr int C_QKV = mk::QKV * 8, C_O = mk::H * 8, C_GU = 2 * mk::INTER * 8, C_D = mk::H * 15;
                constexpr int C_CW = mk::INTER * 2 / 4, C_CB = mk::INTER / 4;
                constexpr int C_ALL = C_QKV + C_O + C_GU + C_D + C_CW + C_CB;
                constexpr int PER = (C_ALL + mk::THREADS - 1) / mk::THREADS;
                uint4 v[PER];
                int dst[PER];
#if G2048_URM_STAGE_OPAQUE
                // an opaque per-staging copy of the thread index: the chunks' source offsets are then
                // recomputed here (a few VALU each) instead of hoisted out of the batch loop, spilled
                // to scratch and reloaded one vmcnt(0) wait at a time (which serialised the loads)
                int tid_s = tid;
                asm volatile("" : "+v"(tid_s));
#else
                const int tid_s = tid;
#endif
#pragma unroll
                for (int u = 0; u < PER; u++) {
                    int e = tid_s + u * mk::THREADS;
                    const char *src = nullptr;
                    int d = -1;
                    if (e < C_QKV) {
                        src = reinterpret_cast<const char *>(W.qkv[l]) + 16 * e;
                        d = mk::OFF_QKV + (e >> 3) * mk::P64 * 2 + 16 * (e & 7);
                    } else if ((e -= C_QKV) < C_O) {
                        src = reinterpret_cast<const char *>(W.o[l]) + 16 * e;
                        d = mk::OFF_O + (e >> 3) * mk::P64 * 2 + 16 * (e & 7);
                    } else if ((e -= C_O) < C_GU) {
                        const int r = e >> 3;
                        src = reinterpret_cast<const char *>(W.gu[l]) + 16 * e;
                        d = mk::OFF_GU + (r < mk::INTER ? r : r + 8) * mk::P64 * 2 + 16 * (e & 7);
                    } else if ((e -= C_GU) < C_D) {
                        const int r = e / 15, c = e - 15 * r;
                        src = reinterpret_cast<const char *>(W.dn[l]) + 16 * e;
                        d = mk::OFF_D + r * mk::PD * 2 + 16 * c;
                    } else if ((e -= C_D) < C_CW) {
                        src = reinterpret_cast<const char *>(W.cw[l]) + 16 * e;
                        d = mk::OFF_CW + 16 * e;
                    } else if ((e -= C_CW) < C_CB) {
                        src = reinterpret_cast<const char *>(W.cb[l]) + 16 * e;
                        d = mk::OFF_CB + 16 * e;
                    }
                    v[u] = src ? *reinterpret_cast<const uint4 *>(src) : make_uint4(0u, 0u, 0u, 0u);
                    dst[u] = d;
                }
#pragma unroll
                for (int u = 0; u < PER; u++)
                    if (dst[u] >= 0) *reinterpret_cast<uint4 *>(smem + dst[u]) = v[u];
                __syncthreads();
            }
#pragma unroll
            for (int nb = 0; nb < mk::NB; nb++) {
                f32x4 *xr = x[nb];
                // xb -> tile, qkv
                tile_put<4>(tile, reinterpret_cast<const f32x4(&)[4]>(*xr), t, g);
                wave_lds_sync();
                {   // qkv in three 64-feature chunks (16 accumulators live), xb fragments held in registers
                    bf16x8 fb[2];
                    fb[0] = lds16(tile + (t * mk::TP + 8 * g) * 2);
                    fb[1] = lds16(tile + (t * mk::TP + 32 + 8 * g) * 2);
                    wave_lds_sync();
#pragma unroll
                    for (int c = 0; c < 3; c++) {
                        f32x4 q[4];
                        frag_gemm<4, 2>(q, smem + mk::OFF_QKV + 64 * c * mk::P64 * 2, mk::P64, fb, t, g);
                        tile_put<4>(tile, q, t, g, 64 * c);
                    }
                    wave_lds_sync();
                }
                // attention, per head: O over the head's Q columns
#pragma unroll 1
                for (int hh = 0; hh < 4; hh++) {
                    const s16x4 ka = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(tile + (t * mk::TP + 64 + 16 * hh + 4 * g) * 2));
                    const s16x4 qb = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(tile + (t * mk::TP + 16 * hh + 4 * g) * 2));
                    s16x4 va;
#pragma unroll
                    for (int jj = 0; jj < 4; jj++)
                        va[jj] = *reinterpret_cast<const short *>(tile + ((4 * g + jj) * mk::TP + 128 + 16 * hh + t) * 2);
                    f32x4 st = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ka, qb, f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
                    float p[4], m = -INFINITY;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        p[r] = st[r] * 0.25f;  // 1 / sqrt(head_dim 16)
                        m = fmaxf(m, p[r]);
                    }
                    m = xmax32(xmax16(m));
                    float sum = 0.0f;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        p[r] = __expf(p[r] - m);
                        sum += p[r];
                    }
                    sum = xsum32(xsum16(sum));
#if G2048_URM_RCP
                    const float inv = __builtin_amdgcn_rcpf(sum);  // v_rcp_f32 (1 ulp) instead of the IEEE division sequence
#else
                    const float inv = 1.0f / sum;
#endif
                    s16x4 pb;
                    if constexpr (kDrop) {  // the mask of URMAttentionFn at counter c0 + app
                        float km[4];
                        int64_t b = bt * per_batch + wave * mk::NB + nb;
                        b = b < n ? b : n - 1;
                        attn_keep_c(W.drop, drop_c0 + (uint64_t)app, b, hh, t, g, km);
                        pb = __builtin_bit_cast(s16x4, make_uint2(pk2bf(p[0] * inv * km[0], p[1] * inv * km[1]),
                                                                  pk2bf(p[2] * inv * km[2], p[3] * inv * km[3])));
                    } else {
                        pb = __builtin_bit_cast(s16x4, make_uint2(pk2bf(p[0] * inv, p[1] * inv), pk2bf(p[2] * inv, p[3] * inv)));
                    }
                    const f32x4 o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, pb, f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
                    wave_lds_sync();  // every lane's Q / K / V reads of this head are done
                    *reinterpret_cast<uint2 *>(tile + (t * mk::TP + 16 * hh + 4 * g) * 2) =
                        make_uint2(pk2bf(o[0], o[1]),
                                   pk2bf(o[2], o[3]));
                }
                wave_lds_sync();
                {   // o_proj + residual + RMSNorm
                    f32x4 y[4];
                    tile_gemm<4, 2>(y, smem + mk::OFF_O, mk::P64, tile, t, g);
                    rms_update(reinterpret_cast<f32x4(&)[4]>(*xr), y, reinterpret_cast<const f32x4(&)[4]>(*emb[nb]), false, W.eps);
                }
                wave_lds_sync();
                tile_put<4>(tile, reinterpret_cast<const f32x4(&)[4]>(*xr), t, g);
                wave_lds_sync();
                {   // gate_up + SwiGLU + depthwise conv + SiLU -> act (bf16, 128 columns); the gate and up
                    // tiles of a channel group are produced together, so only 8 accumulators are live
                    bf16x8 fb[2];
                    fb[0] = lds16(tile + (t * mk::TP + 8 * g) * 2);
                    fb[1] = lds16(tile + (t * mk::TP + 32 + 8 * g) * 2);
                    const char *wb = smem + mk::OFF_GU + (t * mk::P64 + 8 * g) * 2;
                    f32x4 a[8];
#pragma unroll
                    for (int ct = 0; ct < 8; ct++) {
                        f32x4 ga = f32x4{0.0f, 0.0f, 0.0f, 0.0f}, up = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                        for (int s2 = 0; s2 < 2; s2++) {
                            ga = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds16(wb + (16 * ct * mk::P64 + 32 * s2) * 2), fb[s2], ga, 0, 0, 0);
                            up = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds16(wb + (16 * (ct + 8) * mk::P64 + 32 * s2) * 2), fb[s2], up, 0, 0, 0);
                        }
                        asm volatile("" ::: "memory");
                        const int c = 16 * ct + 4 * g;
                        const float4 w01 = *reinterpret_cast<const float4 *>(cwl + 2 * c);
                        const float4 w23 = *reinterpret_cast<const float4 *>(cwl + 2 * c + 4);
                        const float4 bb = *reinterpret_cast<const float4 *>(cbl + c);
                        const float wk0[4] = {w01.x, w01.z, w23.x, w23.z}, wk1[4] = {w01.y, w01.w, w23.y, w23.w};
                        const float bk[4] = {bb.x, bb.y, bb.z, bb.w};
#if G2048_URM_PK
                        // the same arithmetic on feature pairs: packed multiplies / adds / fmas around the
                        // per-element exp2 / rcp (bitwise the scalar form: silu2)
                        float av[4], prev[4];
#pragma unroll
                        for (int i = 0; i < 4; i += 2) {
                            const f32x2 y = silu2(f32x2{ga[i], ga[i + 1]}) * f32x2{up[i], up[i + 1]};
                            av[i] = y.x;
                            av[i + 1] = y.y;
                        }
#pragma unroll
                        for (int i = 0; i < 4; i++) prev[i] = dpp_prev_token(av[i]);
#pragma unroll
                        for (int i = 0; i < 4; i += 2) {
                            const f32x2 z = __builtin_elementwise_fma(f32x2{wk1[i], wk1[i + 1]}, f32x2{av[i], av[i + 1]},
                                                                      __builtin_elementwise_fma(f32x2{wk0[i], wk0[i + 1]},
                                                                                                f32x2{prev[i], prev[i + 1]},
                                                                                                f32x2{bk[i], bk[i + 1]}));
                            const f32x2 o = silu2(z);
                            a[ct][i] = c + i < mk::INTER ? o.x : 0.0f;
                            a[ct][i + 1] = c + i + 1 < mk::INTER ? o.y : 0.0f;
                        }
#else
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const float av = silu(ga[i]) * up[i];
                            const float prev = dpp_prev_token(av);
                            a[ct][i] = c + i < mk::INTER ? silu(fmaf(wk1[i], av, fmaf(wk0[i], prev, bk[i]))) : 0.0f;
                        }
#endif
                    }
                    wave_lds_sync();
                    tile_put<8>(tile, a, t, g);
                    wave_lds_sync();
                }
                {   // down_proj + residual + RMSNorm [+ emb]
                    f32x4 y[4];
                    tile_gemm<4, 4>(y, smem + mk::OFF_D, mk::PD, tile, t, g);
                    rms_update(reinterpret_cast<f32x4(&)[4]>(*xr), y, reinterpret_cast<const f32x4(&)[4]>(*emb[nb]), loop_end, W.eps);
                }
                wave_lds_sync();
            }
        }
        // ---- mean over the 16 tokens, heads
#pragma unroll
        for (int nb = 0; nb < mk::NB; nb++) {
            const int64_t b = bt * per_batch + wave * mk::NB + nb;
            float acc5[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int ct = 0; ct < 4; ct++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    float pv = x[nb][ct][i];
                    pv += __shfl_xor(pv, 1, 64);
                    pv += __shfl_xor(pv, 2, 64);
                    pv += __shfl_xor(pv, 4, 64);
                    pv += __shfl_xor(pv, 8, 64);
                    pv *= 1.0f / 16.0f;
                    const int f = 16 * ct + 4 * g + i;
#pragma unroll
                    for (int k = 0; k < 4; k++) acc5[k] = fmaf(pv, par[mk::PS_WA + k * mk::H + f], acc5[k]);
                    acc5[4] = fmaf(pv, par[mk::PS_WV + f], acc5[4]);
                }
#pragma unroll
            for (int k = 0; k < 5; k++) {
                acc5[k] = xsum32(xsum16(acc5[k]));
            }
            if (b < n && lane == 0) {
#pragma unroll
                for (int k = 0; k < 4; k++) logits[b * 4 + k] = acc5[k] + par[mk::PS_BA + k];
                value[b] = acc5[4] + par[mk::PS_BV];
            }
        }
    }
}
// Backward of the attention core for head_dim 16 (the default GameURM: h 64, 4 heads), one wave
// per (board, head), for training through autograd (agent.GameURMAttention), on
// v_mfma_f32_16x16x16_bf16 (round 4; the fp32 VALU version read its operands ~400 times per lane
// from LDS and was LDS-bound at ~400 us per call).  Lane (t, g) = (l & 15, l >> 4) loads the 4
// features 4g..4g+3 of head hd of token t of q, k, v and dO -- the A layout of a 16 x 16 operand with
// the token as its row, and the B layout of its transpose.  Then
//   S^T  = K Q^T              lane (i, g) holds S[i][4g + r]: the forward's product, bit for bit,
//                             and its softmax code, so P is the forward's P
//   dP^T = V dO^T             same layout: dP[i][4g + r]  (dP = dO V^T of the dropped P)
//   dS   = P (km dP - rowsum(P km dP))          elementwise + two cross-lane steps
//   dQ^T = K^T dS^T,  dK^T = Q^T dS,  dV^T = dO^T (P km)   each leaves lane (t, g) the features
//                             4g..4g+3 of token t's gradient (one 8-byte store per output)
// The transposed operands (K^T, Q^T, dO^T as A; dS, P km as B with the query as K index) are ONE
// MFMA each against the identity (exact: bf16 values times 1 accumulated in fp32).  P and dS enter
// their products as bf16 (torch's bf16 autocast backward of the same attention does the same).
template <bool kDrop>
__global__ __launch_bounds__(256) void urm_attn_bwd16_kernel(const uint16_t *__restrict__ qkv,
                                                             const uint16_t *__restrict__ dout,
                                                             uint16_t *__restrict__ dqkv, int64_t tasks, int h,
                                                             int heads, AttnDrop drop) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t task = (int64_t)blockIdx.x * 4 + wave;
    if (task >= tasks) return;  // wave-uniform; no block barrier below
    const int64_t b = task / heads;
    const int hd = (int)(task - b * heads);
    const int t = lane & 15, g = lane >> 4;
    const int64_t tok = 16 * b + t;
    const uint16_t *row = qkv + tok * 3 * h + hd * 16 + 4 * g;
    const s16x4 qa = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(row));
    const s16x4 ka = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(row + h));
    const s16x4 va = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(row + 2 * h));
    const s16x4 oa = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(dout + tok * h + hd * 16 + 4 * g));
    s16x4 eye;  // B operand identity: lane (n, g) holds I[4g + r][n]
#pragma unroll
    for (int r = 0; r < 4; r++) eye[r] = (short)(4 * g + r == t ? 0x3F80 : 0);
    const f32x4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
    auto pack4 = [](float a0, float a1, float a2, float a3) {
        return __builtin_bit_cast(s16x4, make_uint2(pk2bf(a0, a1), pk2bf(a2, a3)));
    };
    auto tr = [&](s16x4 x) {  // A-layout operand -> its transpose's A layout (= its own B layout)
        const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x, eye, zero, 0, 0, 0);
        return pack4(d[0], d[1], d[2], d[3]);
    };
    // P = softmax(Q K^T / 4), exactly urm_attn_kernel's arithmetic
    const f32x4 st = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ka, qa, zero, 0, 0, 0);
    const float scale = 0.25f;  // 1 / sqrt(16), scaled_dot_product_attention's default
    float p[4];
    float m = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        p[r] = st[r] * scale;
        m = fmaxf(m, p[r]);
    }
    m = xmax32(xmax16(m));  // = the forward's two xor shuffles (max / + are commutative)
    float sum = 0.0f;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        p[r] = __expf(p[r] - m);
        sum += p[r];
    }
    sum = xsum32(xsum16(sum));
    const float inv = 1.0f / sum;
#pragma unroll
    for (int r = 0; r < 4; r++) p[r] *= inv;
    // dropout: O = Pd V with Pd = P km (the forward's mask, regenerated); dV = Pd^T dO and
    // dS = P (km dPd - rowsum(Pd dPd)), dPd = dO V^T
    float km[4] = {1.0f, 1.0f, 1.0f, 1.0f};
    if (kDrop) attn_keep(drop, b, hd, t, g, km);
    const f32x4 dp = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, oa, zero, 0, 0, 0);
    float rs = (p[0] * km[0] * dp[0] + p[1] * km[1] * dp[1]) + (p[2] * km[2] * dp[2] + p[3] * km[3] * dp[3]);
    rs = xsum32(xsum16(rs));
    const s16x4 dsa = pack4(p[0] * (dp[0] * km[0] - rs), p[1] * (dp[1] * km[1] - rs), p[2] * (dp[2] * km[2] - rs),
                            p[3] * (dp[3] * km[3] - rs));
    const s16x4 pda = pack4(p[0] * km[0], p[1] * km[1], p[2] * km[2], p[3] * km[3]);
    const f32x4 dq = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(tr(ka), dsa, zero, 0, 0, 0);
    const f32x4 dk = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(tr(qa), tr(dsa), zero, 0, 0, 0);
    const f32x4 dv = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(tr(oa), tr(pda), zero, 0, 0, 0);
    uint16_t *drow = dqkv + tok * 3 * h + hd * 16 + 4 * g;
    *reinterpret_cast<uint2 *>(drow) = make_uint2(pk2bf(dq[0] * scale, dq[1] * scale), pk2bf(dq[2] * scale, dq[3] * scale));
    *reinterpret_cast<uint2 *>(drow + h) = make_uint2(pk2bf(dk[0] * scale, dk[1] * scale), pk2bf(dk[2] * scale, dk[3] * scale));
    *reinterpret_cast<uint2 *>(drow + 2 * h) = make_uint2(pk2bf(dv[0], dv[1]), pk2bf(dv[2], dv[3]));
}

// The same two products with one wave per BOARD (round 5; head_dim 16, h = 16 heads <= 64): the
// board's qkv rows (16 x 3h bf16, contiguous in HBM) come into the wave's LDS tile with 16-byte loads
// (6 per lane at h 64) and the heads' fragments are read from there; the per-(board, head) kernels
// above issued three or four 8-byte loads per lane per wave and ran at about half of HBM.  Every
// product, softmax and rounding is theirs, operand for operand (V^T read transposed from the tile is
// the identity-MFMA transpose's exact value), so the results are bit for bit the same.  Outputs
// go back through the tile (each head's region is only its own) and leave as 16-byte stores.
constexpr int kAbTP = 200;  // bf16 pitch of a board tile row (>= 3 x 64 + 8: rows 36 banks apart)

constexpr int kAbOP = 72;   // bf16 pitch of the dO tile (h <= 64 columns, rows 36 banks apart)

__device__ __forceinline__ void attn_board_load(uint16_t *tile, const uint16_t *src, int cols, int lane,
                                                int pitch = kAbTP) {
    const int cpr = cols / 8;  // 16-byte chunks per row
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    for (int c = lane; c < 16 * cpr; c += 64) {
        const int r = c / cpr, k = c - r * cpr;
        *reinterpret_cast<uint4 *>(tile + r * pitch + 8 * k) = s4[c];
    }
}

__device__ __forceinline__ void attn_board_store(uint16_t *dst, const uint16_t *tile, int cols, int lane) {
    const int cpr = cols / 8;
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    for (int c = lane; c < 16 * cpr; c += 64) {
        const int r = c / cpr, k = c - r * cpr;
        d4[c] = *reinterpret_cast<const uint4 *>(tile + r * kAbTP + 8 * k);
    }
}

template <bool kDrop>
__global__ __launch_bounds__(256) void urm_attn16b_kernel(const uint16_t *__restrict__ qkv, uint16_t *__restrict__ out,
                                                          int64_t n, int h, int heads, AttnDrop drop) {
    __shared__ __attribute__((aligned(16))) uint16_t tiles[4][16 * kAbTP];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t b = (int64_t)blockIdx.x * 4 + wave;
    if (b >= n) return;  // wave-uniform; no block barrier below
    uint16_t *tile = tiles[wave];
    const int t = lane & 15, g = lane >> 4;
    attn_board_load(tile, qkv + b * 16 * (int64_t)(3 * h), 3 * h, lane);
    wave_lds_sync();
    for (int hh = 0; hh < heads; hh++) {
        const s16x4 ka = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(tile + t * kAbTP + h + 16 * hh + 4 * g));
        const s16x4 qb = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(tile + t * kAbTP + 16 * hh + 4 * g));
        s16x4 va;  // V^T[dim t][key 4g + jj]
#pragma unroll
        for (int jj = 0; jj < 4; jj++) va[jj] = (short)tile[(4 * g + jj) * kAbTP + 2 * h + 16 * hh + t];
        const f32x4 st = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ka, qb, f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
        const float scale = 1.0f / sqrtf(16.0f);
        float p[4];
        float m = -INFINITY;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            p[r] = st[r] * scale;
            m = fmaxf(m, p[r]);
        }
        m = xmax32(xmax16(m));
        float sum = 0.0f;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            p[r] = __expf(p[r] - m);
            sum += p[r];
        }
        sum = xsum32(xsum16(sum));
        const float inv = 1.0f / sum;
        float km[4] = {1.0f, 1.0f, 1.0f, 1.0f};
        if (kDrop) attn_keep(drop, b, hh, t, g, km);
        s16x4 pb;
#pragma unroll
        for (int r = 0; r < 4; r++) pb[r] = (short)f2bf(kDrop ? p[r] * inv * km[r] : p[r] * inv);
        const f32x4 o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, pb, f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
        wave_lds_sync();  // every lane's Q / K / V reads of this head are done
        *reinterpret_cast<uint2 *>(tile + t * kAbTP + 16 * hh + 4 * g) = make_uint2(pk2bf(o[0], o[1]), pk2bf(o[2], o[3]));
    }
    wave_lds_sync();
    attn_board_store(out + b * 16 * (int64_t)h, tile, h, lane);
}

template <bool kDrop>
__global__ __launch_bounds__(256) void urm_attn_bwd16b_kernel(const uint16_t *__restrict__ qkv,
                                                              const uint16_t *__restrict__ dout,
                                                              uint16_t *__restrict__ dqkv, int64_t n, int h, int heads,
                                                              AttnDrop drop) {
    __shared__ __attribute__((aligned(16))) uint16_t tiles[4][16 * kAbTP];
    __shared__ __attribute__((aligned(16))) uint16_t otiles[4][16 * kAbOP];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t b = (int64_t)blockIdx.x * 4 + wave;
    if (b >= n) return;
    uint16_t *tile = tiles[wave], *otile = otiles[wave];
    const int t = lane & 15, g = lane >> 4;
    attn_board_load(tile, qkv + b * 16 * (int64_t)(3 * h), 3 * h, lane);
    attn_board_load(otile, dout + b * 16 * (int64_t)h, h, lane, kAbOP);
    wave_lds_sync();
    s16x4 eye;
#pragma unroll
    for (int r = 0; r < 4; r++) eye[r] = (short)(4 * g + r == t ? 0x3F80 : 0);
    const f32x4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
    auto pack4 = [](float a0, float a1, float a2, float a3) {
        return __builtin_bit_cast(s16x4, make_uint2(pk2bf(a0, a1), pk2bf(a2, a3)));
    };
    auto tr = [&](s16x4 x) {
        const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x, eye, zero, 0, 0, 0);
        return pack4(d[0], d[1], d[2], d[3]);
    };
    for (int hd = 0; hd < heads; hd++) {
        const uint16_t *row = tile + t * kAbTP + hd * 16 + 4 * g;
        const s16x4 qa = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(row));
        const s16x4 ka = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(row + h));
        const s16x4 va = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(row + 2 * h));
        const s16x4 oa = __builtin_bit_cast(s16x4, *reinterpret_cast<const uint2 *>(otile + t * kAbOP + hd * 16 + 4 * g));
        const f32x4 st = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ka, qa, zero, 0, 0, 0);
        const float scale = 0.25f;
        float p[4];
        float m = -INFINITY;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            p[r] = st[r] * scale;
            m = fmaxf(m, p[r]);
        }
        m = xmax32(xmax16(m));
        float sum = 0.0f;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            p[r] = __expf(p[r] - m);
            sum += p[r];
        }
        sum = xsum32(xsum16(sum));
        const float inv = 1.0f / sum;
#pragma unroll
        for (int r = 0; r < 4; r++) p[r] *= inv;
        float km[4] = {1.0f, 1.0f, 1.0f, 1.0f};
        if (kDrop) attn_keep(drop, b, hd, t, g, km);
        const f32x4 dp = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, oa, zero, 0, 0, 0);
        float rs = (p[0] * km[0] * dp[0] + p[1] * km[1] * dp[1]) + (p[2] * km[2] * dp[2] + p[3] * km[3] * dp[3]);
        rs = xsum32(xsum16(rs));
        const s16x4 dsa = pack4(p[0] * (dp[0] * km[0] - rs), p[1] * (dp[1] * km[1] - rs), p[2] * (dp[2] * km[2] - rs),
                                p[3] * (dp[3] * km[3] - rs));
        const s16x4 pda = pack4(p[0] * km[0], p[1] * km[1], p[2] * km[2], p[3] * km[3]);
        const f32x4 dq = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(tr(ka), dsa, zero, 0, 0, 0);
        const f32x4 dk = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(tr(qa), tr(dsa), zero, 0, 0, 0);
        const f32x4 dv = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(tr(oa), tr(pda), zero, 0, 0, 0);
        wave_lds_sync();  // this head's reads are done: its region takes the gradients
        uint16_t *drow = tile + t * kAbTP + hd * 16 + 4 * g;
        *reinterpret_cast<uint2 *>(drow) = make_uint2(pk2bf(dq[0] * scale, dq[1] * scale), pk2bf(dq[2] * scale, dq[3] * scale));
        *reinterpret_cast<uint2 *>(drow + h) = make_uint2(pk2bf(dk[0] * scale, dk[1] * scale), pk2bf(dk[2] * scale, dk[3] * scale));
        *reinterpret_cast<uint2 *>(drow + 2 * h) = make_uint2(pk2bf(dv[0], dv[1]), pk2bf(dv[2], dv[3]));
    }
    wave_lds_sync();
    attn_board_store(dqkv + b * 16 * (int64_t)(3 * h), tile, 3 * h, lane);
}

// Training-path residual RMSNorm of GameURMBlock (game.py:1346, 1350 with rms_norm :1223-1229) as
// one kernel each way, h = 64, for autograd (agent.GameURMBlock): 16 lanes per row (float4 each),
// row sums by 4 xor shuffles inside the 16-lane group.
//   forward  s = h + a, r = rsqrt(mean(s^2) + eps), out = s r          (h, out fp32; a bf16 or fp32)
//   backward ds = r (dout - out mean(dout out));  dh = ds (fp32), da = ds (a's dtype)
__device__ __forceinline__ float sum16(float x) {
    x += __shfl_xor(x, 1);
    x += __shfl_xor(x, 2);
    x += __shfl_xor(x, 4);
    return x + __shfl_xor(x, 8);
}

template <bool ABF>
__global__ __launch_bounds__(256) void urm_rms_res_fwd_kernel(const float *__restrict__ hin, const void *__restrict__ a,
                                                              float *__restrict__ out, float *__restrict__ rstd,
                                                              int64_t rows, float eps, uint16_t *__restrict__ outb) {
    const int lane = threadIdx.x & 15;
    const int64_t stride = (int64_t)gridDim.x * 16;
    for (int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); r < rows; r += stride) {
        const float4 hv = reinterpret_cast<const float4 *>(hin + r * 64)[lane];
        float4 av;
        if (ABF) {
            const uint2 w = reinterpret_cast<const uint2 *>(static_cast<const uint16_t *>(a) + r * 64)[lane];
            av = make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xFFFF0000u), __uint_as_float(w.y << 16),
                             __uint_as_float(w.y & 0xFFFF0000u));
        } else {
            av = reinterpret_cast<const float4 *>(static_cast<const float *>(a) + r * 64)[lane];
        }
        const float4 sv = make_float4(hv.x + av.x, hv.y + av.y, hv.z + av.z, hv.w + av.w);
        const float ms = sum16(sv.x * sv.x + sv.y * sv.y + sv.z * sv.z + sv.w * sv.w) * (1.0f / 64.0f);
        const float rs = rsqrtf(ms + eps);
        const float4 ov = make_float4(sv.x * rs, sv.y * rs, sv.z * rs, sv.w * rs);
        reinterpret_cast<float4 *>(out + r * 64)[lane] = ov;
        if (outb) {  // the next projection's bf16 operand (what autocast's cast would produce)
            const __attribute__((ext_vector_type(2))) __bf16 p0 = {(__bf16)ov.x, (__bf16)ov.y}, p1 = {(__bf16)ov.z, (__bf16)ov.w};
            reinterpret_cast<uint2 *>(outb + r * 64)[lane] =
                make_uint2(__builtin_bit_cast(uint32_t, p0), __builtin_bit_cast(uint32_t, p1));
        }
        if (lane == 0) rstd[r] = rs;
    }
}

// dpool (optional, instead of dout): the mean-pool's gradient [rows / 16, 64], broadcast over the 16
// token rows of each board (GameURM.forward's h.mean(dim=1), game.py:1450, whose backward is
// dpooled / 16 expanded): never materialised as a [rows, 64] tensor
template <bool ABF>
__global__ __launch_bounds__(256) void urm_rms_res_bwd_kernel(const float *__restrict__ dout, const float *__restrict__ out,
                                                              const float *__restrict__ rstd, float *__restrict__ dh,
                                                              void *__restrict__ da, int64_t rows,
                                                              const uint16_t *__restrict__ doutb,
                                                              const float *__restrict__ dpool) {
    const int lane = threadIdx.x & 15;
    const int64_t stride = (int64_t)gridDim.x * 16;
    for (int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); r < rows; r += stride) {
        float4 g = dout ? reinterpret_cast<const float4 *>(dout + r * 64)[lane] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (dpool) g = reinterpret_cast<const float4 *>(dpool + (r >> 4) * 64)[lane];
        if (doutb) {  // + the bf16 copy's gradient (autocast's cast backward: to fp32, then added)
            const uint2 w = reinterpret_cast<const uint2 *>(doutb + r * 64)[lane];
            g.x += __uint_as_float(w.x << 16);
            g.y += __uint_as_float(w.x & 0xFFFF0000u);
            g.z += __uint_as_float(w.y << 16);
            g.w += __uint_as_float(w.y & 0xFFFF0000u);
        }
        const float4 o = reinterpret_cast<const float4 *>(out + r * 64)[lane];
        const float rs = rstd[r];
        const float mg = sum16(g.x * o.x + g.y * o.y + g.z * o.z + g.w * o.w) * (1.0f / 64.0f);
        const float4 ds = make_float4(rs * (g.x - o.x * mg), rs * (g.y - o.y * mg), rs * (g.z - o.z * mg),
                                      rs * (g.w - o.w * mg));
        reinterpret_cast<float4 *>(dh + r * 64)[lane] = ds;
        if (ABF) {
            const __attribute__((ext_vector_type(2))) __bf16 p0 = {(__bf16)ds.x, (__bf16)ds.y}, p1 = {(__bf16)ds.z, (__bf16)ds.w};
            reinterpret_cast<uint2 *>(static_cast<uint16_t *>(da) + r * 64)[lane] =
                make_uint2(__builtin_bit_cast(uint32_t, p0), __builtin_bit_cast(uint32_t, p1));
        } else {
            reinterpret_cast<float4 *>(static_cast<float *>(da) + r * 64)[lane] = ds;
        }
    }
}

// Training-path SwiGLU + depthwise conv (kernel 2) of GameConvSwiGLU (game.py:1264-1276) for
// autograd (agent.GameConvSwiGLU): one thread per channel, a block per board (grid-stride), the 16
// tokens in a register loop, so the conv's one-token shift is a register carry.  The arithmetic
// follows the reference's autocast dtypes: y = bf16(bf16(silu(gate)) * up), y2 = y_{t-1} w0 +
// y_t w1 + b in fp32, act = silu(y2) (stored bf16: the down_proj operand).  The backward recomputes
// y and y2 and writes dgate / dup (bf16) and per-block partials of dw0, dw1, db (fp32 [3][inter]).
constexpr int kScThreads = 128;

__device__ __forceinline__ float bfr(float x) { return (float)(__bf16)x; }
// sigmoid on the hardware exp / reciprocal (v_exp_f32, v_rcp_f32: 1-2 ulp) instead of the libm expf
// and an IEEE division (~25 instructions, which made these kernels VALU-bound)
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ uint16_t f2bf16(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }
__device__ __forceinline__ float bf16f(uint16_t x) { return __uint_as_float((uint32_t)x << 16); }

__global__ __launch_bounds__(kScThreads) void urm_swiglu_conv_fwd_kernel(const uint16_t *__restrict__ gu,
                                                                         const float *__restrict__ w,
                                                                         const float *__restrict__ bias,
                                                                         uint16_t *__restrict__ act, int64_t nb,
                                                                         int inter) {
    const int c = threadIdx.x;
    if (c >= inter) return;
    const float w0 = w[2 * c], w1 = w[2 * c + 1], b = bias[c];
    for (int64_t bd = blockIdx.x; bd < nb; bd += gridDim.x) {
        float yp = 0.0f;
        uint16_t gr[16], ur[16];  // the board's 32 loads in flight before any arithmetic
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const int64_t r = 16 * bd + t;
            gr[t] = gu[r * 2 * inter + c];
            ur[t] = gu[r * 2 * inter + inter + c];
        }
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const int64_t r = 16 * bd + t;
            const float g = bf16f(gr[t]), u = bf16f(ur[t]);
            const float y = bfr(bfr(g * sigm(g)) * u);
            const float y2 = yp * w0 + y * w1 + b;
            act[r * inter + c] = f2bf16(y2 * sigm(y2));
            yp = y;
        }
    }
}

// The same forward with one thread per channel PAIR (4-byte gate / up loads and act stores) and
// four boards per 256-thread block (64 threads per board, inter / 2 <= 64 of them active): half the
// memory instructions of the one-channel kernel and twice the boards in flight per CU.  Same
// arithmetic per channel, so the outputs are identical.
__global__ __launch_bounds__(256) void urm_swiglu_conv_fwd2_kernel(const uint16_t *__restrict__ gu,
                                                                   const float *__restrict__ w,
                                                                   const float *__restrict__ bias,
                                                                   uint16_t *__restrict__ act, int64_t nb, int inter) {
    const int cp = threadIdx.x & 63;
    if (2 * cp >= inter) return;
    const int c = 2 * cp;
    const float w00 = w[2 * c], w01 = w[2 * c + 1], w10 = w[2 * c + 2], w11 = w[2 * c + 3];
    const float b0 = bias[c], b1 = bias[c + 1];
    for (int64_t bd = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); bd < nb; bd += (int64_t)gridDim.x * 4) {
        uint32_t gr[16], ur[16];
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const uint16_t *row = gu + (16 * bd + t) * 2 * inter;
            gr[t] = *reinterpret_cast<const uint32_t *>(row + c);
            ur[t] = *reinterpret_cast<const uint32_t *>(row + inter + c);
        }
        float yp0 = 0.0f, yp1 = 0.0f;
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const float g0 = __uint_as_float(gr[t] << 16), g1 = __uint_as_float(gr[t] & 0xFFFF0000u);
            const float u0 = __uint_as_float(ur[t] << 16), u1 = __uint_as_float(ur[t] & 0xFFFF0000u);
            const float y0 = bfr(bfr(g0 * sigm(g0)) * u0), y1 = bfr(bfr(g1 * sigm(g1)) * u1);
            const float z0 = yp0 * w00 + y0 * w01 + b0, z1 = yp1 * w10 + y1 * w11 + b1;
            *reinterpret_cast<uint32_t *>(act + (16 * bd + t) * inter + c) =
                pk2bf(z0 * sigm(z0), z1 * sigm(z1));
            yp0 = y0;
            yp1 = y1;
        }
    }
}

__global__ __launch_bounds__(kScThreads) void urm_swiglu_conv_bwd_kernel(const uint16_t *__restrict__ gu,
                                                                         const float *__restrict__ w,
                                                                         const float *__restrict__ bias,
                                                                         const uint16_t *__restrict__ dact,
                                                                         uint16_t *__restrict__ dgu,
                                                                         float *__restrict__ part, int64_t nb,
                                                                         int inter) {
    const int c = threadIdx.x;
    if (c >= inter) return;
    const float w0 = w[2 * c], w1 = w[2 * c + 1], b = bias[c];
    float s0 = 0.0f, s1 = 0.0f, sb = 0.0f;
    for (int64_t bd = blockIdx.x; bd < nb; bd += gridDim.x) {
        float g[16], u[16], y[16], d2[16], sgg[16];
        float yp = 0.0f;
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const int64_t r = 16 * bd + t;
            g[t] = bf16f(gu[r * 2 * inter + c]);
            u[t] = bf16f(gu[r * 2 * inter + inter + c]);
            sgg[t] = sigm(g[t]);
            y[t] = bfr(bfr(g[t] * sgg[t]) * u[t]);
            const float y2 = yp * w0 + y[t] * w1 + b, sg = sigm(y2);
            d2[t] = bf16f(dact[r * inter + c]) * (sg * (1.0f + y2 * (1.0f - sg)));  // d act / d y2
            s1 += d2[t] * y[t];
            s0 += d2[t] * yp;
            sb += d2[t];
            yp = y[t];
        }
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const int64_t r = 16 * bd + t;
            const float dy = d2[t] * w1 + (t + 1 < 16 ? d2[t + 1] * w0 : 0.0f);
            const float sg = sgg[t], sl = bfr(g[t] * sg);
            dgu[r * 2 * inter + c] = f2bf16(dy * u[t] * (sg * (1.0f + g[t] * (1.0f - sg))));
            dgu[r * 2 * inter + inter + c] = f2bf16(dy * sl);
        }
    }
    float *pp = part + (int64_t)blockIdx.x * 3 * inter;
    pp[c] = s0;
    pp[inter + c] = s1;
    pp[2 * inter + c] = sb;
}

// The same backward with one thread per channel PAIR (4-byte gu / dact loads and dgu stores) and
// four partial rows per 256-thread block (64 threads each, inter / 2 <= 64 of them active), the 16
// tokens in ONE pass with a one-token lag (token t - 1's dgate / dup need d2 of token t): nothing
// but the board's raw loads is kept in registers.  Partial row `row` takes boards row, row + nrows,
// ... exactly like block `row` of urm_swiglu_conv_bwd_kernel, with the same per-channel arithmetic,
// so dgu and the partials are bitwise those of the one-channel kernel.
__global__ __launch_bounds__(256) void urm_swiglu_conv_bwd2_kernel(const uint16_t *__restrict__ gu,
                                                                   const float *__restrict__ w,
                                                                   const float *__restrict__ bias,
                                                                   const uint16_t *__restrict__ dact,
                                                                   uint16_t *__restrict__ dgu, float *__restrict__ part,
                                                                   int64_t nb, int inter, int nrows) {
    const int cp = threadIdx.x & 63, row = (int)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= nrows || 2 * cp >= inter) return;  // no barriers below
    const int c = 2 * cp;
    const float w0[2] = {w[2 * c], w[2 * c + 2]}, w1[2] = {w[2 * c + 1], w[2 * c + 3]}, bb[2] = {bias[c], bias[c + 1]};
    float s0[2] = {0.0f, 0.0f}, s1[2] = {0.0f, 0.0f}, sb[2] = {0.0f, 0.0f};
    for (int64_t bd = row; bd < nb; bd += nrows) {
        uint32_t gr[16], ur[16], dr[16];  // the board's 48 loads in flight before any arithmetic
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const uint16_t *rw = gu + (16 * bd + t) * 2 * inter;
            gr[t] = *reinterpret_cast<const uint32_t *>(rw + c);
            ur[t] = *reinterpret_cast<const uint32_t *>(rw + inter + c);
            dr[t] = *reinterpret_cast<const uint32_t *>(dact + (16 * bd + t) * inter + c);
        }
        float yp[2] = {0.0f, 0.0f}, gq[2] = {0.0f, 0.0f}, uq[2] = {0.0f, 0.0f}, sq[2] = {0.0f, 0.0f}, dq[2] = {0.0f, 0.0f};
#pragma unroll
        for (int t = 0; t <= 16; t++) {
            float d2[2] = {0.0f, 0.0f}, g[2] = {0.0f, 0.0f}, u[2] = {0.0f, 0.0f}, sg[2] = {0.0f, 0.0f};
            uint16_t og[2], ou[2];
#pragma unroll
            for (int j = 0; j < 2; j++) {
                if (t < 16) {
                    g[j] = __uint_as_float(j ? gr[t] & 0xFFFF0000u : gr[t] << 16);
                    u[j] = __uint_as_float(j ? ur[t] & 0xFFFF0000u : ur[t] << 16);
                    const float da = __uint_as_float(j ? dr[t] & 0xFFFF0000u : dr[t] << 16);
                    sg[j] = sigm(g[j]);
                    const float y = bfr(bfr(g[j] * sg[j]) * u[j]);
                    const float y2 = yp[j] * w0[j] + y * w1[j] + bb[j], s2 = sigm(y2);
                    d2[j] = da * (s2 * (1.0f + y2 * (1.0f - s2)));  // d act / d y2
                    s1[j] += d2[j] * y;
                    s0[j] += d2[j] * yp[j];
                    sb[j] += d2[j];
                    yp[j] = y;
                }
                if (t > 0) {  // token t - 1
                    const float dy = dq[j] * w1[j] + (t < 16 ? d2[j] * w0[j] : 0.0f);
                    og[j] = f2bf16(dy * uq[j] * (sq[j] * (1.0f + gq[j] * (1.0f - sq[j]))));
                    ou[j] = f2bf16(dy * bfr(gq[j] * sq[j]));
                }
                gq[j] = g[j];
                uq[j] = u[j];
                sq[j] = sg[j];
                dq[j] = d2[j];
            }
            if (t > 0) {
                uint16_t *dw = dgu + (16 * bd + t - 1) * 2 * inter;
                *reinterpret_cast<uint32_t *>(dw + c) = (uint32_t)og[0] | ((uint32_t)og[1] << 16);
                *reinterpret_cast<uint32_t *>(dw + inter + c) = (uint32_t)ou[0] | ((uint32_t)ou[1] << 16);
            }
        }
    }
    float *pp = part + (int64_t)row * 3 * inter;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        pp[c + j] = s0[j];
        pp[inter + c + j] = s1[j];
        pp[2 * inter + c + j] = sb[j];
    }
}

// dw [inter][2] (w0, w1 interleaved as the conv weight), db [inter] from the nblk partial rows:
// a block per 16 columns, 16 row slices per column (slice s sums rows s, s + 16, ... in order, 8
// loads in flight), then the 16 slice sums added in slice order -- a fixed order, deterministic.
__global__ __launch_bounds__(256) void urm_swiglu_conv_colsum_kernel(const float *__restrict__ part, int nblk, int inter,
                                                                     float *__restrict__ dw, float *__restrict__ db,
                                                                     int acc) {
    __shared__ float red[16][17];
    const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
    const int j = blockIdx.x * 16 + cl, ncol = 3 * inter;
    float t = 0.0f;
    if (j < ncol) {
        int k = sl;
        for (; k + 16 * 7 < nblk; k += 16 * 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = part[(int64_t)(k + 16 * u) * ncol + j];
#pragma unroll
            for (int u = 0; u < 8; u++) t += v[u];
        }
        for (; k < nblk; k += 16) t += part[(int64_t)k * ncol + j];
    }
    red[sl][cl] = t;
    __syncthreads();
    if (sl != 0 || j >= ncol) return;
    t = 0.0f;
#pragma unroll
    for (int u = 0; u < 16; u++) t += red[u][cl];
    // acc: added to the gradient already there (a weight shared by several applications, summed in
    // autograd's order: the same bits as its accumulation of returned gradients)
    float *o = j < inter ? dw + 2 * j : j < 2 * inter ? dw + 2 * (j - inter) + 1 : db + (j - 2 * inter);
    *o = acc ? *o + t : t;
}

// Training-path stem of GameURM (game.py:1376-1380: Linear(3 -> 64, no bias) + LayerNorm + SiLU)
// for autograd (agent.GameURM under bf16 autocast), one kernel each way, 16 lanes per token row (4
// features per lane, row sums by 4 xor shuffles).  Autocast's rounding points: the Linear takes
// bf16 x and W and returns bf16 y; LayerNorm and SiLU run in fp32.
//   forward  y = bf16(x W^T), xh = (y - mean) rstd, z = xh g + b, emb = z sigmoid(z)
//   backward dz = demb silu'(z); dg = sum dz xh; db = sum dz; dy = bf16(rstd (dxh - mean(dxh) -
//            xh mean(dxh xh))) with dxh = dz g; dW = sum dy x (fp32); everything recomputed from x
//            (12 bytes per token), so nothing is saved between the passes.  The parameter gradients
//            are per-block partials [nblk][320] (dW f*3+k, dg 192+f, db 256+f) summed in a fixed
//            order by urm_colsum_kernel: deterministic.
constexpr int kStemCols = 5 * 64;

template <bool XBF>
__device__ __forceinline__ void stem_row(const void *__restrict__ obs, int64_t r, const float (&wr)[4][3], float eps,
                                         float xk[3], float y[4], float xh[4], float &rstd) {
#pragma unroll
    for (int k = 0; k < 3; k++)
        xk[k] = XBF ? bf16f(static_cast<const uint16_t *>(obs)[r * 3 + k]) : bfr(static_cast<const float *>(obs)[r * 3 + k]);
#pragma unroll
    for (int u = 0; u < 4; u++) y[u] = bfr(__builtin_fmaf(xk[2], wr[u][2], __builtin_fmaf(xk[1], wr[u][1], xk[0] * wr[u][0])));
    const float mean = sum16(y[0] + y[1] + y[2] + y[3]) * (1.0f / 64.0f);
    float d[4], v = 0.0f;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        d[u] = y[u] - mean;
        v += d[u] * d[u];
    }
    rstd = rsqrtf(sum16(v) * (1.0f / 64.0f) + eps);
#pragma unroll
    for (int u = 0; u < 4; u++) xh[u] = d[u] * rstd;
}

template <bool XBF>
__global__ __launch_bounds__(256) void urm_stem_fwd_kernel(const void *__restrict__ obs, const float *__restrict__ w,
                                                           const float *__restrict__ lnw, const float *__restrict__ lnb,
                                                           float *__restrict__ emb, int64_t rows, float eps) {
    const int lane = threadIdx.x & 15, f0 = 4 * lane;
    float wr[4][3], g[4], bb[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
#pragma unroll
        for (int k = 0; k < 3; k++) wr[u][k] = bfr(w[(f0 + u) * 3 + k]);
        g[u] = lnw[f0 + u];
        bb[u] = lnb[f0 + u];
    }
    const int64_t stride = (int64_t)gridDim.x * 16;
    for (int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); r < rows; r += stride) {
        float xk[3], y[4], xh[4], rstd;
        stem_row<XBF>(obs, r, wr, eps, xk, y, xh, rstd);
        float e[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const float z = __builtin_fmaf(xh[u], g[u], bb[u]);
            e[u] = z * sigm(z);
        }
        reinterpret_cast<float4 *>(emb + r * 64)[lane] = make_float4(e[0], e[1], e[2], e[3]);
    }
}

template <bool XBF>
__global__ __launch_bounds__(256) void urm_stem_bwd_kernel(const void *__restrict__ obs, const float *__restrict__ w,
                                                           const float *__restrict__ lnw, const float *__restrict__ lnb,
                                                           const float *__restrict__ demb, float *__restrict__ part,
                                                           int64_t rows, float eps) {
    __shared__ float red[16][kStemCols + 1];
    const int lane = threadIdx.x & 15, grp = threadIdx.x >> 4, f0 = 4 * lane;
    float wr[4][3], g[4], bb[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
#pragma unroll
        for (int k = 0; k < 3; k++) wr[u][k] = bfr(w[(f0 + u) * 3 + k]);
        g[u] = lnw[f0 + u];
        bb[u] = lnb[f0 + u];
    }
    float aw[4][3] = {}, ag[4] = {}, ab[4] = {};
    const int64_t stride = (int64_t)gridDim.x * 16;
    for (int64_t r = (int64_t)blockIdx.x * 16 + grp; r < rows; r += stride) {
        const float4 de = reinterpret_cast<const float4 *>(demb + r * 64)[lane];
        const float dev[4] = {de.x, de.y, de.z, de.w};
        float xk[3], y[4], xh[4], rstd;
        stem_row<XBF>(obs, r, wr, eps, xk, y, xh, rstd);
        float dxh[4], m1 = 0.0f, m2 = 0.0f;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const float z = __builtin_fmaf(xh[u], g[u], bb[u]), sg = sigm(z);
            const float dz = dev[u] * (sg * (1.0f + z * (1.0f - sg)));
            ag[u] += dz * xh[u];
            ab[u] += dz;
            dxh[u] = dz * g[u];
            m1 += dxh[u];
            m2 += dxh[u] * xh[u];
        }
        m1 = sum16(m1) * (1.0f / 64.0f);
        m2 = sum16(m2) * (1.0f / 64.0f);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const float dy = bfr(rstd * (dxh[u] - m1 - xh[u] * m2));
#pragma unroll
            for (int k = 0; k < 3; k++) aw[u][k] = __builtin_fmaf(dy, xk[k], aw[u][k]);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
#pragma unroll
        for (int k = 0; k < 3; k++) red[grp][(f0 + u) * 3 + k] = aw[u][k];
        red[grp][192 + f0 + u] = ag[u];
        red[grp][256 + f0 + u] = ab[u];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < kStemCols; c += 256) {
        float t = 0.0f;
#pragma unroll
        for (int q = 0; q < 16; q++) t += red[q][c];
        part[(int64_t)blockIdx.x * kStemCols + c] = t;
    }
}

// out[c] = sum over the nblk partial rows of column c, in row order per slice (see the swiglu one)
__global__ __launch_bounds__(256) void urm_colsum_kernel(const float *__restrict__ part, int nblk, int ncol,
                                                         float *__restrict__ out, int acc = 0, float *out2 = nullptr,
                                                         int j2 = 0, float *out3 = nullptr, int j3 = 0) {
    __shared__ float red[16][17];
    const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
    const int j = blockIdx.x * 16 + cl;
    float t = 0.0f;
    if (j < ncol) {
        int k = sl;
        for (; k + 16 * 7 < nblk; k += 16 * 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = part[(int64_t)(k + 16 * u) * ncol + j];
#pragma unroll
            for (int u = 0; u < 8; u++) t += v[u];
        }
        for (; k < nblk; k += 16) t += part[(int64_t)k * ncol + j];
    }
    red[sl][cl] = t;
    __syncthreads();
    if (sl != 0 || j >= ncol) return;
    t = 0.0f;
#pragma unroll
    for (int u = 0; u < 16; u++) t += red[u][cl];
    // columns j2.. / j3.. to their own outputs when given (one launch for several parameters)
    float *o = out3 && j >= j3 ? out3 + (j - j3) : out2 && j >= j2 ? out2 + (j - j2) : out + j;
    *o = acc ? *o + t : t;
}

// Weight gradient of a projection for autograd training (the URM Functions' backward and any
// y = x W^T of the default GameURM): dW [N, K] = dY^T X over M token rows, dY bf16 [M, N], X bf16
// [M, K], fp32 result.  The reduction runs over M (1 M rows per minibatch): a block per CU takes a
// contiguous row range in 64-row chunks staged in LDS (the next chunk's 16-byte global loads in
// flight during the MFMAs), both operands read back M-major by the transposing ds_read_b64_tr_b16
// (the fragment layout of v_mfma_f32_16x16x32_bf16 needs 8 consecutive rows per lane), the output
// tiles spread over the 8 waves; per-block partials [nblk][N K] summed in a fixed order by
// urm_colsum_kernel -- deterministic.  (A library GEMM with K = 1 M and N, K <= 240 runs ~1-2 ms.)
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
constexpr int kWgChunk = 64, kWgMaxT = 8, kWgThreads = 512;

__device__ __forceinline__ int wg_pitch(int cols) {  // bytes; row stride = 8 (mod 32) dwords
    const int dw = cols / 2;                           // dwords of a row of `cols` bf16
    return 4 * (dw + ((8 - dw % 32) + 32) % 32);
}

__device__ __forceinline__ bf16x8 wg_frag(const char *img, int pitch, int m0, int c0, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int r1 = m0 + 8 * g + q;
    const char *a1 = img + r1 * pitch + (c0 + 4 * p) * 2;
    const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)a1);
    const s16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a1 + 4 * pitch));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(t1, t2, 0, 1, 2, 3, 4, 5, 6, 7));
}

__global__ __launch_bounds__(kWgThreads) void urm_wgrad_kernel(const uint16_t *__restrict__ dy,
                                                               const uint16_t *__restrict__ x, int64_t M, int N,
                                                               int K, int Kp, int64_t rows_per_blk,
                                                               float *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int pn = wg_pitch(N), pk = wg_pitch(Kp);
    char *sY = smem, *sX = smem + kWgChunk * pn;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int NT = N / 16, KT = Kp / 16, T = NT * KT;
    const int64_t m_beg = (int64_t)blockIdx.x * rows_per_blk;
    const int64_t m_end = m_beg + rows_per_blk < M ? m_beg + rows_per_blk : M;
    // zero the X image's K padding columns once (Kp > K); chunk stores never touch them
    for (int e = tid; e < kWgChunk * (Kp - K); e += kWgThreads) {
        const int r = e / (Kp - K), c = K + e % (Kp - K);
        reinterpret_cast<uint16_t *>(sX + r * pk)[c] = 0;
    }
    const int yq = N / 8, xq = K / 8;  // 16-byte pieces per row (N % 8 == K % 8 == 0)
    const int per_chunk = kWgChunk * (yq + xq);
    constexpr int kMaxPer = 8;  // pieces per thread per chunk: 64 x (240 + 120) / 8 / 512 < 6
    uint4 v[kMaxPer];
    auto load = [&](int64_t m0) {
#pragma unroll
        for (int u = 0; u < kMaxPer; u++) {
            const int e = tid + u * kWgThreads;
            uint4 w = make_uint4(0u, 0u, 0u, 0u);
            if (e < per_chunk) {
                const bool isy = e < kWgChunk * yq;
                const int e2 = isy ? e : e - kWgChunk * yq, q = isy ? yq : xq;
                const int r = e2 / q, c8 = e2 - r * q;
                if (m0 + r < m_end)
                    w = isy ? reinterpret_cast<const uint4 *>(dy + (m0 + r) * N)[c8]
                            : reinterpret_cast<const uint4 *>(x + (m0 + r) * K)[c8];
            }
            v[u] = w;
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int u = 0; u < kMaxPer; u++) {
            const int e = tid + u * kWgThreads;
            if (e < per_chunk) {
                const bool isy = e < kWgChunk * yq;
                const int e2 = isy ? e : e - kWgChunk * yq, q = isy ? yq : xq;
                const int r = e2 / q, c8 = e2 - r * q;
                *reinterpret_cast<uint4 *>((isy ? sY + r * pn : sX + r * pk) + 16 * c8) = v[u];
            }
        }
    };
    f32x4 acc[kWgMaxT];
#pragma unroll
    for (int j = 0; j < kWgMaxT; j++) acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (m_beg < m_end) load(m_beg);
    for (int64_t m0 = m_beg; m0 < m_end; m0 += kWgChunk) {
        __syncthreads();  // the previous chunk's fragment reads are done
        store();
        __syncthreads();
        if (m0 + kWgChunk < m_end) load(m0 + kWgChunk);  // in flight during the MFMAs
#pragma unroll
        for (int ks = 0; ks < kWgChunk; ks += 32) {
#pragma unroll
            for (int j = 0; j < kWgMaxT; j++) {
                int t = wave + 8 * j;
                t = t < T ? t : T - 1;  // duplicates are computed but never stored (no divergent MFMA)
                const int ti = t / KT, tk = t - ti * KT;
                const bf16x8 fa = wg_frag(sY, pn, ks, 16 * ti, lane);
                const bf16x8 fb = wg_frag(sX, pk, ks, 16 * tk, lane);
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[j], 0, 0, 0);
            }
        }
    }
    // lane: acc[j][r] = dW[16 ti + 4 (lane >> 4) + r][16 tk + (lane & 15)]
    float *pp = part + (int64_t)blockIdx.x * N * K;
#pragma unroll
    for (int j = 0; j < kWgMaxT; j++) {
        const int t = wave + 8 * j;
        if (t >= T) break;
        const int ti = t / KT, tk = t - ti * KT;
        const int col = 16 * tk + (lane & 15);
        if (col < K) {
#pragma unroll
            for (int r = 0; r < 4; r++) pp[(16 * ti + 4 * (lane >> 4) + r) * K + col] = acc[j][r];
        }
    }
}

// The same product on the LDS-DMA ring of wgrad_ring.hpp (round 4) for the default GameURM's
// shapes: the kernel above keeps one 64-row chunk in flight per CU (3.7-4.6 TB/s on 1 M rows); the
// ring keeps three 32-row stages in flight with no register staging.  Same partial layout.
template <int N, int K, int BI, int BJ, int WI>
__global__ __launch_bounds__(g2048::wgr::kThreads) void urm_wgrad_ring_kernel(g2048::wgr::Prod pr, int64_t m) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    g2048::wgr::product<N, K, BI, BJ, WI>(pr, m, blockIdx.x, smem);
}

// ---------------------------------------------------------------------------------------------
// The whole backward of LinResRMSFn (o_proj / down_proj + residual + post-norm at h = 64, K = the
// projection's input width 64 / 120) in ONE pass (round 5).  A wave takes 32 token rows (two boards)
// at a time:
//   prologue  g = dout [or the board's dpool row] [+ the bf16 doutb], ds = rstd (g - out mean(g out))
//             (urm_rms_res_bwd_kernel's formula; the mean summed 16 features per lane, then across the
//             token's 4 lanes) -> dh fp32, and da = bf16(ds) straight into the dgrad's B fragments
//             (registers) and the wave's da image in LDS -- da never goes to HBM
//   dgrad     dx [rows, K] = da W on v_mfma_f32_16x16x32_bf16 with W^T staged once per block:
//             urm_linear_kernel's wt path (its fragments, k order and 16-byte output stores), so dx
//             is bitwise g2048_urm_linear_t of the same da
//   wgrad     dW [64, K] += da^T x over the 32 rows: the x rows copied into the wave's LDS image,
//             both operands read back by ds_read_b64_tr_b16 (wgrad_ring.hpp's frag: 32 rows = one
//             k-step), accumulated in registers over all of the wave's row pairs; the block's waves
//             added in wave order -> per-block partials [nblk][64 K] -> urm_colsum_kernel
// Replaces urm_rms_res_bwd_kernel + urm_linear_kernel<2, CT, EPI_STORE> (wt) + urm_wgrad_ring_kernel:
// the bf16 da write and its two reads (3 x 2 B per element) and two launches.  One wave per SIMD
// (512 registers: the 4 x CT dW tiles stay resident); a wave has its next pair's loads in flight
// only through the other three waves of the CU, so each wave issues a whole pair's loads at once.
constexpr int kLrThreads = 256;

template <int K>
struct LinResBwd {
    static constexpr int CT = (K + 15) / 16;  // dx output tiles = dW column tiles
    static constexpr int KS = 2;              // contraction of the dgrad: 64 features, two k-steps
    static constexpr int W_BYTES = 16 * CT * LinW<KS>::PITCH * 2;
    static constexpr int A_BYTES = 32 * 128;            // da image: 32 rows x 64 bf16
    static constexpr int B_BYTES = 32 * 2 * K + 16;     // x image: 32 rows x K bf16 (+ the last tile's over-read)
    static constexpr int TP = 2 * K + 16;               // dx staging row pitch (bytes)
    static constexpr int T_BYTES = 16 * TP;
    static constexpr int WAVE_BYTES = (A_BYTES + B_BYTES + T_BYTES + 15) / 16 * 16;
    static constexpr int RED_BYTES = 64 * 16 * CT * 4;  // the block's dW sum [64][16 CT] fp32
    static constexpr int LDS = (W_BYTES + 4 * WAVE_BYTES) > RED_BYTES ? (W_BYTES + 4 * WAVE_BYTES) : RED_BYTES;
};

template <int K>
__global__ __launch_bounds__(kLrThreads, K == 64 ? 2 : 1) void urm_linres_bwd_kernel(
    const float *__restrict__ dout, const float *__restrict__ dpool, const uint16_t *__restrict__ doutb,
    const float *__restrict__ out, const float *__restrict__ rstd, const uint16_t *__restrict__ w,
    const uint16_t *__restrict__ xin, float *__restrict__ dh, uint16_t *__restrict__ dx, float *__restrict__ part,
    int64_t rows) {
    using C = LinResBwd<K>;
    using LW = LinW<C::KS>;
    constexpr int CT = C::CT;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, t = lane & 15, g = lane >> 4;
    // W^T staged (rows q = dx feature < K, 64 k each; rows past K zero): the wt path of urm_linear_kernel
    for (int e = tid; e < C::W_BYTES / 16; e += kLrThreads) reinterpret_cast<uint4 *>(smem)[e] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    for (int e = tid; e < K * 16; e += kLrThreads) {
        const int q = e % K, c4 = e / K;
        const uint16_t *src = w + (int64_t)(4 * c4) * K + q;
        const uint32_t lo = (uint32_t)src[0] | ((uint32_t)src[K] << 16);
        const uint32_t hi = (uint32_t)src[2 * K] | ((uint32_t)src[3 * K] << 16);
        *reinterpret_cast<uint2 *>(smem + LW::piece(q, c4)) = make_uint2(lo, hi);
    }
    __syncthreads();
    char *imgA = smem + C::W_BYTES + wave * C::WAVE_BYTES;
    char *imgB = imgA + C::A_BYTES;
    char *tile = imgB + C::B_BYTES;
    int wo[C::KS];
#pragma unroll
    for (int s = 0; s < C::KS; s++) wo[s] = LW::frag(t, g, s);
    f32x4 aw[4][CT];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < CT; j++) aw[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int64_t boards = rows >> 4, pairs = (boards + 1) >> 1;
    constexpr int NX = (4 * K + 63) / 64;  // 16-byte chunks of the pair's x rows per lane
    for (int64_t pr = (int64_t)blockIdx.x * 4 + wave; pr < pairs; pr += (int64_t)gridDim.x * 4) {
        const int64_t r0 = 32 * pr;
        const int64_t nbytes = (rows - r0 < 32 ? rows - r0 : 32) * 2 * K;  // valid bytes of the pair's x rows
        // ---- every load of the pair first: x rows, then per board g / doutb / out / rstd
        uint4 xv[NX];
#pragma unroll
        for (int u = 0; u < NX; u++) {
            const int c = lane + 64 * u;
            xv[u] = (c < 4 * K && 16 * (int64_t)c < nbytes) ? *reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(xin + r0 * K) + 16 * c)
                                                          : make_uint4(0u, 0u, 0u, 0u);
        }
        float gv[2][16], ov[2][16], rs[2];
#pragma unroll
        for (int b = 0; b < 2; b++) {
            const int64_t bd = 2 * pr + b;
            const bool ok = bd < boards;
            const int64_t r = ok ? 16 * bd + t : 0;
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int64_t base = r * 64 + 32 * s + 8 * g;
                float4 g0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), g1 = g0;
                if (dpool) {
                    g0 = *reinterpret_cast<const float4 *>(dpool + (r >> 4) * 64 + 32 * s + 8 * g);
                    g1 = *reinterpret_cast<const float4 *>(dpool + (r >> 4) * 64 + 32 * s + 8 * g + 4);
                } else if (dout) {
                    g0 = *reinterpret_cast<const float4 *>(dout + base);
                    g1 = *reinterpret_cast<const float4 *>(dout + base + 4);
                }
                float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
                if (doutb) {  // + the bf16 copy's gradient (autocast's cast backward: to fp32, then added)
                    const uint4 wv = *reinterpret_cast<const uint4 *>(doutb + base);
                    const uint32_t wd[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        gg[2 * i] += __uint_as_float(wd[i] << 16);
                        gg[2 * i + 1] += __uint_as_float(wd[i] & 0xFFFF0000u);
                    }
                }
                const float4 o0 = *reinterpret_cast<const float4 *>(out + base);
                const float4 o1 = *reinterpret_cast<const float4 *>(out + base + 4);
                const float oo[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    gv[b][8 * s + i] = ok ? gg[i] : 0.0f;
                    ov[b][8 * s + i] = ok ? oo[i] : 0.0f;
                }
            }
            rs[b] = ok ? rstd[r] : 0.0f;
        }
        // ---- x rows into the image (the wgrad's B' operand)
#pragma unroll
        for (int u = 0; u < NX; u++) {
            const int c = lane + 64 * u;
            if (c < 4 * K) *reinterpret_cast<uint4 *>(imgB + 16 * c) = xv[u];
        }
        // ---- prologue + dgrad per board
#pragma unroll
        for (int b = 0; b < 2; b++) {
            const int64_t bd = 2 * pr + b;
            const bool ok = bd < boards;
            const int64_t r = 16 * bd + t;
            float dot = 0.0f;
#pragma unroll
            for (int i = 0; i < 16; i++) dot += gv[b][i] * ov[b][i];
            const float mg = xsum32(xsum16(dot)) * (1.0f / 64.0f);
            bf16x8 fb[2];
#pragma unroll
            for (int s = 0; s < 2; s++) {
                float d[8];
#pragma unroll
                for (int i = 0; i < 8; i++) d[i] = rs[b] * (gv[b][8 * s + i] - ov[b][8 * s + i] * mg);
                if (ok) {
                    float *dp = dh + r * 64 + 32 * s + 8 * g;
                    *reinterpret_cast<float4 *>(dp) = make_float4(d[0], d[1], d[2], d[3]);
                    *reinterpret_cast<float4 *>(dp + 4) = make_float4(d[4], d[5], d[6], d[7]);
                }
                const uint4 da = make_uint4(pk2bf(d[0], d[1]), pk2bf(d[2], d[3]), pk2bf(d[4], d[5]), pk2bf(d[6], d[7]));
                fb[s] = __builtin_bit_cast(bf16x8, da);
                *reinterpret_cast<uint4 *>(imgA + (16 * b + t) * 128 + (32 * s + 8 * g) * 2) = da;
            }
            if (dx) {  // dx = da W: urm_linear_kernel<2, CT, EPI_STORE>'s products and stores
                f32x4 acc[CT];
#pragma unroll
                for (int ct = 0; ct < CT; ct++) {
                    acc[ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                    for (int s = 0; s < C::KS; s++)
                        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8 *>(smem + 16 * ct * LW::PITCH * 2 + wo[s]),
                                                                          fb[s], acc[ct], 0, 0, 0);
                }
#pragma unroll
                for (int ct = 0; ct < CT; ct++) {
                    const int c = 16 * ct + 4 * g;
                    if (c < K)
                        *reinterpret_cast<uint2 *>(tile + t * C::TP + 2 * c) = make_uint2(pk2bf(acc[ct][0], acc[ct][1]), pk2bf(acc[ct][2], acc[ct][3]));
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                if (ok) {
                    constexpr int per_row = K / 8;  // 16-byte chunks per row
                    uint16_t *dst = dx + bd * 16 * (int64_t)K;
                    for (int q = lane; q < 16 * per_row; q += 64) {
                        const int row = q / per_row, c8 = q - row * per_row;
                        *reinterpret_cast<uint4 *>(dst + row * K + 8 * c8) = *reinterpret_cast<const uint4 *>(tile + row * C::TP + 16 * c8);
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();  // the tile is rewritten by the next board
            }
        }
        // ---- dW += da^T x over the pair's 32 rows (images written by this wave only)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        {
            g2048::wgr::bf16x8_t fx[CT];
#pragma unroll
            for (int j = 0; j < CT; j++) fx[j] = g2048::wgr::frag(imgB, 2 * K, 16 * j, lane);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const g2048::wgr::bf16x8_t fa = g2048::wgr::frag(imgA, 128, 16 * i, lane);
#pragma unroll
                for (int j = 0; j < CT; j++) aw[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fx[j], aw[i][j], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();  // the images are rewritten by the next pair
    }
    // ---- the block's dW: waves added in order into LDS, then the partial row [64][K]
    __syncthreads();
    float *red = reinterpret_cast<float *>(smem);
    constexpr int KP = 16 * CT;
    const int c = lane & 15, rq = (lane >> 4) * 4;
    for (int wv = 0; wv < 4; wv++) {
        if (wave == wv) {
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < CT; j++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        float *p = red + (16 * i + rq + r) * KP + 16 * j + c;
                        *p = wv == 0 ? aw[i][j][r] : *p + aw[i][j][r];
                    }
        }
        __syncthreads();
    }
    float *pb = part + (int64_t)blockIdx.x * 64 * K;
    for (int e = tid; e < 64 * K; e += kLrThreads) {
        const int n = e / K, k = e - n * K;
        pb[e] = red[n * KP + k];
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// A loop start of GameURM training (game.py:1441: hidden_states + emb): out = a + e (fp32) and its
// bf16 copy (the first block's qkv operand under autocast) in one pass; `a` may be a per-board
// broadcast of `a_rows` rows (init_hidden [16, h] expanded over the boards).  Backward: the two
// gradient halves (fp32 from the residual RMSNorm, bf16 from the projection) summed into one fp32.
__global__ __launch_bounds__(256) void urm_add_cast_kernel(const float4 *__restrict__ a, int64_t a4,
                                                           const float4 *__restrict__ e, float4 *__restrict__ out,
                                                           uint2 *__restrict__ outb, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const float4 x = a[a4 ? i % a4 : i], y = e[i];
        const float4 o = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
        out[i] = o;
        outb[i] = make_uint2(pk2bf(o.x, o.y), pk2bf(o.z, o.w));
    }
}

// acc_out (optional) = acc_in + dx (acc_in NULL: = dx): the emb gradient summed over the loops in the
// order autograd would sum it (the last loop's first), so the separate accumulation adds over
// [rows, h] fp32 disappear; dx itself may be skipped (NULL) when h needs no gradient.
__global__ __launch_bounds__(256) void urm_add_cast_bwd_kernel(const float4 *__restrict__ dout,
                                                               const uint2 *__restrict__ doutb, float4 *__restrict__ dx,
                                                               int64_t n4, const float4 *__restrict__ acc_in,
                                                               float4 *__restrict__ acc_out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        float4 d = dout ? dout[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (doutb) {
            const uint2 b = doutb[i];
            d = make_float4(d.x + __uint_as_float(b.x << 16), d.y + __uint_as_float(b.x & 0xFFFF0000u),
                            d.z + __uint_as_float(b.y << 16), d.w + __uint_as_float(b.y & 0xFFFF0000u));
        }
        if (dx) dx[i] = d;
        if (acc_out) {
            if (acc_in) {
                const float4 a = acc_in[i];
                d = make_float4(a.x + d.x, a.y + d.y, a.z + d.z, a.w + d.w);
            }
            acc_out[i] = d;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// The backward of GateUpSwiGLUFn with gu RECOMPUTED (round 5): the forward no longer stores gate_up's
// output gu [rows, 2 inter] (503 MB per call at 65 536 boards) -- this kernel recomputes it from the
// saved operand x [rows, h] (128 MB) on MFMA, with exactly the forward's fragments and k order
// (urm_linear_kernel<.., EPI_SWIGLU_T>: the same gu bits), hands it through a per-wave LDS tile from
// the MFMA layout (lane = token) to urm_swiglu_conv_bwd2_kernel's (lane = channel pair, the 16
// tokens in a register loop with a one-token lag), and runs bwd2's arithmetic on it.  Waves take
// the boards of bwd2's partial rows (row = global wave index, nrows = the grid's waves, boards row,
// row + nrows, ...), each wave writes its own partial row: dgu and the dw / db partials are those of
// bwd2 on the stored gu, term for term.
constexpr int kGusTP = 16 * 16 + 4;  // bf16 pitch of the gu tile rows (130 dwords: conflict-free 8-byte stores)

template <int KS, int CT>
__global__ __launch_bounds__(kThreads) void urm_gate_up_swiglu_bwd_kernel(
    const uint16_t *__restrict__ in, const uint16_t *__restrict__ w, const float *__restrict__ cw,
    const float *__restrict__ cb, const uint16_t *__restrict__ dact, uint16_t *__restrict__ dgu,
    float *__restrict__ part, int64_t rows, int K, int inter, int nrows) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int kPitch = LinW<KS>::PITCH;
    constexpr int kRowsW = 16 * CT, CH = CT / 2;
    constexpr int kLinWBytes = kRowsW * kPitch * 2;
    static_assert(kRowsW <= 16 * 16, "gu tile width");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, t = lane & 15, g = lane >> 4;
    char *tile = smem + kLinWBytes + wave * (16 * kGusTP * 2);
    for (int e = tid; e < kRowsW * kPitch / 8; e += kThreads) reinterpret_cast<uint4 *>(smem)[e] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    {   // the forward's staging: gate rows at q < kRowsW / 2, up rows above (zero past inter)
        const int k4 = K >> 2;
        for (int e = tid; e < kRowsW * k4; e += kThreads) {
            const int q = e / k4, c4 = e - q * k4;
            const int hq = q - kRowsW / 2;
            const int src = q < kRowsW / 2 ? (q < inter ? q : -1) : (hq < inter ? inter + hq : -1);
            if (src >= 0)
                *reinterpret_cast<uint2 *>(smem + LinW<KS>::piece(q, c4)) =
                    *reinterpret_cast<const uint2 *>(w + (int64_t)src * K + 4 * c4);
        }
    }
    __syncthreads();
    int wo[KS];
#pragma unroll
    for (int s = 0; s < KS; s++) wo[s] = LinW<KS>::frag(t, g, s);
    // the channel pair of this lane in the token loop (bwd2's thread); lanes past inter / 2 idle there
    const int c = 2 * lane;
    const bool act_ch = c < inter;
    const int cc = act_ch ? c : 0;
    const float w0[2] = {cw[2 * cc], cw[2 * cc + 2]}, w1[2] = {cw[2 * cc + 1], cw[2 * cc + 3]}, bb[2] = {cb[cc], cb[cc + 1]};
    float s0[2] = {0.0f, 0.0f}, s1[2] = {0.0f, 0.0f}, sb[2] = {0.0f, 0.0f};
    const int64_t nb = rows >> 4;
    const int row = blockIdx.x * (kThreads / 64) + wave;  // (waves past nrows: no boards, no partial row)
    for (int64_t bd = row; row < nrows && bd < nb; bd += nrows) {
        // the board's output gradient (bwd2's loads), in flight during the gu recompute
        uint32_t dr[16];
#pragma unroll
        for (int tt = 0; tt < 16; tt++)
            dr[tt] = act_ch ? *reinterpret_cast<const uint32_t *>(dact + (16 * bd + tt) * inter + c) : 0u;
        // gu = bf16(x W^T) in the forward's MFMA order -> the wave's tile [token][gate 0..127 | up 128..255]
        const uint16_t *xr = in + (bd * 16 + t) * K;
        bf16x8 fb[KS];
#pragma unroll
        for (int s = 0; s < KS; s++) {
            const int kk = 32 * s + 8 * g;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (kk + 8 <= K) {
                v = *reinterpret_cast<const uint4 *>(xr + kk);
            } else if (kk < K) {
                const uint2 tl = *reinterpret_cast<const uint2 *>(xr + kk);
                v = make_uint4(tl.x, tl.y, 0u, 0u);
            }
            fb[s] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll 2
        for (int ct = 0; ct < CT; ct++) {
            asm volatile("" ::: "memory");
            f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int s = 0; s < KS; s++)
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8 *>(smem + 16 * ct * kPitch * 2 + wo[s]),
                                                              fb[s], acc, 0, 0, 0);
            const int col = ct < CH ? 16 * ct + 4 * g : 128 + 16 * (ct - CH) + 4 * g;
            *reinterpret_cast<uint2 *>(tile + (t * kGusTP + col) * 2) = make_uint2(pk2bf(acc[0], acc[1]), pk2bf(acc[2], acc[3]));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        uint32_t gr[16], ur[16];
#pragma unroll
        for (int tt = 0; tt < 16; tt++) {
            gr[tt] = *reinterpret_cast<const uint32_t *>(tile + (tt * kGusTP + cc) * 2);
            ur[tt] = *reinterpret_cast<const uint32_t *>(tile + (tt * kGusTP + 128 + cc) * 2);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();  // the next board's tile stores come after every lane's reads
        if (act_ch) {  // urm_swiglu_conv_bwd2_kernel's token loop, verbatim arithmetic
            float yp[2] = {0.0f, 0.0f}, gq[2] = {0.0f, 0.0f}, uq[2] = {0.0f, 0.0f}, sq[2] = {0.0f, 0.0f}, dq[2] = {0.0f, 0.0f};
#pragma unroll
            for (int tt = 0; tt <= 16; tt++) {
                float d2[2] = {0.0f, 0.0f}, gv[2] = {0.0f, 0.0f}, uv[2] = {0.0f, 0.0f}, sg[2] = {0.0f, 0.0f};
                uint16_t og[2], ou[2];
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    if (tt < 16) {
                        gv[j] = __uint_as_float(j ? gr[tt] & 0xFFFF0000u : gr[tt] << 16);
                        uv[j] = __uint_as_float(j ? ur[tt] & 0xFFFF0000u : ur[tt] << 16);
                        const float da = __uint_as_float(j ? dr[tt] & 0xFFFF0000u : dr[tt] << 16);
                        sg[j] = sigm(gv[j]);
                        const float y = bfr(bfr(gv[j] * sg[j]) * uv[j]);
                        const float y2 = yp[j] * w0[j] + y * w1[j] + bb[j], s2 = sigm(y2);
                        d2[j] = da * (s2 * (1.0f + y2 * (1.0f - s2)));  // d act / d y2
                        s1[j] += d2[j] * y;
                        s0[j] += d2[j] * yp[j];
                        sb[j] += d2[j];
                        yp[j] = y;
                    }
                    if (tt > 0) {  // token tt - 1
                        const float dy = dq[j] * w1[j] + (tt < 16 ? d2[j] * w0[j] : 0.0f);
                        og[j] = f2bf16(dy * uq[j] * (sq[j] * (1.0f + gq[j] * (1.0f - sq[j]))));
                        ou[j] = f2bf16(dy * bfr(gq[j] * sq[j]));
                    }
                    gq[j] = gv[j];
                    uq[j] = uv[j];
                    sq[j] = sg[j];
                    dq[j] = d2[j];
                }
                if (tt > 0) {
                    uint16_t *dw = dgu + (16 * bd + tt - 1) * 2 * inter;
                    *reinterpret_cast<uint32_t *>(dw + c) = (uint32_t)og[0] | ((uint32_t)og[1] << 16);
                    *reinterpret_cast<uint32_t *>(dw + inter + c) = (uint32_t)ou[0] | ((uint32_t)ou[1] << 16);
                }
            }
        }
    }
    if (act_ch && row < nrows) {  // this wave's partial row (bwd2's row `row`)
        float *pp = part + (int64_t)row * 3 * inter;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            pp[c + j] = s0[j];
            pp[inter + c + j] = s1[j];
            pp[2 * inter + c + j] = sb[j];
        }
    }
}

template <int KS, int CT>
int launch_gus_bwd(hipStream_t s, const uint16_t *in, const uint16_t *w, const float *cw, const float *cb,
                   const uint16_t *dact, uint16_t *dgu, float *part, int64_t rows, int K, int inter, int nrows) {
    const size_t lds = (size_t)16 * CT * LinW<KS>::PITCH * 2 + (size_t)(kThreads / 64) * 16 * kGusTP * 2;
    const int nblk = (nrows + kThreads / 64 - 1) / (kThreads / 64);
    hipLaunchKernelGGL((urm_gate_up_swiglu_bwd_kernel<KS, CT>), dim3((unsigned)nblk), dim3(kThreads), lds, s, in, w, cw, cb,
                       dact, dgu, part, rows, K, inter, nrows);
    return launch_status();
}

extern "C" {

int g2048_urm_stem(g2048_stream_t stream, const void *obs, int32_t obs_dtype, const float *w, const float *ln_w,
                   const float *ln_b, const float *init_hidden, float *emb, float *x, uint16_t *xb, int64_t n,
                   int32_t h) {
    if (n < 0 || !h_ok(h) || (obs_dtype != 0 && obs_dtype != 1)) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!obs || !w || !ln_w || !ln_b || !init_hidden || !emb || !x || !xb) return G2048_EINVAL;
    const int64_t rows = 16 * n;
    if (obs_dtype == 1)
        hipLaunchKernelGGL(urm_stem_kernel<true>, dim3(blocks(rows, kThreads / 64)), dim3(kThreads), 0,
                           (hipStream_t)stream, obs, w, ln_w, ln_b, init_hidden, emb, x, xb, rows, (int)h);
    else
        hipLaunchKernelGGL(urm_stem_kernel<false>, dim3(blocks(rows, kThreads / 64)), dim3(kThreads), 0,
                           (hipStream_t)stream, obs, w, ln_w, ln_b, init_hidden, emb, x, xb, rows, (int)h);
    return launch_status();
}

static bool attn_drop_args(float p, uint64_t seed, const uint64_t *counter, AttnDrop &d) {
    if (!(p >= 0.0f && p < 1.0f)) return false;
    d.thr = (uint32_t)lrintf(p * 65536.0f);
    d.scale = 1.0f / (1.0f - p);
    d.k0 = (uint32_t)seed;
    d.k1 = (uint32_t)(seed >> 32);
    d.counter = counter;
    return d.thr == 0 || counter != nullptr;
}

int g2048_urm_attention_drop_at(g2048_stream_t stream, const uint16_t *qkv, uint16_t *out, int64_t n, int32_t h,
                                int32_t heads, float p, uint64_t seed, const uint64_t *counter, uint64_t offset) {
    AttnDrop d{};
    if (n < 0 || !h_ok(h) || heads <= 0 || h % heads != 0 || h / heads > 64) return G2048_EINVAL;
    if (!attn_drop_args(p, seed, counter, d)) return G2048_EINVAL;
    d.offset = offset;
    if (n == 0) return G2048_OK;
    if (!qkv || !out) return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    if (h == 16 * heads && h <= 64 && ((uintptr_t)qkv | (uintptr_t)out) % 16 == 0) {  // one wave per board
        const dim3 gb((unsigned)((n + 3) / 4));
        if (d.thr != 0) hipLaunchKernelGGL(urm_attn16b_kernel<true>, gb, dim3(256), 0, s, qkv, out, n, (int)h, (int)heads, d);
        else hipLaunchKernelGGL(urm_attn16b_kernel<false>, gb, dim3(256), 0, s, qkv, out, n, (int)h, (int)heads, d);
        return launch_status();
    }
    const int64_t tasks = n * heads;
    const dim3 grid(blocks(tasks, kThreads / 64));
    const bool al = (h / heads) % 4 == 0, dr = d.thr != 0;
    if (al && dr) hipLaunchKernelGGL((urm_attn_kernel<true, true>), grid, dim3(kThreads), 0, s, qkv, out, tasks, (int)h, (int)heads, d);
    else if (al) hipLaunchKernelGGL((urm_attn_kernel<true, false>), grid, dim3(kThreads), 0, s, qkv, out, tasks, (int)h, (int)heads, d);
    else if (dr) hipLaunchKernelGGL((urm_attn_kernel<false, true>), grid, dim3(kThreads), 0, s, qkv, out, tasks, (int)h, (int)heads, d);
    else hipLaunchKernelGGL((urm_attn_kernel<false, false>), grid, dim3(kThreads), 0, s, qkv, out, tasks, (int)h, (int)heads, d);
    return launch_status();
}

int g2048_urm_attention_drop(g2048_stream_t stream, const uint16_t *qkv, uint16_t *out, int64_t n, int32_t h,
                             int32_t heads, float p, uint64_t seed, const uint64_t *counter) {
    return g2048_urm_attention_drop_at(stream, qkv, out, n, h, heads, p, seed, counter, 0);
}

int g2048_urm_attention(g2048_stream_t stream, const uint16_t *qkv, uint16_t *out, int64_t n, int32_t h,
                        int32_t heads) {
    return g2048_urm_attention_drop(stream, qkv, out, n, h, heads, 0.0f, 0, nullptr);
}

int g2048_urm_attention_bwd_drop_at(g2048_stream_t stream, const uint16_t *qkv, const uint16_t *dout,
                                    uint16_t *dqkv, int64_t n, int32_t h, int32_t heads, float p, uint64_t seed,
                                    const uint64_t *counter, uint64_t offset) {
    AttnDrop d{};
    if (n < 0 || heads <= 0 || h != 16 * heads || h > 512) return G2048_EINVAL;
    if (!attn_drop_args(p, seed, counter, d)) return G2048_EINVAL;
    d.offset = offset;
    if (n == 0) return G2048_OK;
    if (!qkv || !dout || !dqkv || ((uintptr_t)qkv | (uintptr_t)dout | (uintptr_t)dqkv) % 8) return G2048_EINVAL;
    if (h <= 64 && ((uintptr_t)qkv | (uintptr_t)dout | (uintptr_t)dqkv) % 16 == 0) {  // one wave per board
        const dim3 gb((unsigned)((n + 3) / 4));
        if (d.thr != 0)
            hipLaunchKernelGGL(urm_attn_bwd16b_kernel<true>, gb, dim3(256), 0, (hipStream_t)stream, qkv, dout, dqkv, n,
                               (int)h, (int)heads, d);
        else
            hipLaunchKernelGGL(urm_attn_bwd16b_kernel<false>, gb, dim3(256), 0, (hipStream_t)stream, qkv, dout, dqkv, n,
                               (int)h, (int)heads, d);
        return launch_status();
    }
    const int64_t tasks = n * heads;
    if (d.thr != 0)
        hipLaunchKernelGGL(urm_attn_bwd16_kernel<true>, dim3(blocks(tasks, 4)), dim3(256), 0, (hipStream_t)stream, qkv,
                           dout, dqkv, tasks, (int)h, (int)heads, d);
    else
        hipLaunchKernelGGL(urm_attn_bwd16_kernel<false>, dim3(blocks(tasks, 4)), dim3(256), 0, (hipStream_t)stream, qkv,
                           dout, dqkv, tasks, (int)h, (int)heads, d);
    return launch_status();
}

int g2048_urm_attention_bwd_drop(g2048_stream_t stream, const uint16_t *qkv, const uint16_t *dout, uint16_t *dqkv,
                                 int64_t n, int32_t h, int32_t heads, float p, uint64_t seed, const uint64_t *counter) {
    return g2048_urm_attention_bwd_drop_at(stream, qkv, dout, dqkv, n, h, heads, p, seed, counter, 0);
}

int g2048_urm_attention_bwd(g2048_stream_t stream, const uint16_t *qkv, const uint16_t *dout, uint16_t *dqkv,
                            int64_t n, int32_t h, int32_t heads) {
    return g2048_urm_attention_bwd_drop(stream, qkv, dout, dqkv, n, h, heads, 0.0f, 0, nullptr);
}

int g2048_urm_rms_res_fwd2(g2048_stream_t stream, const float *h, const void *a, int32_t a_dtype, float *out,
                           uint16_t *outb, float *rstd, int64_t rows, int32_t hidden, float eps) {
    if (rows < 0 || hidden != 64 || (a_dtype != 0 && a_dtype != 1)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!h || !a || !out || !rstd || ((uintptr_t)h | (uintptr_t)out) % 16 || ((uintptr_t)a | (uintptr_t)outb) % 8)
        return G2048_EINVAL;
    const int64_t nb = (rows + 15) / 16;
    const dim3 grid((unsigned)(nb < 4096 ? nb : 4096));
    if (a_dtype == 1)
        hipLaunchKernelGGL(urm_rms_res_fwd_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, h, a, out, rstd, rows, eps,
                           outb);
    else
        hipLaunchKernelGGL(urm_rms_res_fwd_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, h, a, out, rstd, rows,
                           eps, outb);
    return launch_status();
}

int g2048_urm_add_cast(g2048_stream_t stream, const float *a, int64_t a_rows, const float *e, float *out, uint16_t *outb,
                       int64_t rows, int32_t hidden) {
    if (rows < 0 || hidden <= 0 || hidden % 4 || a_rows < 0 || (a_rows && rows % a_rows)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!a || !e || !out || !outb || ((uintptr_t)a | (uintptr_t)e | (uintptr_t)out) % 16 || (uintptr_t)outb % 8)
        return G2048_EINVAL;
    const int64_t n4 = rows * hidden / 4;
    const int64_t blocks = (n4 + 255) / 256;
    hipLaunchKernelGGL(urm_add_cast_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                       (hipStream_t)stream, reinterpret_cast<const float4 *>(a), a_rows * hidden / 4,
                       reinterpret_cast<const float4 *>(e), reinterpret_cast<float4 *>(out),
                       reinterpret_cast<uint2 *>(outb), n4);
    return launch_status();
}

int g2048_urm_add_cast_bwd_acc(g2048_stream_t stream, const float *dout, const uint16_t *doutb, float *dx,
                               const float *acc_in, float *acc_out, int64_t rows, int32_t hidden) {
    if (rows < 0 || hidden <= 0 || hidden % 4 || (acc_in && !acc_out)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if ((!dx && !acc_out) || ((uintptr_t)dout | (uintptr_t)dx | (uintptr_t)acc_in | (uintptr_t)acc_out) % 16 ||
        (uintptr_t)doutb % 8)
        return G2048_EINVAL;
    const int64_t n4 = rows * hidden / 4;
    const int64_t blocks = (n4 + 255) / 256;
    hipLaunchKernelGGL(urm_add_cast_bwd_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                       (hipStream_t)stream, reinterpret_cast<const float4 *>(dout), reinterpret_cast<const uint2 *>(doutb),
                       reinterpret_cast<float4 *>(dx), n4, reinterpret_cast<const float4 *>(acc_in),
                       reinterpret_cast<float4 *>(acc_out));
    return launch_status();
}

int g2048_urm_add_cast_bwd(g2048_stream_t stream, const float *dout, const uint16_t *doutb, float *dx, int64_t rows,
                           int32_t hidden) {
    if (!dx) return G2048_EINVAL;
    return g2048_urm_add_cast_bwd_acc(stream, dout, doutb, dx, nullptr, nullptr, rows, hidden);
}

int g2048_urm_rms_res_fwd(g2048_stream_t stream, const float *h, const void *a, int32_t a_dtype, float *out,
                          float *rstd, int64_t rows, int32_t hidden, float eps) {
    return g2048_urm_rms_res_fwd2(stream, h, a, a_dtype, out, nullptr, rstd, rows, hidden, eps);
}

int g2048_urm_rms_res_bwd3(g2048_stream_t stream, const float *dout, const float *dpool, const uint16_t *doutb,
                           const float *out, const float *rstd, float *dh, void *da, int32_t a_dtype, int64_t rows,
                           int32_t hidden) {
    if (rows < 0 || hidden != 64 || (a_dtype != 0 && a_dtype != 1) || (dout && dpool) || (dpool && rows % 16))
        return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if ((!dout && !doutb && !dpool) || !out || !rstd || !dh || !da ||
        ((uintptr_t)dout | (uintptr_t)dpool | (uintptr_t)out | (uintptr_t)dh) % 16 || ((uintptr_t)da | (uintptr_t)doutb) % 8)
        return G2048_EINVAL;
    const int64_t nb = (rows + 15) / 16;
    const dim3 grid((unsigned)(nb < 4096 ? nb : 4096));
    if (a_dtype == 1)
        hipLaunchKernelGGL(urm_rms_res_bwd_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, dout, out, rstd, dh, da,
                           rows, doutb, dpool);
    else
        hipLaunchKernelGGL(urm_rms_res_bwd_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, dout, out, rstd, dh,
                           da, rows, doutb, dpool);
    return launch_status();
}

int g2048_urm_rms_res_bwd2(g2048_stream_t stream, const float *dout, const uint16_t *doutb, const float *out,
                           const float *rstd, float *dh, void *da, int32_t a_dtype, int64_t rows, int32_t hidden) {
    return g2048_urm_rms_res_bwd3(stream, dout, nullptr, doutb, out, rstd, dh, da, a_dtype, rows, hidden);
}

int g2048_urm_rms_res_bwd(g2048_stream_t stream, const float *dout, const float *out, const float *rstd, float *dh,
                          void *da, int32_t a_dtype, int64_t rows, int32_t hidden) {
    if (!dout) return G2048_EINVAL;
    return g2048_urm_rms_res_bwd2(stream, dout, nullptr, out, rstd, dh, da, a_dtype, rows, hidden);
}

static int sc_blocks(int64_t nb) { return (int)(nb < 2048 ? nb : 2048); }

size_t g2048_urm_swiglu_conv_partials(int64_t n, int32_t inter) {
    if (n <= 0 || inter <= 0 || inter > kScThreads) return 0;
    return (size_t)sc_blocks(n) * 3 * inter;
}

int g2048_urm_gate_up_swiglu_bwd_supported(int32_t h, int32_t inter) {
    return (h == 64 && inter > 64 && inter <= 128 && inter % 8 == 0) || (h == 32 && inter > 32 && inter <= 64 && inter % 8 == 0)
               ? 1 : 0;
}

int g2048_urm_gate_up_swiglu_bwd_acc(g2048_stream_t stream, const uint16_t *x, const uint16_t *w, const float *conv_w,
                                     const float *conv_b, const uint16_t *dact, uint16_t *dgu, float *dw, float *db,
                                     float *partials, int64_t n, int32_t h, int32_t inter, int32_t accumulate) {
    if (n <= 0 || !g2048_urm_gate_up_swiglu_bwd_supported(h, inter)) return G2048_EINVAL;
    if (!x || !w || !conv_w || !conv_b || !dact || !dgu || !dw || !db || !partials ||
        ((uintptr_t)x | (uintptr_t)dgu) % 16 || ((uintptr_t)w | (uintptr_t)dact) % 8)
        return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    // bwd2's partial rows (sc_blocks(n) of them, boards row, row + nrows, ...): one per wave
    const int nrows = sc_blocks(n);
    const int64_t rows = 16 * n;
    int st = G2048_EINVAL;
    if (h == 64) st = launch_gus_bwd<2, 16>(s, x, w, conv_w, conv_b, dact, dgu, partials, rows, h, inter, nrows);
    else st = launch_gus_bwd<1, 8>(s, x, w, conv_w, conv_b, dact, dgu, partials, rows, h, inter, nrows);
    if (st) return st;
    hipLaunchKernelGGL(urm_swiglu_conv_colsum_kernel, dim3((3 * inter + 15) / 16), dim3(256), 0, s, partials, nrows,
                       (int)inter, dw, db, accumulate ? 1 : 0);
    return launch_status();
}

int g2048_urm_gate_up_swiglu_bwd(g2048_stream_t stream, const uint16_t *x, const uint16_t *w, const float *conv_w,
                                 const float *conv_b, const uint16_t *dact, uint16_t *dgu, float *dw, float *db,
                                 float *partials, int64_t n, int32_t h, int32_t inter) {
    return g2048_urm_gate_up_swiglu_bwd_acc(stream, x, w, conv_w, conv_b, dact, dgu, dw, db, partials, n, h, inter, 0);
}

int g2048_urm_swiglu_conv_fwd(g2048_stream_t stream, const uint16_t *gu, const float *w, const float *b, uint16_t *act,
                              int64_t n, int32_t inter) {
    if (n < 0 || inter <= 0 || inter > kScThreads) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!gu || !w || !b || !act) return G2048_EINVAL;
    if (inter % 2 == 0 && inter <= 128 && ((uintptr_t)gu | (uintptr_t)act) % 4 == 0) {
        const int64_t nb4 = (n + 3) / 4;
        hipLaunchKernelGGL(urm_swiglu_conv_fwd2_kernel, dim3((unsigned)(nb4 < 4096 ? nb4 : 4096)), dim3(256), 0,
                           (hipStream_t)stream, gu, w, b, act, n, (int)inter);
        return launch_status();
    }
    hipLaunchKernelGGL(urm_swiglu_conv_fwd_kernel, dim3(sc_blocks(n)), dim3(kScThreads), 0, (hipStream_t)stream, gu, w, b,
                       act, n, (int)inter);
    return launch_status();
}

int g2048_urm_swiglu_conv_bwd(g2048_stream_t stream, const uint16_t *gu, const float *w, const float *b,
                              const uint16_t *dact, uint16_t *dgu, float *dw, float *db, float *partials, int64_t n,
                              int32_t inter) {
    if (n <= 0 || inter <= 0 || inter > kScThreads) return G2048_EINVAL;
    if (!gu || !w || !b || !dact || !dgu || !dw || !db || !partials) return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    const int nblk = sc_blocks(n);
    if (inter % 2 == 0 && inter <= 128 && ((uintptr_t)gu | (uintptr_t)dact | (uintptr_t)dgu) % 4 == 0)
        hipLaunchKernelGGL(urm_swiglu_conv_bwd2_kernel, dim3((unsigned)((nblk + 3) / 4)), dim3(256), 0, s, gu, w, b, dact,
                           dgu, partials, n, (int)inter, nblk);
    else
        hipLaunchKernelGGL(urm_swiglu_conv_bwd_kernel, dim3(nblk), dim3(kScThreads), 0, s, gu, w, b, dact, dgu, partials,
                           n, (int)inter);
    hipLaunchKernelGGL(urm_swiglu_conv_colsum_kernel, dim3((3 * inter + 15) / 16), dim3(256), 0, s, partials, nblk,
                       (int)inter, dw, db, 0);
    return launch_status();
}

static int stem_blocks(int64_t rows) {
    const int64_t b = (rows + 15) / 16;
    return (int)(b < 2048 ? b : 2048);
}

size_t g2048_urm_stem_partials(int64_t n) { return n <= 0 ? 0 : (size_t)stem_blocks(16 * n) * kStemCols; }

int g2048_urm_stem_fwd(g2048_stream_t stream, const void *obs, int32_t obs_dtype, const float *w, const float *ln_w,
                       const float *ln_b, float *emb, int64_t n, int32_t h, float eps) {
    if (n < 0 || h != 64 || (obs_dtype != 0 && obs_dtype != 1)) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!obs || !w || !ln_w || !ln_b || !emb || (uintptr_t)emb % 16) return G2048_EINVAL;
    const int64_t rows = 16 * n;
    const hipStream_t s = (hipStream_t)stream;
    if (obs_dtype == 1)
        hipLaunchKernelGGL(urm_stem_fwd_kernel<true>, dim3(stem_blocks(rows)), dim3(256), 0, s, obs, w, ln_w, ln_b, emb,
                           rows, eps);
    else
        hipLaunchKernelGGL(urm_stem_fwd_kernel<false>, dim3(stem_blocks(rows)), dim3(256), 0, s, obs, w, ln_w, ln_b, emb,
                           rows, eps);
    return launch_status();
}

int g2048_urm_stem_bwd3(g2048_stream_t stream, const void *obs, int32_t obs_dtype, const float *w, const float *ln_w,
                        const float *ln_b, const float *demb, float *dw, float *dln_w, float *dln_b, int32_t accumulate,
                        float *partials, int64_t n, int32_t h, float eps) {
    if (n <= 0 || h != 64 || (obs_dtype != 0 && obs_dtype != 1)) return G2048_EINVAL;
    if (!obs || !w || !ln_w || !ln_b || !demb || !dw || !dln_w || !dln_b || !partials || (uintptr_t)demb % 16)
        return G2048_EINVAL;
    const int64_t rows = 16 * n;
    const int nblk = stem_blocks(rows);
    const hipStream_t s = (hipStream_t)stream;
    if (obs_dtype == 1)
        hipLaunchKernelGGL(urm_stem_bwd_kernel<true>, dim3(nblk), dim3(256), 0, s, obs, w, ln_w, ln_b, demb, partials,
                           rows, eps);
    else
        hipLaunchKernelGGL(urm_stem_bwd_kernel<false>, dim3(nblk), dim3(256), 0, s, obs, w, ln_w, ln_b, demb, partials,
                           rows, eps);
    hipLaunchKernelGGL(urm_colsum_kernel, dim3((kStemCols + 15) / 16), dim3(256), 0, s, partials, nblk, kStemCols,
                       dw, accumulate ? 1 : 0, dln_w, 192, dln_b, 256);
    return launch_status();
}

int g2048_urm_stem_bwd(g2048_stream_t stream, const void *obs, int32_t obs_dtype, const float *w, const float *ln_w,
                       const float *ln_b, const float *demb, float *grads, float *partials, int64_t n, int32_t h,
                       float eps) {
    if (!grads) return G2048_EINVAL;
    return g2048_urm_stem_bwd3(stream, obs, obs_dtype, w, ln_w, ln_b, demb, grads, grads + 192, grads + 256, 0, partials,
                               n, h, eps);
}

static int wgrad_blocks(int64_t m) {
    const int64_t chunks = (m + kWgChunk - 1) / kWgChunk;
    return (int)(chunks < 256 ? chunks : 256);
}

int g2048_urm_wgrad_supported(int32_t n, int32_t k) {
    return n > 0 && k > 0 && n % 16 == 0 && k % 8 == 0 && n <= 256 && k <= 256 &&
           (n / 16) * ((k + 15) / 16) <= kWgMaxT * (kWgThreads / 64);
}

size_t g2048_urm_wgrad_partials(int64_t m, int32_t n, int32_t k) {
    if (m <= 0 || n <= 0 || k <= 0) return 0;
    return (size_t)wgrad_blocks(m) * n * k;
}

int g2048_urm_wgrad_acc(g2048_stream_t stream, const uint16_t *dy, const uint16_t *x, float *dw, float *partials,
                        int64_t m, int32_t n, int32_t k, int32_t accumulate) {
    const int acc = accumulate ? 1 : 0;
    if (m <= 0 || !g2048_urm_wgrad_supported(n, k)) return G2048_EINVAL;
    if (!dy || !x || !dw || !partials || ((uintptr_t)dy | (uintptr_t)x) % 16) return G2048_EINVAL;
    const int nblk = wgrad_blocks(m);
    const hipStream_t s = (hipStream_t)stream;
    {   // the ring kernel for the default GameURM's projections (every block writes its partial)
        int64_t rr = (m + nblk - 1) / nblk;
        rr = (rr + g2048::wgr::kRows - 1) / g2048::wgr::kRows * g2048::wgr::kRows;
        const g2048::wgr::Prod pr{reinterpret_cast<const char *>(dy), reinterpret_cast<const char *>(x), partials, rr,
                                  nblk, 0};
        bool ring = true;
        const dim3 gd((unsigned)nblk), bk(g2048::wgr::kThreads);
        const size_t lds = g2048::wgr::kLds;
        if (n == 192 && k == 64) hipLaunchKernelGGL((urm_wgrad_ring_kernel<192, 64, 3, 2, 4>), gd, bk, lds, s, pr, m);
        else if (n == 64 && k == 64) hipLaunchKernelGGL((urm_wgrad_ring_kernel<64, 64, 1, 2, 4>), gd, bk, lds, s, pr, m);
        else if (n == 240 && k == 64) hipLaunchKernelGGL((urm_wgrad_ring_kernel<240, 64, 4, 2, 4>), gd, bk, lds, s, pr, m);
        else if (n == 64 && k == 120) hipLaunchKernelGGL((urm_wgrad_ring_kernel<64, 120, 1, 4, 4>), gd, bk, lds, s, pr, m);
        else ring = false;
        if (ring) {
            hipLaunchKernelGGL(urm_colsum_kernel, dim3((unsigned)((n * k + 15) / 16)), dim3(256), 0, s, partials, nblk,
                               (int)(n * k), dw, acc);
            return launch_status();
        }
    }
    int64_t rows = (m + nblk - 1) / nblk;
    rows = (rows + kWgChunk - 1) / kWgChunk * kWgChunk;
    const int kp = (k + 15) / 16 * 16;
    auto pitch = [](int cols) { const int dw = cols / 2; return 4 * (dw + ((8 - dw % 32) + 32) % 32); };
    const size_t lds = (size_t)kWgChunk * (pitch(n) + pitch(kp));
    hipLaunchKernelGGL(urm_wgrad_kernel, dim3(nblk), dim3(kWgThreads), lds, s, dy, x, m, (int)n, (int)k, kp, rows,
                       partials);
    hipLaunchKernelGGL(urm_colsum_kernel, dim3((unsigned)((n * k + 15) / 16)), dim3(256), 0, s, partials, nblk,
                       (int)(n * k), dw, acc);
    return launch_status();
}

int g2048_urm_wgrad(g2048_stream_t stream, const uint16_t *dy, const uint16_t *x, float *dw, float *partials,
                    int64_t m, int32_t n, int32_t k) {
    return g2048_urm_wgrad_acc(stream, dy, x, dw, partials, m, n, k, 0);
}

// blocks of urm_linres_bwd_kernel: up to one per CU (K = 120: 282 registers per lane, one wave per
// SIMD) or two (K = 64: 200 registers, 50 KB of LDS)
static int linres_bwd_blocks(int64_t rows, int k) {
    const int64_t pairs = ((rows >> 4) + 1) >> 1;
    const int64_t b = (pairs + 3) / 4, cap = k == 64 ? 512 : 256;
    return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

int g2048_urm_linres_bwd_supported(int32_t hidden, int32_t k) { return hidden == 64 && (k == 64 || k == 120) ? 1 : 0; }

size_t g2048_urm_linres_bwd_partials(int64_t rows, int32_t k) {
    return rows <= 0 || (k != 64 && k != 120) ? 0 : (size_t)linres_bwd_blocks(rows, k) * 64 * (size_t)k;
}

int g2048_urm_linres_bwd(g2048_stream_t stream, const float *dout, const float *dpool, const uint16_t *doutb,
                         const float *out, const float *rstd, const uint16_t *w, const uint16_t *x, float *dh,
                         uint16_t *dx, float *dw, float *partials, int32_t accumulate, int64_t rows, int32_t hidden,
                         int32_t k) {
    if (!g2048_urm_linres_bwd_supported(hidden, k) || rows <= 0 || rows % 16) return G2048_EINVAL;
    if (!out || !rstd || !w || !x || !dh || !dw || !partials) return G2048_EINVAL;
    const uintptr_t al = (uintptr_t)dout | (uintptr_t)dpool | (uintptr_t)doutb | (uintptr_t)out | (uintptr_t)x |
                         (uintptr_t)dh | (uintptr_t)dx;
    if (al % 16 || (uintptr_t)w % 2) return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    const int nblk = linres_bwd_blocks(rows, k);
    if (k == 64)
        hipLaunchKernelGGL(urm_linres_bwd_kernel<64>, dim3(nblk), dim3(kLrThreads), LinResBwd<64>::LDS, s, dout, dpool, doutb,
                           out, rstd, w, x, dh, dx, partials, rows);
    else
        hipLaunchKernelGGL(urm_linres_bwd_kernel<120>, dim3(nblk), dim3(kLrThreads), LinResBwd<120>::LDS, s, dout, dpool,
                           doutb, out, rstd, w, x, dh, dx, partials, rows);
    hipLaunchKernelGGL(urm_colsum_kernel, dim3((unsigned)((64 * k + 15) / 16)), dim3(256), 0, s, partials, nblk, 64 * k,
                       dw, accumulate ? 1 : 0);
    return launch_status();
}

int g2048_urm_residual_rms(g2048_stream_t stream, float *x, const uint16_t *y, const float *emb, uint16_t *xb,
                           int64_t rows, int32_t h, float eps) {
    if (rows < 0 || !h_ok(h)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!x || !y || !xb) return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    if (h <= 64)
        hipLaunchKernelGGL(urm_residual_rms_vec_kernel<16>, dim3(blocks(rows, 4 * (kThreads / 64))), dim3(kThreads), 0, s,
                           x, y, emb, xb, rows, (int)h, eps);
    else if (h <= 128)
        hipLaunchKernelGGL(urm_residual_rms_vec_kernel<32>, dim3(blocks(rows, 2 * (kThreads / 64))), dim3(kThreads), 0, s,
                           x, y, emb, xb, rows, (int)h, eps);
    else if (h <= 256)
        hipLaunchKernelGGL(urm_residual_rms_vec_kernel<64>, dim3(blocks(rows, kThreads / 64)), dim3(kThreads), 0, s, x,
                           y, emb, xb, rows, (int)h, eps);
    else
        hipLaunchKernelGGL(urm_residual_rms_kernel, dim3(blocks(rows, kThreads / 64)), dim3(kThreads), 0, s, x, y, emb,
                           xb, rows, (int)h, eps);
    return launch_status();
}

int g2048_urm_swiglu_conv(g2048_stream_t stream, const uint16_t *gu, const float *w, const float *b, uint16_t *out,
                          int64_t n, int32_t inter) {
    if (n < 0 || inter <= 0) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!gu || !w || !b || !out) return G2048_EINVAL;
    if (inter % 8 == 0)  // GameConvSwiGLU rounds inter up to a multiple of 8 (game.py:1248-1250)
        hipLaunchKernelGGL(urm_swiglu_conv2_kernel, dim3(blocks(n * (inter / 2), kThreads)), dim3(kThreads), 0,
                           (hipStream_t)stream, gu, w, b, out, n, (int)inter);
    else
        hipLaunchKernelGGL(urm_swiglu_conv_kernel, dim3(blocks(n * inter, kThreads)), dim3(kThreads), 0,
                           (hipStream_t)stream, gu, w, b, out, n, (int)inter);
    return launch_status();
}

int g2048_urm_pool_heads(g2048_stream_t stream, const float *x, const float *wa, const float *ba, const float *wv,
                         const float *bv, float *logits, float *value, int64_t n, int32_t h) {
    if (n < 0 || !h_ok(h)) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!x || !wa || !ba || !wv || !bv || !logits || !value) return G2048_EINVAL;
    hipLaunchKernelGGL(urm_pool_heads_kernel, dim3(blocks(n, kThreads / 64)), dim3(kThreads), 0,
                       (hipStream_t)stream, x, wa, ba, wv, bv, logits, value, n, (int)h);
    return launch_status();
}


int g2048_urm_linear_supported(int32_t epilogue, int32_t k, int32_t n, int32_t inter) {
    if (epilogue < 0 || epilogue > 4 || k <= 0 || k % 4 || n <= 0 || n % 4 ||
        ((epilogue == 2 || epilogue == 3) && (inter <= 0 || inter % 4)))
        return 0;
    return dispatch_lin(nullptr, epilogue, nullptr, nullptr, 0, k, n, inter, nullptr, nullptr, nullptr, nullptr, 0.0f,
                        nullptr, nullptr, true) == G2048_OK ? 1 : 0;
}

int g2048_urm_linear(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, uint16_t *out, int64_t rows,
                     int32_t k, int32_t n) {
    if (rows < 0 || rows % 16 || n % 8 || !g2048_urm_linear_supported(0, k, n, 0)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!in || !w || !out) return G2048_EINVAL;
    return dispatch_lin((hipStream_t)stream, 0, in, w, rows, k, n, 0, out, nullptr, nullptr, nullptr, 0.0f, nullptr,
                        nullptr, false);
}

int g2048_urm_linear_rms(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, float *x, const float *emb,
                         uint16_t *xb, int64_t rows, int32_t k, int32_t h, float eps) {
    if (rows < 0 || rows % 16 || !g2048_urm_linear_supported(1, k, h, 0)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!in || !w || !x || !xb) return G2048_EINVAL;
    return dispatch_lin((hipStream_t)stream, 1, in, w, rows, k, h, 0, nullptr, x, emb, xb, eps, nullptr, nullptr, false);
}

int g2048_urm_linear_t(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, uint16_t *out, int64_t rows,
                       int32_t k, int32_t n) {
    if (rows < 0 || rows % 16 || n % 8 || k % 4 || !g2048_urm_linear_supported(0, k, n, 0)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!in || !w || !out) return G2048_EINVAL;
    return dispatch_lin((hipStream_t)stream, 0, in, w, rows, k, n, 0, out, nullptr, nullptr, nullptr, 0.0f, nullptr,
                        nullptr, false, nullptr, 1);
}

int g2048_urm_linear_bias(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, const float *bias, uint16_t *out,
                          int64_t rows, int32_t k, int32_t n) {
    if (rows < 0 || rows % 16 || n % 8 || !g2048_urm_linear_supported(0, k, n, 0)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!in || !w || !bias || !out || (uintptr_t)bias % 16) return G2048_EINVAL;
    return dispatch_lin((hipStream_t)stream, 0, in, w, rows, k, n, 0, out, nullptr, nullptr, nullptr, 0.0f, bias, nullptr,
                        false);
}

int g2048_urm_linear_res_rms(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, const float *h, float *out,
                             uint16_t *outb, float *rstd, int64_t rows, int32_t k, int32_t n, float eps) {
    if (rows < 0 || rows % 16 || !g2048_urm_linear_supported(4, k, n, 0)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!in || !w || !h || !out || !rstd || ((uintptr_t)h | (uintptr_t)out) % 16 || (outb && (uintptr_t)outb % 8))
        return G2048_EINVAL;
    return dispatch_lin((hipStream_t)stream, 4, in, w, rows, k, n, 0, nullptr, out, h, outb, eps, nullptr, nullptr, false,
                        rstd);
}

int g2048_urm_linear_swiglu(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, const float *conv_w,
                            const float *conv_b, uint16_t *out, int64_t rows, int32_t h, int32_t inter) {
    if (rows < 0 || rows % 16 || !g2048_urm_linear_supported(2, h, 2 * inter, inter)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!in || !w || !conv_w || !conv_b || !out) return G2048_EINVAL;  // conv params: staged through LDS
    return dispatch_lin((hipStream_t)stream, 2, in, w, rows, h, 2 * inter, inter, out, nullptr, nullptr, nullptr, 0.0f,
                        conv_w, conv_b, false);
}

int g2048_urm_linear_swiglu_train(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, const float *conv_w,
                                  const float *conv_b, uint16_t *gu, uint16_t *act, int64_t rows, int32_t h,
                                  int32_t inter) {
    // the epilogue writes 8 features per lane with 16-byte stores: inter % 8, 16-byte aligned outputs
    if (rows < 0 || rows % 16 || inter % 8 || !g2048_urm_linear_supported(3, h, 2 * inter, inter)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!in || !w || !conv_w || !conv_b || !act || ((uintptr_t)gu | (uintptr_t)act) % 16)
        return G2048_EINVAL;  // (conv params: staged through LDS, any 4-byte alignment)
    return dispatch_lin((hipStream_t)stream, 3, in, w, rows, h, 2 * inter, inter, act, nullptr, nullptr, gu, 0.0f,
                        conv_w, conv_b, false);
}

int g2048_urm_forward_supported(int32_t hidden, int32_t heads, int32_t inter, int32_t num_layers, int32_t conv_kernel) {
    return hidden == mk::H && heads == 4 && inter == mk::INTER && (num_layers == 1 || num_layers == 2) &&
                   conv_kernel == 2 ? 1 : 0;
}

int g2048_urm_forward(g2048_stream_t stream, const g2048_urm_weights *w, const void *obs, int32_t obs_dtype,
                      float *logits, float *value, int64_t n) {
    return g2048_urm_forward_drop(stream, w, obs, obs_dtype, logits, value, n, 0.0f, 0, nullptr);
}

int g2048_urm_forward_drop(g2048_stream_t stream, const g2048_urm_weights *w, const void *obs, int32_t obs_dtype,
                           float *logits, float *value, int64_t n, float p, uint64_t seed, const uint64_t *counter) {
    AttnDrop drop{};
    if (!attn_drop_args(p, seed, counter, drop)) return G2048_EINVAL;
    if (!w || n < 0 || (obs_dtype != 0 && obs_dtype != 1) || w->num_loops <= 0 ||
        !g2048_urm_forward_supported(w->hidden, w->heads, w->inter, w->num_layers, 2))
        return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!obs || !logits || !value || !w->stem_w || !w->ln_w || !w->ln_b || !w->init_hidden || !w->wa || !w->ba ||
        !w->wv || !w->bv)
        return G2048_EINVAL;
    UrmW a{};
    a.stem_w = w->stem_w; a.ln_w = w->ln_w; a.ln_b = w->ln_b; a.init = w->init_hidden;
    a.wa = w->wa; a.ba = w->ba; a.wv = w->wv; a.bv = w->bv;
    for (int l = 0; l < w->num_layers; l++) {
        if (!w->qkv[l] || !w->o[l] || !w->gate_up[l] || !w->down[l] || !w->conv_w[l] || !w->conv_b[l])
            return G2048_EINVAL;
        if (((uintptr_t)w->qkv[l] | (uintptr_t)w->o[l] | (uintptr_t)w->gate_up[l] | (uintptr_t)w->down[l] |
             (uintptr_t)w->conv_w[l] | (uintptr_t)w->conv_b[l]) % 16)
            return G2048_EINVAL;  // staged as 16-byte chunks
        a.qkv[l] = w->qkv[l]; a.o[l] = w->o[l]; a.gu[l] = w->gate_up[l]; a.dn[l] = w->down[l];
        a.cw[l] = w->conv_w[l]; a.cb[l] = w->conv_b[l];
    }
    a.layers = w->num_layers;
    a.loops = w->num_loops;
    a.eps = w->eps;
    a.drop = drop;
    const int64_t per_batch = (int64_t)mk::WAVES * mk::NB;
    int64_t grid = (n + per_batch - 1) / per_batch;
    grid = grid > 256 ? 256 : grid;  // one block per CU: the layer's weights fill most of the LDS
    const size_t lds = (size_t)mk::W_BYTES + (size_t)mk::WAVES * mk::TILE_BYTES + (size_t)mk::PS_ALL * 4;
    const hipStream_t s = (hipStream_t)stream;
    const dim3 gd((unsigned)grid), bk(mk::THREADS);
    if (drop.thr) {  // the training-mode variant carries the Philox mask code; inference does not
        if (obs_dtype == 1) hipLaunchKernelGGL((urm_forward_kernel<true, true>), gd, bk, lds, s, obs, a, logits, value, n);
        else hipLaunchKernelGGL((urm_forward_kernel<false, true>), gd, bk, lds, s, obs, a, logits, value, n);
    } else {
        if (obs_dtype == 1) hipLaunchKernelGGL((urm_forward_kernel<true, false>), gd, bk, lds, s, obs, a, logits, value, n);
        else hipLaunchKernelGGL((urm_forward_kernel<false, false>), gd, bk, lds, s, obs, a, logits, value, n);
    }
    return launch_status();
}

}  // extern "C"
