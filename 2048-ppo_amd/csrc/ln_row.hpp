// ln_row.hpp -- the LayerNorm + ReLU row epilogue of a GameMLP layer (game.py:1033-1046, stem
// :1145-1150) in the MFMA output layout "lane (g, c) holds features 16 n + 4 g + r of its row",
// shared by mlp_fwd_kernel (ppo_update.hip: the update's forward and the per-step rollout policy)
// and policy_rollout_kernel (the fused rollout).  Every floating-point operation is written out
// (explicit fmas, fixed summation order, packed fp32 only where it is per element the same
// operation), so both kernels compute bitwise the same activations whatever the contraction flags
// of their translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace g2048 {
namespace lnrow {

// A pair of fp32 features.  Round 5: a native 2-vector, so + * fma become v_pk_add_f32 /
// v_pk_mul_f32 / v_pk_fma_f32 -- per element the same IEEE operation (same bits), two features per
// instruction.  These epilogues run between a wave's own products at one wave per SIMD (no partner
// wave's MFMAs beside them), where tools/probe/pk_rate.hip measured 4.6 cycles per v_pk_fma_f32 vs
// 5.1 per v_fma_f32: 2.2x the FMAs.  (Beside MFMAs a packed op costs ~22 cycles more than the two
// scalar ones, MI355X_MICROARCH.md 'price of one filler beside MFMAs': G2048_LN_SCALAR restores the
// scalar pairs.)
#ifdef G2048_LN_SCALAR
struct f32x2 {
    float x, y;
};
__device__ __forceinline__ f32x2 operator+(f32x2 a, f32x2 b) { return f32x2{a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ f32x2 operator*(f32x2 a, f32x2 b) { return f32x2{a.x * b.x, a.y * b.y}; }
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) {
    return f32x2{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y)};
}
#else
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
#endif
typedef float f32x4 __attribute__((ext_vector_type(4)));
#ifndef LN_PERM
#define LN_PERM 1
#endif
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr float kEps = 1e-5f;  // nn.LayerNorm default

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {  // RNE (v_cvt_pk_bf16_f32)
    const bf16x2 v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }

// x + (x of the lane 16 / 32 away), i.e. the butterfly steps of __shfl_xor(x, 16) / (x, 32), on the
// VALU cross-lane swaps instead of an LDS round trip (fp add is commutative: same bits)
__device__ __forceinline__ float xor16_add(float x) {
    const uint32_t u = __float_as_uint(x);
    const auto s = __builtin_amdgcn_permlane16_swap(u, u, false, false);  // rows {0,0,2,2} / {1,1,3,3}
    return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
__device__ __forceinline__ float xor32_add(float x) {
    const uint32_t u = __float_as_uint(x);
    const auto s = __builtin_amdgcn_permlane32_swap(u, u, false, false);  // rows {0,1,0,1} / {2,3,2,3}
    return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

// G = bf16(acc) as the layer stores it: gbits (packed bf16) and v (the same values as fp32 pairs)
template <int NT>
__device__ __forceinline__ void round_g(const f32x4 (&acc)[NT], f32x2 (&v)[NT][2], uint2 (&gbits)[NT]) {
#pragma unroll
    for (int n = 0; n < NT; n++) {
        const uint32_t w0 = pack_bf2(acc[n][0], acc[n][1]), w1 = pack_bf2(acc[n][2], acc[n][3]);
        gbits[n] = make_uint2(w0, w1);
#if LN_PERM
        // the halves by v_perm (zero bytes below): the compiler cannot fold these back into
        // single conversions + shift + mask, as it does with bf_lo / bf_hi of a fresh pack
        v[n][0] = f32x2{__uint_as_float(__builtin_amdgcn_perm(w0, 0u, 0x05040C0Cu)), __uint_as_float(__builtin_amdgcn_perm(w0, 0u, 0x07060C0Cu))};
        v[n][1] = f32x2{__uint_as_float(__builtin_amdgcn_perm(w1, 0u, 0x05040C0Cu)), __uint_as_float(__builtin_amdgcn_perm(w1, 0u, 0x07060C0Cu))};
#else
        v[n][0] = f32x2{bf_lo(w0), bf_hi(w0)};
        v[n][1] = f32x2{bf_lo(w1), bf_hi(w1)};
#endif
    }
}

// Row statistics over the valid features (valid(n): tile n's 4-group of this lane is < h): the sum
// as packed fp32 pairs in tile order (element pairs (0, 1) and (2, 3) of a tile), the pair's two
// halves added, then the xor-16 / xor-32 lane sums; v becomes dv = v - sum/h (one fma); the
// variance of dv likewise (packed fmas); rstd = rsqrt(var/h + eps).  Returns the mean (sum/h)
// and rstd.
template <int NT, class Valid>
__device__ __forceinline__ void stats(f32x2 (&v)[NT][2], Valid valid, float inv_n, float &mean, float &rstd) {
    f32x2 s2 = {0.0f, 0.0f};
#pragma unroll
    for (int n = 0; n < NT; n++) {
        const f32x2 t = v[n][0] + v[n][1];
        s2 = valid(n) ? s2 + t : s2;
    }
    float sum = xor32_add(xor16_add(s2.x + s2.y));
    const f32x2 nsum = {-sum, -sum}, invn = {inv_n, inv_n};
    f32x2 q2 = {0.0f, 0.0f};
#pragma unroll
    for (int n = 0; n < NT; n++) {
        v[n][0] = fma2(nsum, invn, v[n][0]);
        v[n][1] = fma2(nsum, invn, v[n][1]);
        const f32x2 q = fma2(v[n][1], v[n][1], fma2(v[n][0], v[n][0], q2));
        q2 = valid(n) ? q : q2;
    }
    const float var = xor32_add(xor16_add(q2.x + q2.y));
    mean = sum * inv_n;
    // round 5: the hardware reciprocal square root (v_rsq_f32, ~1 ulp; torch's layer_norm kernel
    // takes rsqrt too) instead of the correctly rounded 1 / sqrt (~25 instructions per row per layer
    // with its denormal scaling): every kernel on this header computes the same rstd bits
    rstd = __builtin_amdgcn_rsqf(__builtin_fmaf(var, inv_n, kEps));
}

// ReLU(LayerNorm) of a feature pair: max(fma(dv * rstd, gamma, beta), 0)
__device__ __forceinline__ f32x2 affine_relu(f32x2 dv, float rstd, f32x2 gamma, f32x2 beta) {
    const f32x2 y = fma2(dv * f32x2{rstd, rstd}, gamma, beta);
    return f32x2{fmaxf(y.x, 0.0f), fmaxf(y.y, 0.0f)};
}

}  // namespace lnrow
}  // namespace g2048
