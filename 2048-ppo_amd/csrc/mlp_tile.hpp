// mlp_tile.hpp -- GameMLP (game.py:1033-1220) on 16-board MFMA tiles with the layer hand-off in
// registers, shared by the fused rollout (policy_rollout.hip: eval mode, K env steps per launch)
// and the fused PPO-update passes (ppo_fused.hip: the training forward + loss, the KL re-forward).
//
// Layout (v_mfma_f32_16x16x32_bf16, computed as Y^T = W X^T): lane (g, c) = (lane >> 4, lane & 15)
// of a 16-board tile holds features 16 n + 4 g + r (r < 4) of board c of the tile, as fp32
// accumulators acc[n] and then as bf16 pairs act[n] (uint2).  act_frag turns a layer's output
// into the next layer's B fragment by permlane swaps (no LDS round trip); the stem's B fragment is
// built from the board bytes (to_model_format, game.py:92-101) through a constant recipe table.
// The LayerNorm epilogue is ln_row.hpp's arithmetic, so these kernels compute bitwise the same
// activations as g2048_mlp_fwd (ppo_update.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ln_row.hpp"
#include "ppo_common.hpp"

namespace g2048 {
namespace tile {
namespace {  // internal linkage per translation unit (the __constant__ recipe table)

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kMaxLayers = 3;  // stem + 2 residual blocks (GameMLP num_layers = 2)

// ---------------------------------------------------------------- stem fragment table -------
// The stem's B fragment of k-step ks for lane group g holds obs features k = 32 ks + 8 g + j
// (to_model_format order: [exponent, row/3, col/3] per cell).  Per (g, ks): the position features
// as bf16 constants (exponent slots zero), the up to three exponent cells c0 .. c0+2 (inside board
// dwords d, d+1; `xsel` gathers their bytes), and per fragment dword a v_perm selector merging the
// exponents (bf16) into the constants.
struct StemFrag {
    uint32_t c[4], sel[4], xsel, d, pad_[2];
};
struct StemTable {
    StemFrag f[4][2];
    static constexpr uint32_t bf16_rne(float x) {
        const uint32_t u = __builtin_bit_cast(uint32_t, x);
        return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
    }
    constexpr StemTable() : f{} {
        constexpr float thirds[4] = {0.0f, 1.0f / 3.0f, 2.0f / 3.0f, 1.0f};
        for (int g = 0; g < 4; g++)
            for (int ks = 0; ks < 2; ks++) {
                StemFrag &e = f[g][ks];
                int c0 = -1, slot[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
                uint32_t val[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                for (int j = 0; j < 8; j++) {
                    const int k = 32 * ks + 8 * g + j, cell = k / 3, kind = k % 3;
                    if (k >= 48) continue;
                    if (kind == 0) {
                        if (c0 < 0) c0 = cell;
                        slot[j] = cell - c0;  // exponent number 0..2
                    } else {
                        val[j] = bf16_rne(thirds[kind == 1 ? (cell >> 2) : (cell & 3)]);
                    }
                }
                const int cc = c0 < 0 ? 0 : c0;
                const int d = (cc >> 2) < 3 ? (cc >> 2) : 2;
                e.d = (uint32_t)d;
                e.xsel = 0x0C0C0C0Cu;
                for (int s = 0; s < 3; s++) {
                    const int byte = cc + s - 4 * d;
                    if (byte < 8) e.xsel = (e.xsel & ~(0xFFu << (8 * s))) | ((uint32_t)byte << (8 * s));
                }
                for (int w = 0; w < 4; w++) {
                    e.c[w] = val[2 * w] | (val[2 * w + 1] << 16);
                    uint32_t sel = 0;
                    for (int p = 0; p < 2; p++) {
                        const int j = 2 * w + p, sl = slot[j];
                        // exponent s: bf16 in E01 (s = 0: bytes 0,1; s = 1: bytes 2,3) or E2 (bytes
                        // 0,1) = the v_perm high source (selector 4..7); a constant: bytes of c[w]
                        const uint32_t b0 = sl < 0 ? (uint32_t)(2 * p) : (uint32_t)(4 + 2 * (sl == 1));
                        sel |= (b0 | ((b0 + 1u) << 8)) << (16 * p);
                    }
                    e.sel[w] = sel;
                }
            }
    }
};
__constant__ const StemTable kStem = StemTable();

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
    const bf16x2_t v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
__device__ __forceinline__ bf16x8_t as_frag(const uint4 &v) { return __builtin_bit_cast(bf16x8_t, v); }

// LDS geometry of one block weight image for hidden size h: row pitch P = round_up(h, 8) bf16 in
// 16-byte granules.  (A conflict-free pitch for h = 196, 544 B, does not fit two images in 160 KiB.)
__host__ __device__ constexpr int pr_pitch(int h) { return ((2 * ((h + 7) & ~7)) + 15) & ~15; }
__host__ __device__ constexpr int pr_wbytes(int h) { return h * pr_pitch(h); }
// Round 5: at h = 196 (P = 25 units of 16 B) the A-fragment read of lane (g, c) -- row 16 n + c,
// unit 4 ks + g -- hit 2-way bank conflicts in ds_read_b128's lane groups {0-3, 12-15, 20-27}, ...
// (MI355X_MICROARCH.md §LDS: unit 9 c + g mod 16 repeats, 8 LDS cycles per read instead of 4).
// Rows with (c >> 2 ^ c >> 3) odd store their 4-unit k-step groups with the units' low bit flipped
// (g ^ 1), which makes all 16 units of every lane group distinct; the last, partial group (unit 24:
// k 192..199) is stored as is.  Other h keep the plain layout (no 2-bit XOR resolves their pitches).
__host__ __device__ constexpr int pr_swz(int h, int c) { return h == 196 ? (((c >> 2) ^ (c >> 3)) & 1) : 0; }
// k-step ks's unit group lies inside the row (the swizzled groups)
__host__ __device__ constexpr bool pr_ks_swz(int h, int ks) { return 4 * ks + 3 < pr_pitch(h) / 16; }
// LDS byte offset of 8-byte piece q (bf16 k = 4 q .. 4 q + 3) of row r of an image
__host__ __device__ constexpr int pr_piece(int h, int r, int q) {
    const int u = q >> 1;
    const int us = (u | 3) < pr_pitch(h) / 16 ? (u ^ pr_swz(h, r & 15)) : u;
    return r * pr_pitch(h) + 16 * us + 8 * (q & 1);
}
__host__ __device__ constexpr int pr_ln_floats(int nt) { return 16 * nt; }  // one affine vector, zero padded
__host__ __device__ constexpr int pr_lds_bytes(int h, int nt) {
    return 2 * pr_wbytes(h) + 2 * kMaxLayers * pr_ln_floats(nt) * 4 + 16;
}

// This lane group's stem fragment recipe (kStem) for k-steps 0 and 1.
struct StemRecipe {
    uint4 sc[2], ss[2];
    uint32_t sx[2], sd[2];
};
__device__ __forceinline__ StemRecipe stem_recipe(int g) {
    StemRecipe r;
#pragma unroll
    for (int ks = 0; ks < 2; ks++) {
        const StemFrag &e = kStem.f[g][ks];
        r.sc[ks] = make_uint4(e.c[0], e.c[1], e.c[2], e.c[3]);
        r.ss[ks] = make_uint4(e.sel[0], e.sel[1], e.sel[2], e.sel[3]);
        r.sx[ks] = e.xsel;
        r.sd[ks] = e.d;
    }
    return r;
}

// The stem's B fragment of k-step ks (obs features 32 ks + 8 g .. + 7, bf16) of the board whose
// four row dwords are B0 .. B3 (byte j of dword i = the exponent of cell 4 i + j).
__device__ __forceinline__ uint4 stem_frag(const StemRecipe &r, int ks, uint32_t B0, uint32_t B1, uint32_t B2,
                                           uint32_t B3) {
    const uint32_t d = r.sd[ks];
    const uint32_t lo = d == 0u ? B0 : d == 1u ? B1 : B2;
    const uint32_t hi = d == 0u ? B1 : d == 1u ? B2 : B3;
    const uint32_t X = __builtin_amdgcn_perm(hi, lo, r.sx[ks]);  // the exponents' bytes
    const uint32_t e01 = pack_bf2((float)(X & 0xFFu), (float)((X >> 8) & 0xFFu));
    const uint32_t e2 = pack_bf2((float)((X >> 16) & 0xFFu), 0.0f);
    return make_uint4(__builtin_amdgcn_perm(e01, r.sc[ks].x, r.ss[ks].x), __builtin_amdgcn_perm(e01, r.sc[ks].y, r.ss[ks].y),
                      __builtin_amdgcn_perm(e01, r.sc[ks].z, r.ss[ks].z), __builtin_amdgcn_perm(e2, r.sc[ks].w, r.ss[ks].w));
}

// --------------------------------------------------------------- layer epilogues --------------
// g2048_mlp_fwd's epilogue (ppo_update.hip, mlp_fwd_kernel) on one board tile: G = bf16(acc),
// LayerNorm statistics in the same order (features in tile order, then the xor-16 and xor-32 lane
// sums), Y = [X +] ReLU(LN(G)) rounded to bf16.  act[n] holds the layer input (residual) on entry
// and the output on exit; features >= h are zero.
template <int NT, int h, bool RES>
__device__ __forceinline__ void ln_epilogue(f32x4_t (&acc)[NT], uint2 (&act)[NT], const float *sgam, const float *sbet,
                                            int g, float inv_n) {
    namespace R = lnrow;
    R::f32x2 v[NT][2];
    uint2 gb[NT];
    R::round_g<NT>(acc, v, gb);
    auto valid = [&](int n) { return 16 * n + 4 * g < h; };  // folds to true except in the last tile
    float mean, rstd;
    R::stats<NT>(v, valid, inv_n, mean, rstd);
#pragma unroll
    for (int n = 0; n < NT; n++) {
        const int f0 = 16 * n + 4 * g;
        const float4 ga = *reinterpret_cast<const float4 *>(sgam + f0);
        const float4 be = *reinterpret_cast<const float4 *>(sbet + f0);
        R::f32x2 y0 = R::affine_relu(v[n][0], rstd, R::f32x2{ga.x, ga.y}, R::f32x2{be.x, be.y});
        R::f32x2 y1 = R::affine_relu(v[n][1], rstd, R::f32x2{ga.z, ga.w}, R::f32x2{be.z, be.w});
        if (RES) {  // Y = X + ..., the residual being this layer's input
            y0 = R::f32x2{bf_lo(act[n].x), bf_hi(act[n].x)} + y0;
            y1 = R::f32x2{bf_lo(act[n].y), bf_hi(act[n].y)} + y1;
        }
        act[n] = valid(n) ? make_uint2(pack_bf2(y0.x, y0.y), pack_bf2(y1.x, y1.y)) : make_uint2(0u, 0u);
    }
}

// A layer output row in the lane layout (lane (g, c): features 16 n + 4 g .. + 3 of row c as v[n])
// written with 16-byte stores: tiles n, n + 1 (n even) paired by one v_permlane16_swap per dword
// between the lane rows g, g ^ 1 -- lane g even then holds features 16 n + 4 g .. + 7, lane g odd
// 16 (n + 1) + 4 (g - 1) .. + 7 (urm.hip EPI_SWIGLU_T's pairing); an odd last tile keeps 8-byte
// stores.  Round 5: half the store instructions of the train pass's G / H rows (its stores were a
// third of its time: time_fused 71.7 -> 50.4 us with none).  p = the row's first byte.
template <int NT, int h>
__device__ __forceinline__ void store_row16(char *p, const uint2 (&v)[NT], int g) {
    static_assert(16 * (NT - (NT & 1)) <= h, "paired tiles lie inside the row");
    const int cb = (g & 1) ? 16 + 4 * (g - 1) : 4 * g;
#pragma unroll
    for (int n = 0; n + 1 < NT; n += 2) {
        const auto sx = __builtin_amdgcn_permlane16_swap(v[n].x, v[n + 1].x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(v[n].y, v[n + 1].y, false, false);
        *reinterpret_cast<uint4 *>(p + 2 * (16 * n + cb)) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
    }
    if constexpr ((NT & 1) != 0) {
        const int f = 16 * (NT - 1) + 4 * g;
        if (f < h) *reinterpret_cast<uint2 *>(p + 2 * f) = v[NT - 1];
    }
}

// The training epilogue: ln_epilogue with nn.Dropout in train mode (the keep mask of row `row`
// drawn exactly as mlp_fwd_wide_kernel draws it: one Philox call per feature-tile pair n, n + 1)
// between the ReLU and the residual add, the pre-norm G bits stored and the row statistics
// returned for the backward pass -- bitwise g2048_mlp_fwd's G / Y / mean / rstd.
// gout (nullable): the layer's G [m][h]; this row's bits are written at once (at byte offset goff,
// uniform base + 32-bit lane offset: they need no register past the rounding).
template <int NT, int h, bool RES, bool DROP>
__device__ __forceinline__ void ln_epilogue_train(f32x4_t (&acc)[NT], uint2 (&act)[NT], const float *sgam,
                                                  const float *sbet, int g, float inv_n, const ppo::Drop &d,
                                                  uint32_t row, uint16_t *gout, uint32_t goff, float &mean,
                                                  float &rstd) {
    namespace R = lnrow;
    R::f32x2 v[NT][2];
    {
        uint2 gb[NT];
        R::round_g<NT>(acc, v, gb);
        if (gout) {
            char *p = reinterpret_cast<char *>(gout) + (goff + 8u * (uint32_t)g);
#pragma unroll
            for (int n = 0; n < NT; n++)
                if (16 * n + 4 * g < h) *reinterpret_cast<uint2 *>(p + 32 * n) = gb[n];
        }
    }
    auto valid = [&](int n) { return 16 * n + 4 * g < h; };
    R::stats<NT>(v, valid, inv_n, mean, rstd);
    uint4 dpair = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int n = 0; n < NT; n++) {
        const int f0 = 16 * n + 4 * g;
        const float4 ga = *reinterpret_cast<const float4 *>(sgam + f0);
        const float4 be = *reinterpret_cast<const float4 *>(sbet + f0);
        R::f32x2 y0 = R::affine_relu(v[n][0], rstd, R::f32x2{ga.x, ga.y}, R::f32x2{be.x, be.y});
        R::f32x2 y1 = R::affine_relu(v[n][1], rstd, R::f32x2{ga.z, ga.w}, R::f32x2{be.z, be.w});
        if (DROP) {  // tiles n, n + 1 hold column groups 4 n + g, 4 n + 4 + g: one Philox call
            float k[4];
            if ((n & 1) == 0) dpair = ppo::drop_draw4(d, row, (uint32_t)(f0 >> 2));
            ppo::drop_mult_bits(d, ppo::drop_half(dpair, (uint32_t)(f0 >> 2)), k);
            y0 = y0 * R::f32x2{k[0], k[1]};
            y1 = y1 * R::f32x2{k[2], k[3]};
        }
        if (RES) {
            y0 = R::f32x2{bf_lo(act[n].x), bf_hi(act[n].x)} + y0;
            y1 = R::f32x2{bf_lo(act[n].y), bf_hi(act[n].y)} + y1;
        }
        act[n] = valid(n) ? make_uint2(pack_bf2(y0.x, y0.y), pack_bf2(y1.x, y1.y)) : make_uint2(0u, 0u);
    }
}

// ln_epilogue_train with the keep masks drawn ahead (ppo::drop_keep8 per feature-tile pair, bits
// 4 n .. 4 n + 3 of kb = the 4 features of tile n): the same multipliers k (0 or 1 / (1 - p)), so
// bitwise ln_epilogue_train.
template <int NT, int h, bool RES, bool DROP>
__device__ __forceinline__ void ln_epilogue_train_kb(f32x4_t (&acc)[NT], uint2 (&act)[NT], const float *sgam,
                                                     const float *sbet, int g, float inv_n, float scale,
                                                     const uint32_t (&kb)[2], uint16_t *gout, uint32_t goff,
                                                     float &mean, float &rstd) {
    namespace R = lnrow;
    R::f32x2 v[NT][2];
    {
        uint2 gb[NT];
        R::round_g<NT>(acc, v, gb);
        if (gout) store_row16<NT, h>(reinterpret_cast<char *>(gout) + goff, gb, g);
    }
    auto valid = [&](int n) { return 16 * n + 4 * g < h; };
    R::stats<NT>(v, valid, inv_n, mean, rstd);
#pragma unroll
    for (int n = 0; n < NT; n++) {
        const int f0 = 16 * n + 4 * g;
        const float4 ga = *reinterpret_cast<const float4 *>(sgam + f0);
        const float4 be = *reinterpret_cast<const float4 *>(sbet + f0);
        R::f32x2 y0 = R::affine_relu(v[n][0], rstd, R::f32x2{ga.x, ga.y}, R::f32x2{be.x, be.y});
        R::f32x2 y1 = R::affine_relu(v[n][1], rstd, R::f32x2{ga.z, ga.w}, R::f32x2{be.z, be.w});
        if (DROP) {
            float k[4];
            ppo::keep_mult(kb, n, scale, k);
            y0 = y0 * R::f32x2{k[0], k[1]};
            y1 = y1 * R::f32x2{k[2], k[3]};
        }
        if (RES) {
            y0 = R::f32x2{bf_lo(act[n].x), bf_hi(act[n].x)} + y0;
            y1 = R::f32x2{bf_lo(act[n].y), bf_hi(act[n].y)} + y1;
        }
        act[n] = valid(n) ? make_uint2(pack_bf2(y0.x, y0.y), pack_bf2(y1.x, y1.y)) : make_uint2(0u, 0u);
    }
}

// The B fragment of k-step ks (k = 32 ks + 8 g .. + 7 of the board in column c) from the layer
// output tiles 2 ks and 2 ks + 1 held as "lane g: features 4g .. 4g+3" (see the file comment).
template <int NT>
__device__ __forceinline__ uint4 act_frag(const uint2 (&act)[NT], int ks) {
    const int t0 = 2 * ks, t1 = 2 * ks + 1;
    const uint32_t a0 = act[t0].x, a1 = act[t0].y;
    const uint32_t b0 = t1 < NT ? act[t1 < NT ? t1 : 0].x : 0u, b1 = t1 < NT ? act[t1 < NT ? t1 : 0].y : 0u;
    const auto s0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
    const auto f0 = __builtin_amdgcn_permlane16_swap(s0[0], s0[1], false, false);
    const auto f1 = __builtin_amdgcn_permlane16_swap(s1[0], s1[1], false, false);
    return make_uint4(f0[0], f1[0], f0[1], f1[1]);
}

}  // namespace
}  // namespace tile
}  // namespace g2048
