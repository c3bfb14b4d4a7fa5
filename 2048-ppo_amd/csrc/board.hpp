// board.hpp -- device-side 2048 board arithmetic for gfx950 (CDNA4), one 4x4 board per lane.
//
// A board is 16 int8 exponents held in one uint4 (x,y,z,w = rows 0..3, byte j of a row dword =
// column j), i.e. exactly the 16 bytes of one [N,16] row, loaded with a single global_load_dwordx4.
// All per-cell predicates are SWAR on those four dwords (exponents are < 0x80, so per-byte adds
// never carry across bytes):
//   nz(x)    = (x + 0x7F7F7F7F) & 0x80808080       bit 7 of a byte set  <=> byte != 0
//   ge(a,b)  = ((a | 0x80808080) - b) & 0x80808080  bit 7 of a byte set  <=> a_byte >= b_byte
// The slide/merge itself runs on four scalar bytes per row after a branch-free transform of the
// board into the LEFT frame (transpose for UP/DOWN, byte-reverse for RIGHT/DOWN), so every lane of
// a wave executes the same instruction stream whatever its action.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace g2048 {

// v_bitop3_b32 (gfx950): any 3-input bitwise function in one VALU op.  The immediate is the truth
// table written with kA/kB/kC standing for the inputs a/b/c (e.g. kA ^ kB ^ kC = three-way xor).
constexpr uint32_t kA = 0xF0u, kB = 0xCCu, kC = 0xAAu;
template <uint32_t Imm>
__device__ __forceinline__ uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, Imm & 0xFFu);
}

__device__ __forceinline__ uint32_t zm(uint32_t x) { return bop3<~kA & kC>(x + 0x7F7F7F7Fu, 0u, 0x80808080u); }
__device__ __forceinline__ uint32_t nzm(uint32_t x) { return (x + 0x7F7F7F7Fu) & 0x80808080u; }
__device__ __forceinline__ uint32_t gem(uint32_t a, uint32_t b) { return ((a | 0x80808080u) - b) & 0x80808080u; }
__device__ __forceinline__ uint32_t eqm(uint32_t a, uint32_t b) { return zm(a ^ b); }

__device__ __forceinline__ uint32_t row(const uint4 &b, int i) {
    return i == 0 ? b.x : i == 1 ? b.y : i == 2 ? b.z : b.w;
}

// Bit a of the result = action a legal; the reference's scans (game.py:260-330) reduce to
// "an empty cell before a tile" or "two equal adjacent tiles" along the move axis.  Z[i] = bit 7
// of every empty byte of row i; every term is one or two v_bitop3.
__device__ __forceinline__ uint32_t legal_mask_z(const uint32_t (&r)[4], const uint32_t (&Z)[4]) {
    uint32_t L = 0u, R = 0u, U = 0u, D = 0u;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t zs = Z[i] >> 8;  // byte j: cell j+1 empty (byte 3: never)
        const uint32_t eq = bop3<~kA & ~kB & kC>((r[i] ^ (r[i] >> 8)) + 0x7F7F7F7Fu, Z[i], 0x00808080u);
        L |= bop3<(kA & ~kB & kC)>(Z[i], zs, 0x00808080u) | eq;  // empty j, tile j+1
        R |= bop3<(~kA & kB) | kC>(Z[i], zs, eq);                // tile j, empty j+1
    }
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const uint32_t eq = bop3<~kA & ~kB & kC>((r[i] ^ r[i + 1]) + 0x7F7F7F7Fu, Z[i], 0x80808080u);
        U |= bop3<(kA & ~kB) | kC>(Z[i], Z[i + 1], eq);  // empty above a tile
        D |= bop3<(~kA & kB) | kC>(Z[i], Z[i + 1], eq);  // tile above an empty cell
    }
    return (U ? 1u : 0u) | (D ? 2u : 0u) | (L ? 4u : 0u) | (R ? 8u : 0u);
}

__device__ __forceinline__ uint32_t legal_mask(const uint4 &b) {
    const uint32_t r[4] = {b.x, b.y, b.z, b.w};
    const uint32_t Z[4] = {zm(b.x), zm(b.y), zm(b.z), zm(b.w)};
    return legal_mask_z(r, Z);
}

__device__ __forceinline__ uint32_t bytemax(uint32_t a, uint32_t b) {
    const uint32_t g = gem(a, b);
    return bop3<(kC & kA) | (~kC & kB)>(a, b, g | (g - (g >> 7)));
}

// max exponent of a board: bytes split into 16-bit lanes, packed v_pk_max_u16 tree
typedef uint16_t g2048_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t board_max(const uint4 &b) {
    auto pk = [](uint32_t x) { return __builtin_bit_cast(g2048_u16x2, x); };
    const uint32_t m8 = 0x00FF00FFu;
    const g2048_u16x2 m0 = __builtin_elementwise_max(pk(b.x & m8), pk((b.x >> 8) & m8));
    const g2048_u16x2 m1 = __builtin_elementwise_max(pk(b.y & m8), pk((b.y >> 8) & m8));
    const g2048_u16x2 m2 = __builtin_elementwise_max(pk(b.z & m8), pk((b.z >> 8) & m8));
    const g2048_u16x2 m3 = __builtin_elementwise_max(pk(b.w & m8), pk((b.w >> 8) & m8));
    const uint32_t m = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_elementwise_max(m0, m1),
                                                                              __builtin_elementwise_max(m2, m3)));
    return max(m & 0xFFFFu, m >> 16);
}

__device__ __forceinline__ int emptiness(const uint4 &b) {  // game.py:671-680
    return __popc(zm(b.x)) + __popc(zm(b.y)) + __popc(zm(b.z)) + __popc(zm(b.w));
}

// game.py:683-800.  The best of the four clockwise rotations of (#left>=right + #top>=bottom over
// non-empty adjacent pairs) equals max(L,R) + max(T,B) with L/R/T/B those pair counts in the four
// orientations (each rotation pairs one horizontal with one vertical orientation).  Then x2 if the
// first row-major maximum sits in a corner, else floor(/2).
struct MonoStats {
    int L, R, T, B;
    uint32_t M;    // max exponent
    uint32_t pos;  // first row-major cell holding M
};

// first row-major cell whose byte equals M (M present on the board): per-row v_ffbl (~0 for a row
// without M, which never wins the unsigned min), row i offset by OR-ing 32*i into the bit index
// v_ffbl_b32 itself returns ~0 for a zero input; the generic count-trailing-zeros adds a compare and a
// select to guarantee that, so the instruction is written out
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t first_cell_eq(const uint32_t (&r)[4], uint32_t M) {
    const uint32_t mb = M * 0x01010101u;
    const uint32_t f0 = ffbl(zm(r[0] ^ mb)), f1 = ffbl(zm(r[1] ^ mb)) | 32u;
    const uint32_t f2 = ffbl(zm(r[2] ^ mb)) | 64u, f3 = ffbl(zm(r[3] ^ mb)) | 96u;
    return min(min(f0, f1), min(f2, f3)) >> 3;
}

__device__ __forceinline__ MonoStats mono_stats_z(const uint32_t (&r)[4], const uint32_t (&Z)[4], uint32_t M) {
    MonoStats s{0, 0, 0, 0, M, 0u};
    uint32_t X[4], NZ[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        X[i] = r[i] | 0x80808080u;
        NZ[i] = Z[i] ^ 0x80808080u;
    }
    uint32_t L = 0u, R = 0u, T = 0u, B = 0u;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t both = NZ[i] & (NZ[i] >> 8);
        L = __popc((X[i] - (r[i] >> 8)) & both) + L;
        R = __popc(((X[i] >> 8) - r[i]) & both) + R;
    }
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const uint32_t both = NZ[i] & NZ[i + 1];
        T = __popc((X[i] - r[i + 1]) & both) + T;
        B = __popc((X[i + 1] - r[i]) & both) + B;
    }
    s.L = (int)L;
    s.R = (int)R;
    s.T = (int)T;
    s.B = (int)B;
    s.pos = first_cell_eq(r, M);
    return s;
}

__device__ __forceinline__ MonoStats mono_stats(const uint4 &b) {
    const uint32_t r[4] = {b.x, b.y, b.z, b.w};
    const uint32_t Z[4] = {zm(b.x), zm(b.y), zm(b.z), zm(b.w)};
    return mono_stats_z(r, Z, board_max(b));
}

__device__ __forceinline__ int mono_value(const MonoStats &s) {
    const int best = max(s.L, s.R) + max(s.T, s.B);
    return ((0x9009u >> s.pos) & 1u) ? best * 2 : best >> 1;
}

__device__ __forceinline__ int monotonicity(const uint4 &b) { return mono_value(mono_stats(b)); }

// select dword i (0..3) of a board without a branch (arguments by value: a select between two
// fields of one in-memory uint4 would become a dynamically indexed private array)
__device__ __forceinline__ uint32_t pick_row(uint32_t x, uint32_t y, uint32_t z, uint32_t w, uint32_t i) {
    const uint64_t lo = ((uint64_t)y << 32) | x, hi = ((uint64_t)w << 32) | z;
    return (uint32_t)(((i & 2u) ? hi : lo) >> (32u * (i & 1u)));
}

// Statistics after placing exponent v on the EMPTY cell p of board b (the spawn): only the (up to
// four) pairs through p change, and the max / first-argmax.
__device__ __forceinline__ MonoStats mono_add_tile(MonoStats s, const uint4 &b, uint32_t p, uint32_t v) {
    const uint32_t r = p >> 2, c = p & 3u, sh = 8u * c;
    const uint32_t bx = b.x, by = b.y, bz = b.z, bw = b.w;
    const uint32_t row = pick_row(bx, by, bz, bw, r);
    const uint32_t upr = pick_row(0u, bx, by, bz, r);  // row r-1 (0 above the board)
    const uint32_t dnr = pick_row(by, bz, bw, 0u, r);  // row r+1 (0 below the board)
    const uint32_t left = c > 0u ? (row >> (sh - 8u)) & 0xFFu : 0u;
    const uint32_t right = (row >> sh) >> 8;  // c == 3: 0
    const uint32_t rt = right & 0xFFu;
    const uint32_t up = (upr >> sh) & 0xFFu, dn = (dnr >> sh) & 0xFFu;
    s.L += (int)((left != 0u) & (left >= v)) + (int)((rt != 0u) & (v >= rt));
    s.R += (int)((left != 0u) & (v >= left)) + (int)((rt != 0u) & (rt >= v));
    s.T += (int)((up != 0u) & (up >= v)) + (int)((dn != 0u) & (v >= dn));
    s.B += (int)((up != 0u) & (v >= up)) + (int)((dn != 0u) & (dn >= v));
    const bool gt = v > s.M, eq = v == s.M;
    s.pos = gt ? p : (eq ? min(s.pos, p) : s.pos);
    s.M = gt ? v : s.M;
    return s;
}

// 4x4 byte transpose in two stages of v_perm_b32 (8 byte-selects instead of shift/mask/or chains):
// interleave the low / high byte pairs of rows (0, 1) and (2, 3), then gather each column.
// __builtin_amdgcn_perm(hi, lo, sel): selector bytes 0-3 pick bytes of lo, 4-7 bytes of hi.
__device__ __forceinline__ uint4 transpose(const uint4 &b) {
    const uint32_t p = __builtin_amdgcn_perm(b.y, b.x, 0x05010400u);  // a0 b0 a1 b1
    const uint32_t q = __builtin_amdgcn_perm(b.y, b.x, 0x07030602u);  // a2 b2 a3 b3
    const uint32_t u = __builtin_amdgcn_perm(b.w, b.z, 0x05010400u);  // c0 d0 c1 d1
    const uint32_t v = __builtin_amdgcn_perm(b.w, b.z, 0x07030602u);  // c2 d2 c3 d3
    return make_uint4(__builtin_amdgcn_perm(u, p, 0x05040100u), __builtin_amdgcn_perm(u, p, 0x07060302u),
                      __builtin_amdgcn_perm(v, q, 0x05040100u), __builtin_amdgcn_perm(v, q, 0x07060302u));
}

__device__ __forceinline__ uint4 bswap4(const uint4 &b) {
    return make_uint4(__builtin_bswap32(b.x), __builtin_bswap32(b.y), __builtin_bswap32(b.z),
                      __builtin_bswap32(b.w));
}

__device__ __forceinline__ uint4 sel4(bool c, const uint4 &a, const uint4 &b) {
    return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

// _merge_and_shift_left_with_score (game.py:225-244) on one row dword.  Compaction is a stable
// zero-bubbling network, then the greedy leading-edge merge written as selects.
__device__ __forceinline__ uint32_t slide_row_left(uint32_t x, uint32_t &pts, uint32_t &mx) {
    uint32_t y0 = x & 0xFFu, y1 = (x >> 8) & 0xFFu, y2 = (x >> 16) & 0xFFu, y3 = x >> 24;
#define G2048_CSWAP(a, b)              \
    {                                  \
        const bool z = (a) == 0u;      \
        (a) = z ? (b) : (a);           \
        (b) = z ? 0u : (b);            \
    }
    G2048_CSWAP(y0, y1) G2048_CSWAP(y1, y2) G2048_CSWAP(y2, y3)
    G2048_CSWAP(y0, y1) G2048_CSWAP(y1, y2)
    G2048_CSWAP(y0, y1)
#undef G2048_CSWAP
    const bool m01 = (y0 != 0u) & (y0 == y1);
    const bool m12 = !m01 & (y1 != 0u) & (y1 == y2);
    const bool m23 = (y2 != 0u) & (y2 == y3) & !m12;
    const uint32_t o0 = y0 + (m01 ? 1u : 0u);
    const uint32_t o1 = m01 ? y2 + (m23 ? 1u : 0u) : y1 + (m12 ? 1u : 0u);
    const uint32_t o2 = m01 ? (m23 ? 0u : y3) : (m12 ? y3 : y2 + (m23 ? 1u : 0u));
    const uint32_t o3 = (m01 | m12 | m23) ? 0u : y3;
    pts += (m01 ? (1u << (y0 + 1u)) : 0u) + (m12 ? (1u << (y1 + 1u)) : 0u) + (m23 ? (1u << (y2 + 1u)) : 0u);
    mx = max(mx, max(m01 ? y0 + 1u : 0u, max(m12 ? y1 + 1u : 0u, m23 ? y2 + 1u : 0u)));
    return o0 | (o1 << 8) | (o2 << 16) | (o3 << 24);
}

// simulate_move (game.py:122-160) for a per-lane action, branch-free.
__device__ __forceinline__ uint4 apply_move(const uint4 &b, uint32_t action, uint32_t &pts, uint32_t &mx) {
    const bool vert = action < 2u;                         // UP, DOWN work on columns
    const bool rev = (action == 1u) | (action == 3u);      // DOWN, RIGHT slide toward the far edge
    uint4 w = sel4(vert, transpose(b), b);
    w = sel4(rev, bswap4(w), w);
    pts = 0u;
    mx = 0u;
    w.x = slide_row_left(w.x, pts, mx);
    w.y = slide_row_left(w.y, pts, mx);
    w.z = slide_row_left(w.z, pts, mx);
    w.w = slide_row_left(w.w, pts, mx);
    w = sel4(rev, bswap4(w), w);
    return sel4(vert, transpose(w), w);
}

__device__ __forceinline__ uint32_t nibble_of(uint32_t m80) {  // bits 7,15,23,31 -> bits 0..3
    const uint32_t t = m80 >> 7;
    return (t | (t >> 7) | (t >> 14) | (t >> 21)) & 0xFu;
}

__device__ __forceinline__ uint32_t empty_mask16(const uint4 &b) {  // bit 4i+j = cell (i,j) empty
    return nibble_of(zm(b.x)) | (nibble_of(zm(b.y)) << 4) | (nibble_of(zm(b.z)) << 8) |
           (nibble_of(zm(b.w)) << 12);
}

// position of the k-th (0-based) set bit of a 16-bit mask (k < popcount)
__device__ __forceinline__ uint32_t kth_bit16(uint32_t m, uint32_t k) {
    uint32_t pos = 0, c;
    c = __popc(m & 0xFFu); if (k >= c) { k -= c; m >>= 8; pos += 8; }
    c = __popc(m & 0xFu);  if (k >= c) { k -= c; m >>= 4; pos += 4; }
    c = __popc(m & 0x3u);  if (k >= c) { k -= c; m >>= 2; pos += 2; }
    c = m & 1u;            if (k >= c) { pos += 1; }
    return pos;
}

// k-th (0-based) set bit of a 4-bit mask m (k < popcount(m)): 2-bit answers packed per k in a
// 32-bit constant indexed by m
__device__ __forceinline__ uint32_t kth_bit4(uint32_t m, uint32_t k) {
    constexpr uint32_t T[4] = {
        [] { uint32_t t = 0; for (uint32_t m = 1; m < 16; m++) { uint32_t j = 0; while (!((m >> j) & 1u)) j++; t |= j << (2 * m); } return t; }(),
        [] { uint32_t t = 0; for (uint32_t m = 1; m < 16; m++) { uint32_t c = 0, j = 0; for (; j < 4; j++) if ((m >> j) & 1u) { if (c == 1) break; c++; } t |= (j & 3u) << (2 * m); } return t; }(),
        [] { uint32_t t = 0; for (uint32_t m = 1; m < 16; m++) { uint32_t c = 0, j = 0; for (; j < 4; j++) if ((m >> j) & 1u) { if (c == 2) break; c++; } t |= (j & 3u) << (2 * m); } return t; }(),
        [] { uint32_t t = 0; for (uint32_t m = 1; m < 16; m++) { uint32_t c = 0, j = 0; for (; j < 4; j++) if ((m >> j) & 1u) { if (c == 3) break; c++; } t |= (j & 3u) << (2 * m); } return t; }(),
    };
    const uint32_t t01 = (k & 1u) ? T[1] : T[0], t23 = (k & 1u) ? T[3] : T[2];
    return ((k & 2u) ? t23 : t01) >> (2u * m) & 3u;
}

__device__ __forceinline__ void set_cell(uint4 &b, uint32_t pos, uint32_t v) {
    const uint32_t sh = (pos & 3u) * 8u, bits = v << sh, r = pos >> 2;
    b.x |= r == 0u ? bits : 0u;
    b.y |= r == 1u ? bits : 0u;
    b.z |= r == 2u ? bits : 0u;
    b.w |= r == 3u ? bits : 0u;
}

__device__ __forceinline__ bool eq4(const uint4 &a, const uint4 &b) {
    return ((a.x ^ b.x) | (a.y ^ b.y) | (a.z ^ b.z) | (a.w ^ b.w)) == 0u;
}

// ---------------------------------------------------------------- Philox4x32-10 -------------
// One 32x32->64 product per multiplier (v_mad_u64_u32) instead of separate mul_lo/mul_hi.
__device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        c0 = bop3<kA ^ kB ^ kC>((uint32_t)(p1 >> 32), c1, k0);
        c1 = (uint32_t)p1;
        c2 = bop3<kA ^ kB ^ kC>((uint32_t)(p0 >> 32), c3, k1);
        c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

// Philox in two pieces (rounds [R0, R1) on a running state) so a kernel can place the halves into
// memory-latency windows; philox_rounds<0,10> of the initial state == philox().
struct PhiloxState {
    uint32_t c0, c1, c2, c3, k0, k1;
};
__device__ __forceinline__ PhiloxState philox_start(uint64_t seed, uint64_t step, uint32_t env, uint32_t stream) {
    return PhiloxState{(uint32_t)step, (uint32_t)(step >> 32), env, stream, (uint32_t)seed, (uint32_t)(seed >> 32)};
}
template <int R0, int R1>
__device__ __forceinline__ void philox_rounds(PhiloxState &s) {
#pragma unroll
    for (int r = R0; r < R1; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * s.c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * s.c2;
        s.c0 = bop3<kA ^ kB ^ kC>((uint32_t)(p1 >> 32), s.c1, s.k0 + (uint32_t)r * 0x9E3779B9u);
        s.c1 = (uint32_t)p1;
        s.c2 = bop3<kA ^ kB ^ kC>((uint32_t)(p0 >> 32), s.c3, s.k1 + (uint32_t)r * 0xBB67AE85u);
        s.c3 = (uint32_t)p0;
    }
}

__device__ __forceinline__ uint4 philox_draw(uint64_t seed, uint64_t step, uint32_t env, uint32_t stream) {
    return philox((uint32_t)step, (uint32_t)(step >> 32), env, stream, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// The transcendentals of the masked-softmax sampler (g2048.hip sample_kernel and the fused rollout's
// sample_row, bitwise the same code).  Round 5: the hardware forms (v_exp_f32 / v_log_f32 /
// v_rcp_f32, ~1e-7 relative) instead of the correctly rounded libm sequences (~15 VALU each, five per
// sampled row): logp / entropy stay within the 1e-5 of the reference's golden rows
// (test_sampler_matches_reference_masked_softmax).  G2048_SAMPLE_EXACT restores the libm forms.
#ifdef G2048_SAMPLE_EXACT
__device__ __forceinline__ float smp_exp(float x) { return expf(x); }
__device__ __forceinline__ float smp_log(float x) { return logf(x); }
__device__ __forceinline__ float smp_rcp(float x) { return 1.0f / x; }
#else
__device__ __forceinline__ float smp_exp(float x) { return __expf(x); }
__device__ __forceinline__ float smp_log(float x) { return __logf(x); }
__device__ __forceinline__ float smp_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
#endif

// 0.9 threshold of `random.random() < 0.9` (game.py:939) on a 32-bit uniform: u*2^-32 < 0.9
constexpr uint32_t kTwoThreshold = 3865470567u;

// ---------------------------------------------------------------- MT19937 (parity) ----------
// Word-major state: word w of env e lives at st[w * n + e] (w = 624 is the output index), so a
// wave's accesses to the same word are contiguous.
struct MT {
    uint32_t *st = nullptr;
    int64_t n = 0, e = 0;
    uint32_t idx = 0;
    __device__ void load(uint32_t *s, int64_t n_, int64_t e_) {
        st = s;
        n = n_;
        e = e_;
        idx = st[624 * n + e];
    }
    __device__ void save() { st[624 * n + e] = idx; }
    __device__ uint32_t &w(int k) { return st[(int64_t)k * n + e]; }
    __device__ uint32_t next() {
        if (idx >= 624u) {
            for (int kk = 0; kk < 624; kk++) {
                const uint32_t y = (w(kk) & 0x80000000u) | (w(kk + 1 < 624 ? kk + 1 : 0) & 0x7fffffffu);
                const int src = kk + 397 < 624 ? kk + 397 : kk + 397 - 624;
                w(kk) = w(src) ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            idx = 0;
        }
        uint32_t y = w(idx++);
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    __device__ uint32_t randbelow(uint32_t m) {  // random.Random._randbelow_with_getrandbits
        const int k = 32 - __clz(m);
        for (;;) {
            const uint32_t r = next() >> (32 - k);
            if (r < m) return r;
        }
    }
    __device__ bool below_09() {  // random.random() < 0.9
        const uint32_t a = next() >> 5, b = next() >> 6;
        return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0) < 0.9;
    }
};

}  // namespace g2048
