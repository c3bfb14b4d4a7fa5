// env_rollout.hip -- the synthetic random-legal rollout (the bench's headline workload,
// g2048_env_rollout_random / _adv of include/g2048.h): env_rollout_kernel with its LDS tables and
// per-step helpers, in a translation unit of its own so that it alone is built with the machine
// scheduler's occupancy bias at 0 (Makefile: one wave per SIMD at the benchmark size, where the issue
// schedule, not occupancy, sets the step time; the rest of libg2048 keeps the default bias).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "board.hpp"
#include "rowtable.hpp"
#include "step.hpp"
#include "launch_util.hpp"
#include "../../include/g2048.h"

using namespace g2048;

namespace {

__device__ const lut::Row12Table kRow12 __attribute__((aligned(16))) = lut::Row12Table();
__device__ const lut::Line12Table kLine12 __attribute__((aligned(16))) = lut::Line12Table();

// LDS layout of env_rollout_kernel: kLine12 at byte 0 (41 KiB, so a line's byte address 2 idx fits
// in 16 bits and four of them come out of packed-u16 arithmetic), kRow12 right after it.  Lanes
// whose board holds an exponent >= 12 still issue the (discarded) table reads with 4-bit-masked
// digits, i.e. indices up to 15 * 1885 = 28 275: a kLine12 read may then land in kRow12 and a
// kRow12 read in kFresh (harmless: both inside the allocation).
constexpr uint32_t kRowLds = lut::kLineEntriesPadded * 2u;                   // 41 984
// then the auto-reset boards and their statistics (kFresh)
__device__ const lut::FreshTable kFresh __attribute__((aligned(16))) = lut::FreshTable();
constexpr uint32_t kFreshBoardBase = 137u * 1024u;                          // 15 KiB of boards
constexpr uint32_t kFreshStatBase = kFreshBoardBase + lut::kFreshEntries * 16u;  // 4 KiB of stats
constexpr uint32_t kRolloutLdsWords = (kFreshStatBase + 4096u) / 4u;         // 159 744 B
static_assert(kRowLds + lut::kRowEntries * 4u <= kFreshBoardBase, "kRow12 below kFresh");
static_assert(kRowLds + 4u * 28276u <= kRolloutLdsWords * 4u, "masked kRow12 reads stay inside the allocation");
// kLine12 reads take unmasked digits (line12_addrs): exponents <= 17 and the spawn's + 2 x 2 x 12^3
static_assert(2u * 17u * 1885u + 2u * 2u * 1728u + 2u <= kRolloutLdsWords * 4u, "kLine12 reads stay inside the allocation");
static_assert(2u * (lut::kRowEntries - 1u) < 65536u, "kLine12 byte addresses fit 16 bits");

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }

// LDS byte address of the kRow12 entry of a LEFT-frame row dword (byte j = cell j):
// kRowLds + 4 (c0 + 12 c1 + 144 c2 + 1728 c3) as two packed-u16 dot products.  Bytes are masked
// to 4 bits so any row (even one holding exponents >= 12, whose lane takes the compute path)
// addresses inside the LDS allocation (< kRowLds + 15 * 1885 * 4 bytes).
// kSmall (every exponent <= 10): the digits need no mask, so each pair is one byte-select v_perm
template <bool kSmall = false>
__device__ __forceinline__ uint32_t row12_addr(uint32_t x) {
    const u16x2 k02 = {4, 576}, k13 = {48, 6912};
    const uint32_t a = kSmall ? __builtin_amdgcn_perm(0u, x, 0x0C020C00u) : x & 0x000F000Fu;         // cells 0, 2
    const uint32_t b = kSmall ? __builtin_amdgcn_perm(0u, x, 0x0C030C01u) : (x >> 8) & 0x000F000Fu;  // cells 1, 3
    return __builtin_amdgcn_udot2(as_u16x2(b), k13, __builtin_amdgcn_udot2(as_u16x2(a), k02, kRowLds, false), false);
}
__device__ __forceinline__ uint32_t lds_word(const uint32_t *tab, uint32_t addr) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(tab) + addr);
}
// LDS byte addresses (2 idx) of the kLine12 entries of a board's four rows (a row read left to
// right) and four columns (top to bottom), from the rows' 4-bit digit pairs: A_i = cells (i, 0) and
// (i, 2), B_i = cells (i, 1) and (i, 3) as u16 halves.  Rows: two packed-u16 dot products each.
// Columns: column pairs (0, 2) and (1, 3) at once as packed-u16 multiply-adds over the rows,
// 2 (cell(0, j) + 12 cell(1, j) + 144 cell(2, j) + 1728 cell(3, j)) < 2^16 per half -- no transpose.
// The digit pairs are the bytes themselves (one v_perm each, no 4-bit mask): a board of the SWAR
// fallback (exponents up to 17) gives indices up to 2 x 17 x 1885 = 64 090 bytes, inside the LDS
// allocation (its reads are discarded), and no u16 sum below overflows.
__device__ __forceinline__ void line12_addrs(const uint4 &b, uint32_t (&ra)[4], uint32_t (&ca)[4]) {
    const u16x2 k02 = {2, 288}, k13 = {24, 3456};
    const uint32_t w[4] = {b.x, b.y, b.z, b.w};
    u16x2 A[4], B[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        A[i] = as_u16x2(__builtin_amdgcn_perm(0u, w[i], 0x0C020C00u));
        B[i] = as_u16x2(__builtin_amdgcn_perm(0u, w[i], 0x0C030C01u));
        ra[i] = __builtin_amdgcn_udot2(B[i], k13, __builtin_amdgcn_udot2(A[i], k02, 0u, false), false);
    }
    const u16x2 c02 = A[0] * (u16x2){2, 2} + A[1] * (u16x2){24, 24} + A[2] * (u16x2){288, 288} + A[3] * (u16x2){3456, 3456};
    const u16x2 c13 = B[0] * (u16x2){2, 2} + B[1] * (u16x2){24, 24} + B[2] * (u16x2){288, 288} + B[3] * (u16x2){3456, 3456};
    const uint32_t p02 = __builtin_bit_cast(uint32_t, c02), p13 = __builtin_bit_cast(uint32_t, c13);
    ca[0] = p02 & 0xFFFFu;
    ca[1] = p13 & 0xFFFFu;
    ca[2] = p02 >> 16;
    ca[3] = p13 >> 16;
}
__device__ __forceinline__ uint32_t lds_half(const uint32_t *tab, uint32_t addr) {
    return *reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(tab) + addr);
}
// byte-reverse each row when the lane's selector says so (one v_perm per row, no select)
__device__ __forceinline__ uint4 perm4(const uint4 &w, uint32_t sel) {
    return make_uint4(__builtin_amdgcn_perm(w.x, w.x, sel), __builtin_amdgcn_perm(w.y, w.y, sel),
                      __builtin_amdgcn_perm(w.z, w.z, sel), __builtin_amdgcn_perm(w.w, w.w, sel));
}

// nibble-packed row (bits 0..15 of a table entry) -> row dword with one exponent per byte, byte
// reversed or not by the lane's selector: nibble j is the low nibble of byte j/2 of e (j even) or of
// e >> 4 (j odd), so one v_perm over (e >> 4, e) places all four and a mask clears the high nibbles.
constexpr uint32_t kUnpackSel = 0x05010400u;     // bytes {n0, n1, n2, n3}
constexpr uint32_t kUnpackRevSel = 0x00040105u;  // bytes {n3, n2, n1, n0}
__device__ __forceinline__ uint32_t unpack_row(uint32_t e, uint32_t sel) {
    return __builtin_amdgcn_perm(e >> 4, e, sel) & 0x0F0F0F0Fu;
}

// Packed monotonicity statistics of the rollout kernel, one VGPR per board: bits 0..3 pos (the
// first row-major cell holding the maximum), 8..11 L, 12..15 R, 16..19 T, 20..23 B (board.hpp
// MonoStats), 24..27 M.  Bytes 1 and 2 are the low bytes of a board's kLine12 row / column sums.
__device__ __forceinline__ uint32_t pack_stats(const MonoStats &s) {
    return s.pos | ((uint32_t)s.L << 8) | ((uint32_t)s.R << 12) | ((uint32_t)s.T << 16) | ((uint32_t)s.B << 20) |
           (s.M << 24);
}
// board.hpp mono_value on the packed word: (L, T) and (R, B) as u16 pairs (L, R scaled by 256),
// one packed max and one dot product give 256 (max(L, R) + max(T, B)); x2 for a corner maximum
// (>> 7), floor(/2) otherwise (>> 9).  The bit-field extract reads its offset from bits 0..4 of S.
__device__ __forceinline__ uint32_t mono_value_packed(uint32_t S) {
    const u16x2 m = __builtin_elementwise_max(as_u16x2(S & 0x000F0F00u), as_u16x2((S >> 4) & 0x000F0F00u));
    const uint32_t best256 = __builtin_amdgcn_udot2(m, (u16x2){1, 256}, 0u, false);
    const uint32_t corner = __builtin_amdgcn_ubfe(0x9009u, S, 1u);
    return best256 >> (9u - 2u * corner);
}
// L|R and T|B bytes of a board's kLine12 row sum SR and column sum SC into bytes 1 and 2
__device__ __forceinline__ uint32_t stats_bytes(uint32_t SR, uint32_t SC) {
    return __builtin_amdgcn_perm(SC, SR, 0x0C04000Cu);
}

// Game2048.reset (game.py:942-950) from the four words of one Philox draw: the two spawns of reset()
// on an empty board (same result as fresh_board<Philox>: 16 empties, then 15).
__device__ __forceinline__ uint4 fresh_from_words(const uint4 &r, uint32_t &p1, uint32_t &v1, uint32_t &p2,
                                                  uint32_t &v2) {
    p1 = r.x >> 28;  // (x * 16) >> 32
    v1 = r.y < kTwoThreshold ? 1u : 2u;
    const uint32_t k2 = (uint32_t)(((uint64_t)r.z * 15u) >> 32);
    p2 = k2 + (k2 >= p1 ? 1u : 0u);
    v2 = r.w < kTwoThreshold ? 1u : 2u;
    uint4 b = make_uint4(0u, 0u, 0u, 0u);
    set_cell(b, p1, v1);
    set_cell(b, p2, v2);
    return b;
}

// The rollout kernel's auto-reset from two spare words (oracle or_reset_words): cell 1 = a >> 28,
// its value from the other 28 bits of a; cell 2 = floor(bw * 15 / 2^32) among the 15 cells left,
// its value from the low word of bw * 15.
__device__ __forceinline__ uint4 fresh_from_pair(uint32_t a, uint32_t bw, uint32_t &p1, uint32_t &v1, uint32_t &p2,
                                                 uint32_t &v2) {
    p1 = a >> 28;
    v1 = (a << 4) < kTwoThreshold ? 1u : 2u;
    const uint32_t k2 = __umulhi(bw, 15u);
    p2 = k2 + (k2 >= p1 ? 1u : 0u);
    v2 = bw * 15u < kTwoThreshold ? 1u : 2u;
    uint4 b = make_uint4(0u, 0u, 0u, 0u);
    set_cell(b, p1, v1);
    set_cell(b, p2, v2);
    return b;
}

// Legal mask and monotonicity statistics of a fresh two-tile board in closed form (tiles v1 at p1,
// v2 at p2, p1 != p2).  A direction is blocked only when both tiles already sit against its edge
// on different lines, or they are the two leading cells of one line with different values.
__device__ __forceinline__ uint32_t fresh_stats(uint32_t p1, uint32_t v1, uint32_t p2, uint32_t v2, MonoStats &s) {
    const uint32_t r1 = p1 >> 2, c1 = p1 & 3u, r2 = p2 >> 2, c2 = p2 & 3u;
    const bool same_row = r1 == r2, same_col = c1 == c2, ne = v1 != v2;
    const uint32_t sc = c1 + c2, sr = r1 + r2;
    // blocked-direction bits as 0/1 integers (bool selects here compile to divergent branches)
    const uint32_t srw = same_row, scl = same_col, nev = ne;
    const uint32_t left_blk = (srw & nev & (uint32_t)(sc == 1u)) | ((srw ^ 1u) & (uint32_t)(sc == 0u));
    const uint32_t right_blk = (srw & nev & (uint32_t)(sc == 5u)) | ((srw ^ 1u) & (uint32_t)(sc == 6u));
    const uint32_t up_blk = (scl & nev & (uint32_t)(sr == 1u)) | ((scl ^ 1u) & (uint32_t)(sr == 0u));
    const uint32_t down_blk = (scl & nev & (uint32_t)(sr == 5u)) | ((scl ^ 1u) & (uint32_t)(sr == 6u));
    const uint32_t legal = 15u ^ (up_blk | (down_blk << 1) | (left_blk << 2) | (right_blk << 3));
    const bool hadj = same_row & ((max(c1, c2) - min(c1, c2)) == 1u);
    const bool vadj = same_col & ((max(r1, r2) - min(r1, r2)) == 1u);
    const uint32_t lv = c1 < c2 ? v1 : v2, rv = c1 < c2 ? v2 : v1;  // left / right tile (same row)
    const uint32_t tv = r1 < r2 ? v1 : v2, bv = r1 < r2 ? v2 : v1;  // top / bottom tile (same column)
    s.L = (int)(hadj & (lv >= rv));
    s.R = (int)(hadj & (rv >= lv));
    s.T = (int)(vadj & (tv >= bv));
    s.B = (int)(vadj & (bv >= tv));
    s.M = max(v1, v2);
    s.pos = v1 > v2 ? p1 : v2 > v1 ? p2 : min(p1, p2);
    return legal;
}

// Copy the tables (kLine12, kRow12, kFresh) into LDS by LDS-DMA: each wave instruction moves 1 KiB (16 B per lane)
// straight from global memory into LDS with no VGPR staging, and every piece of the wave is in
// flight before the single wait (one L2/MALL round trip per launch instead of one per batch).
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
__device__ __forceinline__ void stage_row_table(uint32_t *s_row) {
    constexpr int kPieces = (int)(lut::kRowEntries * 4u / 1024u);  // 81 pieces of 1 KiB
    constexpr int kLinePieces = (int)(lut::kLineEntriesPadded * 2u / 1024u);  // + 41 of kLine12
    constexpr int kFreshPieces = (int)(lut::kFreshEntries * 16u / 1024u);  // + 15 boards + 4 stats
    static_assert(lut::kRowEntries * 4u % 1024u == 0u && lut::kLineEntriesPadded * 2u % 1024u == 0u &&
                  lut::kFreshEntries * 16u % 1024u == 0u, "whole 1 KiB pieces");
    constexpr int kAll = kPieces + kLinePieces + kFreshPieces + 4;
    const char *src = reinterpret_cast<const char *>(kLine12.v);  // pieces 0 .. kLinePieces - 1
    const char *src2 = reinterpret_cast<const char *>(kRow12.v);
    const char *src3 = reinterpret_cast<const char *>(kFresh.b);
    const char *src4 = reinterpret_cast<const char *>(kFresh.st);
    char *dst = reinterpret_cast<char *>(s_row);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int c = wave; c < kAll; c += nw) {
        const char *g;
        uint32_t d;
        if (c < kPieces + kLinePieces) {  // kLine12 at 0, then kRow12 at kRowLds (= kLinePieces KiB)
            g = c < kLinePieces ? src + 1024 * c : src2 + 1024 * (c - kLinePieces);
            d = 1024u * (uint32_t)c;
        } else if (c < kPieces + kLinePieces + kFreshPieces) {
            const int k = c - kPieces - kLinePieces;
            g = src3 + 1024 * k;
            d = kFreshBoardBase + 1024u * (uint32_t)k;
        } else {
            const int k = c - kPieces - kLinePieces - kFreshPieces;
            g = src4 + 1024 * k;
            d = kFreshStatBase + 1024u * (uint32_t)k;
        }
        __builtin_amdgcn_global_load_lds((glb_void_t *)(g + 16 * lane), (lds_void_t *)(dst + d), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0): this wave's pieces have landed
    __syncthreads();
}

// Per-lane state of the rollout carried from step to step.
struct RolloutLane {
    uint4 b;          // current board (never finished between steps)
    uint32_t legal;   // its legal mask
    uint32_t S;       // its packed monotonicity statistics (pack_stats)
    int empt_b;       // its empty-cell count
    uint4 D;          // Philox draw of the current pair of steps: x / y = the two steps' words,
                      // z / w = the words of a reset inside the pair (at most one: a reset board
                      // cannot end again one move later)
    PhiloxState ph;   // draw of the next pair, computed half per step inside the LDS round trip
    uint4 fb;         // the board a reset inside the current pair starts (D.z, D.w -> kFresh) ...
    uint32_t flegal;  // ... its legal mask and packed statistics
    uint32_t fS;
};

// the current pair's auto-reset board from kFresh (fresh_from_pair's board and fresh_stats' results,
// read once per pair right after the draw is known, long before a step can need them)
__device__ __forceinline__ void fresh_prep(RolloutLane &s, const uint32_t *__restrict__ tab) {
    const uint32_t a = s.D.z, bw = s.D.w;
    const uint64_t pb = (uint64_t)bw * 15u;  // one v_mad_u64_u32: k2 and the low word
    const uint32_t k2 = (uint32_t)(pb >> 32);
    const uint32_t i = 60u * (a >> 28) + 4u * k2 + ((a << 4) >= kTwoThreshold ? 2u : 0u) +
                       ((uint32_t)pb >= kTwoThreshold ? 1u : 0u);
    const char *t = reinterpret_cast<const char *>(tab);
    s.fb = *reinterpret_cast<const uint4 *>(t + kFreshBoardBase + 16u * i);
    const uint32_t st = *reinterpret_cast<const uint32_t *>(t + kFreshStatBase + 4u * i);
    s.flegal = st >> 28;
    s.fS = st & 0x0FFFFFFFu;
}

struct TrajRows {  // this lane's element of row t of each time-major trajectory array (advanced by n per step)
    uint4 *b;
    uint8_t *a;
    int32_t *p;
    uint32_t *pot;
    uint8_t *f;
    __device__ __forceinline__ void next(int64_t n) {
        b += n;
        a += n;
        p += n;
        pot += n;
        f += n;
    }
};


// One env step of the synthetic random-legal policy (oracle or_step_word + auto-reset).  kOdd = the
// second step of the pair.  One 32-bit word u per step: action k = floor(u * nlegal / 2^32); the
// low word r of that product (uniform given k) picks the spawn cell and value.
template <bool kOdd, bool kSmall = false>
__device__ __forceinline__ void rollout_step(RolloutLane &s, const uint32_t *__restrict__ tab, const TrajRows &tr,
                                             uint64_t seed, uint64_t next_pair, uint32_t env) {
    *tr.b = s.b;
    const uint32_t u = kOdd ? s.D.y : s.D.x;
    const uint64_t pa = (uint64_t)u * (uint32_t)__popc(s.legal);
    const uint32_t a = kth_bit4(s.legal, (uint32_t)(pa >> 32)), r = (uint32_t)pa;
    // the move through the LDS row table in the LEFT frame.  Half of the next pair's Philox rounds
    // fill the LDS round trip: the empty asm statements start them after the table loads are issued
    // (memory clobber) and consume the loaded entries after them.
    const bool vert = a < 2u, rev = (a & 1u) != 0u;  // DOWN / RIGHT: byte-reversed rows
    const uint32_t rsel = rev ? 0x00010203u : 0x03020100u, usel = rev ? kUnpackRevSel : kUnpackSel;
    uint4 w = perm4(sel4(vert, transpose(s.b), s.b), rsel);
    uint32_t e0 = lds_word(tab, row12_addr<kSmall>(w.x)), e1 = lds_word(tab, row12_addr<kSmall>(w.y));
    uint32_t e2 = lds_word(tab, row12_addr<kSmall>(w.z)), e3 = lds_word(tab, row12_addr<kSmall>(w.w));
    asm volatile("" : "+v"(s.ph.c0), "+v"(s.ph.c1), "+v"(s.ph.c2), "+v"(s.ph.c3)::"memory");
    if constexpr (kOdd) philox_rounds<5, 10>(s.ph);
    else philox_rounds<0, 5>(s.ph);
    asm volatile("" : "+v"(s.ph.c0), "+v"(s.ph.c1), "+v"(s.ph.c2), "+v"(s.ph.c3), "+v"(e0), "+v"(e1), "+v"(e2), "+v"(e3));
    const uint32_t mono_b = mono_value_packed(s.S);
    w = make_uint4(unpack_row(e0, usel), unpack_row(e1, usel), unpack_row(e2, usel), unpack_row(e3, usel));
    uint4 moved = sel4(vert, transpose(w), w);
    // merge points / 4 in bits 16..27 of each entry, the slid row's maximum in bits 28..31
    uint32_t pts = (((e0 >> 16) & 0xFFFu) + ((e1 >> 16) & 0xFFFu) + ((e2 >> 16) & 0xFFFu) + ((e3 >> 16) & 0xFFFu)) << 2;
    uint32_t Ma = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_elementwise_max(as_u16x2(e0), as_u16x2(e1)),
                                                                         __builtin_elementwise_max(as_u16x2(e2), as_u16x2(e3)))) >> 28;
    if (!kSmall && (s.S >> 24) > 11u) {  // an exponent outside the table: the SWAR compute path
        uint32_t mx;
        moved = apply_move(s.b, a, pts, mx);
        Ma = board_max(moved);
    }
    const uint32_t rm[4] = {moved.x, moved.y, moved.z, moved.w};
    const uint32_t Zm[4] = {zm(moved.x), zm(moved.y), zm(moved.z), zm(moved.w)};
    const uint32_t pos_a = first_cell_eq(rm, Ma);
    // the moved board's (pre-spawn) lines in kLine12: four rows and four columns, read before the
    // spawn is known; the spawn then changes one row and one column, read again below
    uint32_t ra[4], ca[4];
    line12_addrs(moved, ra, ca);
    const uint32_t f0 = lds_half(tab, ra[0]), f1 = lds_half(tab, ra[1]), f2 = lds_half(tab, ra[2]), f3 = lds_half(tab, ra[3]);
    const uint32_t g0 = lds_half(tab, ca[0]), g1 = lds_half(tab, ca[1]), g2 = lds_half(tab, ca[2]), g3 = lds_half(tab, ca[3]);
    // spawn on the k-th empty cell (row-major), k = floor(r * empties / 2^32), value 1 if the low
    // word of r * empties is below 0.9 * 2^32 (given k that low word is uniform to within
    // empties / 2^32); the row from the prefix counts of empties, the column inside the row likewise
    const uint32_t n0 = __popc(Zm[0]), n01 = __popc(Zm[1]) + n0, n012 = __popc(Zm[2]) + n01;
    const uint32_t empt_a = __popc(Zm[3]) + n012;
    const uint64_t prod = (uint64_t)r * empt_a;
    const uint32_t k = (uint32_t)(prod >> 32);
    const uint32_t v = (uint32_t)prod < kTwoThreshold ? 1u : 2u;
    const bool r1 = k >= n0, r2 = k >= n01, r3 = k >= n012;  // spawn row >= 1, >= 2, == 3
    const uint32_t kr = k - (r3 ? n012 : r2 ? n01 : r1 ? n0 : 0u);
    const uint32_t z = r3 ? Zm[3] : r2 ? Zm[2] : r1 ? Zm[1] : Zm[0];
    const uint32_t b0 = (z >> 7) & 1u, b01 = b0 + ((z >> 15) & 1u), b012 = b01 + ((z >> 23) & 1u);
    const bool c1 = kr >= b0, c2 = kr >= b01, c3 = kr >= b012;  // spawn column >= 1, >= 2, == 3
    const uint32_t row = (uint32_t)r1 + (uint32_t)r2 + (uint32_t)r3, col = (uint32_t)c1 + (uint32_t)c2 + (uint32_t)c3;
    const uint32_t sp = 4u * row + col;
    const uint4 pre = moved;
    const uint32_t bits = v << (8u * col);
    moved.x |= r1 ? 0u : bits;
    moved.y |= (r1 && !r2) ? bits : 0u;
    moved.z |= (r2 && !r3) ? bits : 0u;
    moved.w |= r3 ? bits : 0u;
    s.b = moved;  // the next board (after the spawn)
    // the spawn's row and column in the next board: kLine12 byte address + v * 2 * 12^(column / row)
    constexpr uint64_t kW12 = 0x0D80012000180002ull;  // {2, 24, 288, 3456}
    const uint32_t rp = r3 ? ra[3] : r2 ? ra[2] : r1 ? ra[1] : ra[0], cp = c3 ? ca[3] : c2 ? ca[2] : c1 ? ca[1] : ca[0];
    const uint32_t rq = rp + v * ((uint32_t)(kW12 >> (16u * col)) & 0xFFFFu);
    const uint32_t cq = cp + v * ((uint32_t)(kW12 >> (16u * row)) & 0xFFFFu);
    // the spawn row / column entries after the spawn (the last LDS round trip of the step: two reads)
    // and before it (selected among f0..g3, which have landed by now)
    const uint32_t fq = lds_half(tab, rq), gq = lds_half(tab, cq);
    const uint32_t fp = r3 ? f3 : r2 ? f2 : r1 ? f1 : f0, gp = c3 ? g3 : c2 ? g2 : c1 ? g1 : g0;
    *tr.a = (uint8_t)a;
    *tr.p = (int32_t)pts;
    // line sums of the pre-spawn board; the next board's swap the spawn's row and column entries
    const uint32_t SRp = f0 + f1 + f2 + f3, SCp = g0 + g1 + g2 + g3;
    const uint32_t SR = SRp - fp + fq, SC = SCp - gp + gq;
    // #lines that can move per direction in nibbles {UP, DOWN, LEFT, RIGHT} -> legal bits 0..3: a
    // nibble n in 0..4 gets bit 3 set by n + 7; the 24-bit product gathers bits 3, 7, 11, 15 at 12..15
    const uint32_t nl = __builtin_amdgcn_perm(SR, SC, 0x0C0C0501u);
    s.legal = (__umul24((nl + 0x7777u) & 0x8888u, 0x249u) >> 12) & 15u;
    // statistics before the spawn (the record's mono_a) and after it (carried to the next step): the
    // spawned tile changes the maximum / its first cell only when it reaches the maximum
    uint32_t sa = stats_bytes(SRp, SCp) | pos_a;
    const uint32_t pos2 = v > Ma ? sp : v == Ma ? min(pos_a, sp) : pos_a;
    uint32_t S = stats_bytes(SR, SC) | pos2 | (max(Ma, v) << 24);
    if (!kSmall && Ma > 11u) {  // an exponent outside kLine12: the SWAR statistics and legal mask
        const MonoStats ms = mono_stats(pre);
        sa = pack_stats(ms);
        S = pack_stats(mono_add_tile(ms, pre, sp, v));
        s.legal = legal_mask(moved);
    }
    const uint32_t mono_a = mono_value_packed(sa);
    // game over: a new game from the pair's spare words (kFresh, prepared with the draw); selects,
    // so the whole pair stays one basic block
    const bool over = s.legal == 0u;
    const uint32_t fl = over ? FLAG_DONE | FLAG_RESET | s.flegal : s.legal;
    s.b = sel4(over, s.fb, s.b);
    s.legal = over ? s.flegal : s.legal;
    s.S = over ? s.fS : S;
    *tr.pot = mono_b | (mono_a << 8) | ((uint32_t)s.empt_b << 16) | (empt_a << 24);
    *tr.f = (uint8_t)fl;
    s.empt_b = over ? 14 : (int)empt_a - 1;
    if constexpr (kOdd) {
        s.D = make_uint4(s.ph.c0, s.ph.c1, s.ph.c2, s.ph.c3);
        s.ph = philox_start(seed, next_pair, env, 1u);
        fresh_prep(s, tab);
    }
}

// Synthetic random-legal rollout (the benchmark workload of BASELINE.md): `steps` env steps per
// board per launch, board in registers, auto-reset on done, one time-major trajectory record per
// step: the board the action was taken on [T][N][16], action, points, potentials, flags.
// Step c (absolute Philox counter) takes word c & 1 of the stream-1 draw at counter c >> 1, so one
// Philox draw serves two steps (and the reset that may end one of them).  The legal mask is
// carried from the previous step (the action is always legal); the move goes through the LDS row
// table while every exponent is <= 11 (the SWAR compute path otherwise); points come from the
// table.  Workgroups are persistent over boards, so large N keeps several waves per SIMD with one
// LDS table per CU.
__global__ __launch_bounds__(1024) void env_rollout_kernel(uint4 *__restrict__ boards, int64_t n, int64_t steps,
                                                           uint4 *__restrict__ tb, uint8_t *__restrict__ ta,
                                                           int32_t *__restrict__ tp, uint32_t *__restrict__ tpot,
                                                           uint8_t *__restrict__ tf, RngArgs rng,
                                                           uint32_t *__restrict__ ticket = nullptr) {
    // kRow12 then kLine12; every 4-bit-masked index of either table stays inside (kRolloutLdsWords)
    __shared__ __attribute__((aligned(16))) uint32_t s_row[kRolloutLdsWords];
    stage_row_table(s_row);
    const uint64_t ctr0 = rng_counter(rng);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        RolloutLane s;
        s.b = boards[i];
        const uint32_t env = rng.env_base + (uint32_t)i;
        const uint32_t li = (uint32_t)i;
        s.legal = legal_mask(s.b);
        if (s.legal == 0u) {  // a finished board handed in: start a new game first (counter ctr0 + steps)
            uint32_t p1, v1, p2, v2;
            s.b = fresh_from_words(philox_draw(rng.seed, ctr0 + (uint64_t)steps, env, 2u), p1, v1, p2, v2);
            MonoStats ms;
            s.legal = fresh_stats(p1, v1, p2, v2, ms);
            s.S = pack_stats(ms);
        } else {
            s.S = pack_stats(mono_stats(s.b));
        }
        s.empt_b = emptiness(s.b);
        uint64_t pair = ctr0 >> 1;
        s.D = philox_draw(rng.seed, pair, env, 1u);
        s.ph = philox_start(rng.seed, pair + 1u, env, 1u);
        fresh_prep(s, s_row);
        // per-lane record addresses, advanced one row (n elements) per step: no array base in an SGPR
        // pair across the loop (the loop's SGPR spills)
        TrajRows tr{tb + li, ta + li, tp + li, tpot + li, tf + li};
        int64_t t = 0;
        if ((ctr0 & 1u) && steps > 0) {  // the launch starts on the second step of a pair
            philox_rounds<0, 5>(s.ph);
            rollout_step<true>(s, s_row, tr, rng.seed, pair + 2u, env);
            tr.next(n);
            pair++;
            t = 1;
        }
        for (; t + 2 <= steps; t += 2, pair++) {
            // every board of the wave <= 2^9 at the pair's start: both steps stay inside the tables
            // (the move adds at most 1 to the maximum), so the pair runs without the fallback branches
            if (__all(s.S < (10u << 24))) {
                rollout_step<false, true>(s, s_row, tr, rng.seed, pair + 2u, env);
                tr.next(n);
                rollout_step<true, true>(s, s_row, tr, rng.seed, pair + 2u, env);
            } else {
                rollout_step<false>(s, s_row, tr, rng.seed, pair + 2u, env);
                tr.next(n);
                rollout_step<true>(s, s_row, tr, rng.seed, pair + 2u, env);
            }
            tr.next(n);
        }
        if (t < steps) rollout_step<false>(s, s_row, tr, rng.seed, pair + 2u, env);
        boards[i] = s.b;
    }
    if (ticket) {
        // g2048_env_rollout_random_adv: the device counter advances by `steps` once every block has
        // read it (each block read it before its boards, i.e. before it arrives here): the last block
        // to arrive adds and puts the ticket back to zero -- no counter-bump kernel between launches.
        // Relaxed: every block's counter read was consumed long before its arrival, the next launch
        // sees the add across the kernel boundary, and an agent-scope release here would write back
        // L2 -- with this launch's records in it (measured +6 us per launch with acq_rel)
        __syncthreads();
        if (threadIdx.x == 0 &&
            __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u) {
            __hip_atomic_fetch_add(const_cast<uint64_t *>(rng.counter_dev), (uint64_t)steps, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace

extern "C" {

static int rollout_launch(g2048_stream_t stream, int8_t *boards, int64_t n, int64_t steps, int8_t *traj_boards,
                          uint8_t *traj_actions, int32_t *traj_points, int8_t *traj_pot, uint8_t *traj_flags,
                          const g2048_rng *rng, uint32_t *ticket);

int g2048_env_rollout_random(g2048_stream_t stream, int8_t *boards, int64_t n, int64_t steps, int8_t *traj_boards,
                             uint8_t *traj_actions, int32_t *traj_points, int8_t *traj_pot, uint8_t *traj_flags,
                             const g2048_rng *rng) {
    return rollout_launch(stream, boards, n, steps, traj_boards, traj_actions, traj_points, traj_pot, traj_flags, rng,
                          nullptr);
}

int g2048_env_rollout_random_adv(g2048_stream_t stream, int8_t *boards, int64_t n, int64_t steps, int8_t *traj_boards,
                                 uint8_t *traj_actions, int32_t *traj_points, int8_t *traj_pot, uint8_t *traj_flags,
                                 const g2048_rng *rng, uint32_t *ticket) {
    if (!rng || !rng->counter_dev || !ticket || ((uintptr_t)rng->counter_dev & 7u) || ((uintptr_t)ticket & 3u))
        return G2048_EINVAL;
    return rollout_launch(stream, boards, n, steps, traj_boards, traj_actions, traj_points, traj_pot, traj_flags, rng,
                          ticket);
}

static int rollout_launch(g2048_stream_t stream, int8_t *boards, int64_t n, int64_t steps, int8_t *traj_boards,
                          uint8_t *traj_actions, int32_t *traj_points, int8_t *traj_pot, uint8_t *traj_flags,
                          const g2048_rng *rng, uint32_t *ticket) {
    // n < 2^28: a lane's byte offset into a trajectory row (16 * board id) fits the 32-bit saddr offset
    if (n < 0 || n >= (int64_t(1) << 28) || steps < 0 || !rng || rng->mode != G2048_RNG_PHILOX) return G2048_EINVAL;
    if (n == 0 || steps == 0) return G2048_OK;
    if (!boards || !traj_boards || !traj_actions || !traj_points || !traj_pot || !traj_flags || !aligned16(boards) ||
        !aligned16(traj_boards) || ((uintptr_t)traj_pot & 3u) || ((uintptr_t)traj_points & 3u))
        return G2048_EINVAL;
    // one workgroup per CU holds the 129 KiB LDS tables; its size scales with N up to 1024 threads
    // so that large N runs 4 waves per SIMD while N = 65 536 still spreads over all 256 CUs
    int64_t threads = (n + 255) / 256;
    threads = threads < 64 ? 64 : threads > 1024 ? 1024 : ((threads + 63) / 64) * 64;
    int64_t grid = (n + threads - 1) / threads;
    grid = grid > 256 ? 256 : grid;
    hipLaunchKernelGGL(env_rollout_kernel, dim3((unsigned)grid), dim3((unsigned)threads), 0, (hipStream_t)stream,
                       (uint4 *)boards, n, steps, (uint4 *)traj_boards, traj_actions, traj_points, (uint32_t *)traj_pot,
                       traj_flags, rng_args(rng), ticket);
    return launch_status();
}

}  // extern "C"
