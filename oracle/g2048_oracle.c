/*
 * g2048_oracle.c -- CPU restatement of the reference's 2048 hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the CHECKER for the HIP kernels in 2048-ppo_amd/csrc.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it (via oracle/oracle.py).
 * It is never linked into, or called by, the product path.
 *
 * It restates, in the reference's own algorithmic form (not the closed forms the kernels use):
 *   slide/merge          game.py:225-257   (_merge_and_shift_{left,right}_with_score)
 *   simulate_move        game.py:122-160   (transpose for UP/DOWN)
 *   legality             game.py:260-330   (can_move_in_direction / can_merge_in_direction scans)
 *   monotonicity         game.py:683-800   (4 clockwise rotations + first-argmax corner rule)
 *   emptiness            game.py:671-680
 *   info heuristics      game.py:339-506, 593-668, 803-921 (smoothness, corner, adjacency, chain
 *                        DFS, anchor corner, snake-order topological score) -- info-only in the
 *                        reference, computed here so a CPU step costs what game.step costs
 *   _add_tile / reset    game.py:923-950   (row-major empties, random.choice, random.random()<0.9)
 *   step                 game.py:952-1030  (invalid move path, heuristics before/after, spawn)
 *   CPython random       Modules/_randommodule.c semantics: MT19937, init_by_array seeding for
 *                        random.seed(int), getrandbits(k) = u32 >> (32-k), _randbelow rejection,
 *                        random() = (a>>5, b>>6) 53-bit
 *   Philox4x32-10        Salmon et al. SC'11 (Random123) -- the kernels' fast-mode generator
 *   obs encoding         game.py:92-101    ([e, row/3, col/3] float32 per cell)
 *
 * Parity pin: tests/test_oracle.py checks every function here against the tests/golden fixtures, which
 * tools/gen_golden.py produced by running the reference itself in the build container.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off so the double-precision heuristics round
 * exactly like CPython floats).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_UP 0
#define OR_DOWN 1
#define OR_LEFT 2
#define OR_RIGHT 3

/* ------------------------------------------------------------------------------------------ */
/* CPython-compatible MT19937                                                                  */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    uint32_t mt[624];
    int32_t idx;
} or_mt;

static void mt_init_genrand(or_mt *s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->idx = 624;
}

static void mt_init_by_array(or_mt *s, const uint32_t *key, int klen) {
    mt_init_genrand(s, 19650218u);
    int i = 1, j = 0;
    int k = 624 > klen ? 624 : klen;
    for (; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= 624) { s->mt[0] = s->mt[623]; i = 1; }
        if (j >= klen) j = 0;
    }
    for (k = 623; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= 624) { s->mt[0] = s->mt[623]; i = 1; }
    }
    s->mt[0] = 0x80000000u;
    s->idx = 624;
}

/* random.seed(n) for a non-negative integer n < 2**64 */
void or_mt_seed(or_mt *s, uint64_t seed) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    mt_init_by_array(s, key, key[1] ? 2 : 1);
}

uint32_t or_mt_u32(or_mt *s) {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    uint32_t y;
    if (s->idx >= 624) {
        int kk;
        for (kk = 0; kk < 624 - 397; kk++) {
            y = (s->mt[kk] & 0x80000000u) | (s->mt[kk + 1] & 0x7fffffffu);
            s->mt[kk] = s->mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < 623; kk++) {
            y = (s->mt[kk] & 0x80000000u) | (s->mt[kk + 1] & 0x7fffffffu);
            s->mt[kk] = s->mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (s->mt[623] & 0x80000000u) | (s->mt[0] & 0x7fffffffu);
        s->mt[623] = s->mt[396] ^ (y >> 1) ^ mag01[y & 1u];
        s->idx = 0;
    }
    y = s->mt[s->idx++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* random.Random._randbelow_with_getrandbits(n), 1 <= n <= 2**31 */
uint32_t or_mt_randbelow(or_mt *s, uint32_t n) {
    int k = 0;
    while ((n >> k) != 0) k++; /* n.bit_length() */
    for (;;) {
        uint32_t r = or_mt_u32(s) >> (32 - k);
        if (r < n) return r;
    }
}

/* random.random() */
double or_mt_random(or_mt *s) {
    uint32_t a = or_mt_u32(s) >> 5, b = or_mt_u32(s) >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

/* ------------------------------------------------------------------------------------------ */
/* Philox4x32-10                                                                               */
/* ------------------------------------------------------------------------------------------ */
void or_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* The build's fast-mode draw: key = seed, counter = {step lo, step hi, env id, stream}. */
void or_philox_draw(uint64_t seed, uint64_t step, uint32_t env, uint32_t stream, uint32_t out[4]) {
    uint32_t ctr[4] = {(uint32_t)step, (uint32_t)(step >> 32), env, stream};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    or_philox4x32_10(ctr, key, out);
}

/* ------------------------------------------------------------------------------------------ */
/* Board transition                                                                             */
/* ------------------------------------------------------------------------------------------ */
/* game.py:225-244 */
void or_slide_left(const int8_t in[4], int8_t out[4], int64_t *points, int32_t *max_created) {
    int8_t nz[4];
    int n = 0;
    for (int j = 0; j < 4; j++)
        if (in[j] != 0) nz[n++] = in[j];
    int m = 0, i = 0;
    int64_t score = 0;
    int32_t mx = 0;
    while (i < n) {
        if (i + 1 < n && nz[i] == nz[i + 1]) {
            int e = nz[i] + 1;
            out[m++] = (int8_t)e;
            score += (int64_t)1 << e;
            if (e > mx) mx = e;
            i += 2;
        } else {
            out[m++] = nz[i];
            i += 1;
        }
    }
    while (m < 4) out[m++] = 0;
    *points = score;
    *max_created = mx;
}

/* game.py:253-257 */
void or_slide_right(const int8_t in[4], int8_t out[4], int64_t *points, int32_t *max_created) {
    int8_t rev[4] = {in[3], in[2], in[1], in[0]}, tmp[4];
    or_slide_left(rev, tmp, points, max_created);
    out[0] = tmp[3]; out[1] = tmp[2]; out[2] = tmp[1]; out[3] = tmp[0];
}

/* game.py:122-160: grid row-major b[4*i+j] */
void or_simulate_move(const int8_t b[16], int dir, int8_t out[16], int64_t *points, int32_t *max_created) {
    int64_t total = 0;
    int32_t mx = 0;
    for (int k = 0; k < 4; k++) {
        int8_t line[4], res[4];
        int64_t p;
        int32_t m;
        for (int j = 0; j < 4; j++) line[j] = (dir == OR_UP || dir == OR_DOWN) ? b[4 * j + k] : b[4 * k + j];
        if (dir == OR_UP || dir == OR_LEFT) or_slide_left(line, res, &p, &m);
        else or_slide_right(line, res, &p, &m);
        for (int j = 0; j < 4; j++) {
            if (dir == OR_UP || dir == OR_DOWN) out[4 * j + k] = res[j];
            else out[4 * k + j] = res[j];
        }
        total += p;
        if (m > mx) mx = m;
    }
    *points = total;
    *max_created = mx;
}

/* Transposed/reversed working view exactly as can_move_in_direction builds it (game.py:263-280). */
static void scan_view(const int8_t b[16], int dir, int8_t v[16]) {
    int transposed = (dir == OR_UP || dir == OR_DOWN);
    int reverse = (dir == OR_UP || dir == OR_LEFT); /* UP is turned into LEFT, LEFT is reversed */
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            int8_t x = transposed ? b[4 * j + i] : b[4 * i + j];
            v[4 * i + (reverse ? 3 - j : j)] = x;
        }
}

/* game.py:260-293 */
int or_can_move(const int8_t b[16], int dir) {
    int8_t v[16];
    scan_view(b, dir, v);
    for (int i = 0; i < 4; i++) {
        int found = 0;
        for (int j = 0; j < 4; j++) {
            if (v[4 * i + j] > 0) found = 1;
            if (found && v[4 * i + j] == 0) return 1;
        }
    }
    return 0;
}

/* game.py:302-330 */
int or_can_merge(const int8_t b[16], int dir) {
    int8_t v[16];
    scan_view(b, dir, v);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 3; j++)
            if (v[4 * i + j] == v[4 * i + j + 1] && v[4 * i + j] != 0) return 1;
    return 0;
}

int or_legal_mask(const int8_t b[16]) {
    int m = 0;
    for (int d = 0; d < 4; d++)
        if (or_can_move(b, d) || or_can_merge(b, d)) m |= 1 << d;
    return m;
}

/* game.py:671-680 */
int or_emptiness(const int8_t b[16]) {
    int c = 0;
    for (int i = 0; i < 16; i++) c += b[i] == 0;
    return c;
}

/* game.py:683-800 */
int or_monotonicity(const int8_t b[16]) {
    int8_t g[16], r[16];
    memcpy(g, b, 16);
    int best = -1;
    for (int rot = 0; rot < 4; rot++) {
        int cur = 0;
        for (int row = 0; row < 4; row++)
            for (int col = 0; col < 3; col++) {
                int l = g[4 * row + col], rr = g[4 * row + col + 1];
                if (l > 0 && rr > 0 && l >= rr) cur++;
            }
        for (int col = 0; col < 4; col++)
            for (int row = 0; row < 3; row++) {
                int t = g[4 * row + col], bt = g[4 * (row + 1) + col];
                if (t > 0 && bt > 0 && t >= bt) cur++;
            }
        if (cur > best) best = cur;
        /* rotate clockwise: new[i][j] = old[3-j][i] */
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) r[4 * i + j] = g[4 * (3 - j) + i];
        memcpy(g, r, 16);
    }
    int mv = b[0];
    for (int i = 1; i < 16; i++)
        if (b[i] > mv) mv = b[i];
    int pos = 0;
    for (int i = 0; i < 16; i++)
        if (b[i] == mv) { pos = i; break; }
    if (pos == 0 || pos == 3 || pos == 12 || pos == 15) best *= 2;
    else best = best >= 0 ? best / 2 : -((-best + 1) / 2); /* python floor division */
    return best;
}

/* ---- info-only heuristics (computed on every step by game.py:981-1002) ------------------- */
static int gmax(const int8_t b[16]) {
    int mv = 0;
    for (int i = 0; i < 16; i++)
        if (b[i] > mv) mv = b[i];
    return mv;
}

/* game.py:339-357 */
double or_smoothness(const int8_t b[16]) {
    double s = 0.0;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            int x = b[4 * i + j];
            if (x == 0) continue;
            if (j < 3 && b[4 * i + j + 1] != 0) s -= abs(x - b[4 * i + j + 1]);
            if (i < 3 && b[4 * (i + 1) + j] != 0) s -= abs(x - b[4 * (i + 1) + j]);
        }
    return s;
}

/* game.py:359-399 */
double or_corner_bonus(const int8_t b[16]) {
    int mv = gmax(b);
    if (mv == 0) return 0.0;
    if (b[0] == mv || b[3] == mv || b[12] == mv || b[15] == mv) return (double)mv;
    return -(double)mv;
}

/* game.py:401-442 */
double or_adjacency_bonus(const int8_t b[16]) {
    int mv = 0, mi = 0, mj = 0;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            if (b[4 * i + j] > mv) { mv = b[4 * i + j]; mi = i; mj = j; }
    double bonus = 0.0;
    static const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
    for (int d = 0; d < 4; d++) {
        int ni = mi + di[d], nj = mj + dj[d];
        if (ni >= 0 && ni < 4 && nj >= 0 && nj < 4) {
            int nv = b[4 * ni + nj];
            if (nv > 0) bonus += nv * 0.5;
        }
    }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            int x = b[4 * i + j];
            if (x >= 5) {
                if (j < 3 && b[4 * i + j + 1] >= 5) bonus += (x + b[4 * i + j + 1]) * 0.25;
                if (i < 3 && b[4 * (i + 1) + j] >= 5) bonus += (x + b[4 * (i + 1) + j]) * 0.25;
            }
        }
    return bonus;
}

/* game.py:476-498 (DFS with a visited set) */
static double chain_dfs(const int8_t b[16], int i, int j, int expected, uint32_t *visited) {
    if (!(i >= 0 && i < 4 && j >= 0 && j < 4)) return 0.0;
    int p = 4 * i + j;
    if (*visited >> p & 1u) return 0.0;
    if (b[p] != expected) return 0.0;
    *visited |= 1u << p;
    double score = (double)expected, best = 0.0;
    static const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
    for (int d = 0; d < 4; d++) {
        double c = chain_dfs(b, i + di[d], j + dj[d], expected - 1, visited);
        if (c > best) best = c;
    }
    *visited &= ~(1u << p);
    return score + best;
}

/* game.py:444-506 */
double or_chain_score(const int8_t b[16]) {
    int mv = gmax(b);
    if (mv == 0) return 0.0;
    double best = 0.0;
    for (int p = 0; p < 16; p++)
        if (b[p] == mv) {
            uint32_t vis = 0;
            double c = chain_dfs(b, p / 4, p % 4, mv, &vis);
            if (c > best) best = c;
        }
    return best;
}

/* game.py:634-668 -> corner index packed as 4*row+col */
int or_anchor_corner(const int8_t b[16]) {
    static const int corners[4] = {0, 3, 12, 15};
    int mv = 0, first = -1;
    uint32_t maxpos = 0;
    for (int p = 0; p < 16; p++) {
        if (b[p] > mv) { mv = b[p]; maxpos = 1u << p; first = p; }
        else if (b[p] == mv && mv > 0) maxpos |= 1u << p;
    }
    if (first < 0) return 0;
    for (int p = 0; p < 16; p++)
        if (maxpos >> p & 1u)
            for (int c = 0; c < 4; c++)
                if (corners[c] == p) return p;
    int ti = first / 4, tj = first % 4, best = corners[0], bd = 1 << 30;
    for (int c = 0; c < 4; c++) {
        int d = abs(corners[c] / 4 - ti) + abs(corners[c] % 4 - tj);
        if (d < bd) { bd = d; best = corners[c]; }
    }
    return best;
}

/* game.py:610-632 */
static void snake_order(int corner, int order[16]) {
    int cr = corner / 4, cc = corner % 4, n = 0;
    int rd = cr == 0 ? 1 : -1, cd = cc == 0 ? 1 : -1;
    for (int i = 0; i < 4; i++) {
        int row = cr + i * rd;
        for (int s = 0; s < 4; s++) {
            int col = (i % 2 == 0) ? cc + s * cd : cc + (3 - s) * cd;
            order[n++] = 4 * row + col;
        }
    }
}

/* game.py:802-921 with a single anchor corner (as step() calls it) */
double or_topological(const int8_t b[16], int corner) {
    int mv = gmax(b);
    if (mv == 0) return 0.0;
    int order[16], idx_of[16];
    snake_order(corner, order);
    for (int k = 0; k < 16; k++) idx_of[order[k]] = k;
    double score = 0.0;
    for (int p = 0; p < 16; p++)
        if (b[p] > 0) score += (double)((16 - idx_of[p]) * b[p]) * 0.1;
    double prev = INFINITY, mono = 0.0, inv = 0.0;
    for (int k = 0; k < 16; k++) {
        int v = b[order[k]];
        if (v == 0) continue;
        if ((double)v <= prev) mono += v * 0.2;
        else inv += ((double)v - prev) * 0.5;
        prev = (double)v;
    }
    score += mono - inv;
    if (b[corner] == mv) score += mv * 2.0;
    static const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
    for (int p = 0; p < 16; p++) {
        int v = b[p];
        if (v <= 0 || v < 4) continue;
        int lower = 0, tot = 0, i = p / 4, j = p % 4;
        for (int d = 0; d < 4; d++) {
            int ni = i + di[d], nj = j + dj[d];
            if (ni >= 0 && ni < 4 && nj >= 0 && nj < 4) {
                int nv = b[4 * ni + nj];
                if (nv > 0) { tot++; if (nv < v - 2) lower++; }
            }
        }
        if (tot >= 2 && lower >= tot - 1 && idx_of[p] > 4) score -= v * 1.0;
    }
    return score;
}

/* ------------------------------------------------------------------------------------------ */
/* Spawn / reset / step                                                                         */
/* ------------------------------------------------------------------------------------------ */
#define OR_RNG_MT 1
#define OR_RNG_PHILOX 0
#define OR_RNG_INJECT 2

typedef struct {
    int32_t mode;
    uint32_t env;
    uint64_t seed;     /* Philox key */
    uint64_t step;     /* Philox counter (advanced by the caller) */
    or_mt *mt;         /* MT19937 state for mode 1 */
    int32_t inj_k;     /* mode 2: k-th empty cell */
    int32_t inj_v;     /* mode 2: exponent (1 or 2) */
} or_rng;

/* game.py:923-940; with Philox the (k, value) words u0/u1 are the build's fast-mode convention */
static int add_tile(int8_t b[16], or_rng *r, uint32_t u0, uint32_t u1) {
    int empt[16], n = 0;
    for (int p = 0; p < 16; p++)
        if (b[p] == 0) empt[n++] = p;
    if (n == 0) return 0;
    int k, v;
    if (r->mode == OR_RNG_MT) {
        k = (int)or_mt_randbelow(r->mt, (uint32_t)n);
        v = or_mt_random(r->mt) < 0.9 ? 1 : 2;
    } else if (r->mode == OR_RNG_PHILOX) {
        k = (int)(((uint64_t)u0 * (uint32_t)n) >> 32);
        v = u1 < 3865470567u ? 1 : 2; /* u32 * 2^-32 < 0.9 */
    } else {
        k = r->inj_k;
        v = r->inj_v;
    }
    b[empt[k]] = (int8_t)v;
    return 1;
}

/* game.py:942-950 */
void or_reset(int8_t b[16], or_rng *r) {
    memset(b, 0, 16);
    uint32_t ph[4] = {0, 0, 0, 0};
    if (r->mode == OR_RNG_PHILOX) or_philox_draw(r->seed, r->step, r->env, 2u, ph);
    add_tile(b, r, ph[0], ph[1]);
    add_tile(b, r, ph[2], ph[3]);
}

/* The rollout kernel's auto-reset (build convention, no reference counterpart): the two spawns of
   reset() from two words a, b.  Cell 1 = a >> 28 (16 empties), its value from the remaining 28 bits
   (a << 4 < 0.9 * 2^32); cell 2 = floor(b * 15 / 2^32), its value from the low word of b * 15. */
void or_reset_words(int8_t b[16], uint32_t a, uint32_t bw) {
    or_rng r = {OR_RNG_PHILOX, 0, 0, 0, NULL, 0, 0};
    memset(b, 0, 16);
    add_tile(b, &r, a, a << 4);
    add_tile(b, &r, bw, bw * 15u);
}

typedef struct {
    int64_t points;
    int32_t max_tile;
    int32_t invalid;
    int32_t done;
    int32_t mono_b, mono_a, empt_b, empt_a;
    int32_t maxexp_b, maxexp_a;
    double smooth_d, corner_d, adj_d, chain_d, topo_d;
    int8_t moved[16];
} or_step_out;

/* game.py:952-1030.  `full_info` = 1 computes the info-only heuristics like the reference does.
   Philox spawn words: stream 0 of (seed, step, env) unless `spawn_words` supplies them. */
static void step_impl(int8_t b[16], int dir, or_rng *r, int full_info, or_step_out *o, const uint32_t *spawn_words,
                      int chain);

void or_step(int8_t b[16], int dir, or_rng *r, int full_info, or_step_out *o) {
    step_impl(b, dir, r, full_info, o, NULL, 0);
}

/* The synthetic-policy step: ONE Philox draw of stream 1 gives the action (x: k-th legal action,
   UP/DOWN/LEFT/RIGHT order) and the spawn (y: cell, z: value).  Returns the action. */
int or_step_random(int8_t b[16], or_rng *r, int full_info, or_step_out *o) {
    uint32_t d[4];
    or_philox_draw(r->seed, r->step, r->env, 1u, d);
    int m = or_legal_mask(b), nl = __builtin_popcount(m), dir = 0;
    int k = (int)(((uint64_t)d[0] * (uint32_t)nl) >> 32);
    for (int q = 0; q < 4; q++)
        if (m >> q & 1) { if (k == 0) { dir = q; break; } k--; }
    uint32_t w[2] = {d[1], d[2]};
    step_impl(b, dir, r, full_info, o, w, 0);
    return dir;
}

/* The rollout kernel's synthetic-policy step: ONE 32-bit word u.  Action k = floor(u * nlegal / 2^32)
   (k-th legal action); the low word r of that product picks the spawn: cell floor(r * nempty / 2^32),
   value 1 if the low word of r * nempty is below 0.9 * 2^32.  Returns the action. */
int or_step_word(int8_t b[16], uint32_t u, int full_info, or_step_out *o) {
    int m = or_legal_mask(b), nl = __builtin_popcount(m), dir = 0;
    uint64_t pa = (uint64_t)u * (uint32_t)nl;
    int k = (int)(pa >> 32);
    for (int q = 0; q < 4; q++)
        if (m >> q & 1) { if (k == 0) { dir = q; break; } k--; }
    uint32_t w[2] = {(uint32_t)pa, 0u};
    or_rng r = {OR_RNG_PHILOX, 0, 0, 0, NULL, 0, 0};
    step_impl(b, dir, &r, full_info, o, w, 1);
    return dir;
}

static void step_impl(int8_t b[16], int dir, or_rng *r, int full_info, or_step_out *o, const uint32_t *spawn_words,
                      int chain) {
    memset(o, 0, sizeof(*o));
    if (!(or_can_move(b, dir) || or_can_merge(b, dir))) {
        o->invalid = 1;
        o->done = or_legal_mask(b) == 0;
        memcpy(o->moved, b, 16);
        return;
    }
    double sb = 0, cb = 0, ab = 0, chb = 0, tb = 0;
    int anchor = 0;
    if (full_info) {
        sb = or_smoothness(b); cb = or_corner_bonus(b); ab = or_adjacency_bonus(b); chb = or_chain_score(b);
    }
    o->mono_b = or_monotonicity(b);
    if (full_info) { anchor = or_anchor_corner(b); tb = or_topological(b, anchor); }
    o->empt_b = or_emptiness(b);
    o->maxexp_b = gmax(b);
    int8_t nb[16];
    or_simulate_move(b, dir, nb, &o->points, &o->max_tile);
    memcpy(b, nb, 16);
    memcpy(o->moved, nb, 16);
    if (full_info) {
        o->smooth_d = or_smoothness(b) - sb;
        o->corner_d = or_corner_bonus(b) - cb;
        o->adj_d = or_adjacency_bonus(b) - ab;
        o->chain_d = or_chain_score(b) - chb;
    }
    o->mono_a = or_monotonicity(b);
    o->empt_a = or_emptiness(b);
    if (full_info) o->topo_d = or_topological(b, anchor) - tb;
    o->maxexp_a = gmax(b);
    uint32_t ph[4] = {0, 0, 0, 0};
    if (r->mode == OR_RNG_PHILOX) {
        if (spawn_words) {
            ph[0] = spawn_words[0];
            ph[1] = chain ? (uint32_t)((uint64_t)ph[0] * (uint32_t)or_emptiness(b)) : spawn_words[1];
        }
        else or_philox_draw(r->seed, r->step, r->env, 0u, ph);
    }
    add_tile(b, r, ph[0], ph[1]);
    o->done = or_legal_mask(b) == 0;
}

/* game.py:92-101 */
void or_obs_encode(const int8_t b[16], float out[48]) {
    for (int c = 0; c < 16; c++) {
        out[3 * c + 0] = (float)b[c];
        out[3 * c + 1] = (float)(c / 4) / 3.0f;
        out[3 * c + 2] = (float)(c % 4) / 3.0f;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Batched entry points (numpy arrays through ctypes)                                           */
/* ------------------------------------------------------------------------------------------ */
size_t or_mt_state_bytes(void) { return sizeof(or_mt); }

void or_mt_seed_batch(or_mt *states, const uint64_t *seeds, int64_t n) {
    for (int64_t i = 0; i < n; i++) or_mt_seed(&states[i], seeds[i]);
}

void or_mt_u32_batch(or_mt *state, uint32_t *out, int64_t n) {
    for (int64_t i = 0; i < n; i++) out[i] = or_mt_u32(state);
}

void or_move_batch(const int8_t *boards, const int64_t *dirs, int8_t *out, int64_t *points,
                   int32_t *max_tile, int64_t n) {
    for (int64_t i = 0; i < n; i++) or_simulate_move(boards + 16 * i, (int)dirs[i], out + 16 * i, points + i, max_tile + i);
}

void or_legal_batch(const int8_t *boards, uint8_t *mask, int64_t n) {
    for (int64_t i = 0; i < n; i++) mask[i] = (uint8_t)or_legal_mask(boards + 16 * i);
}

void or_potentials_batch(const int8_t *boards, int32_t *mono, int32_t *empt, int64_t n) {
    for (int64_t i = 0; i < n; i++) {
        mono[i] = or_monotonicity(boards + 16 * i);
        empt[i] = or_emptiness(boards + 16 * i);
    }
}

void or_info_batch(const int8_t *boards, double *out /* [n,5]: smooth, corner, adj, chain, topo(anchor) */,
                   int32_t *anchor, int64_t n) {
    for (int64_t i = 0; i < n; i++) {
        const int8_t *b = boards + 16 * i;
        anchor[i] = or_anchor_corner(b);
        out[5 * i + 0] = or_smoothness(b);
        out[5 * i + 1] = or_corner_bonus(b);
        out[5 * i + 2] = or_adjacency_bonus(b);
        out[5 * i + 3] = or_chain_score(b);
        out[5 * i + 4] = or_topological(b, anchor[i]);
    }
}

void or_obs_batch(const int8_t *boards, float *obs, int64_t n) {
    for (int64_t i = 0; i < n; i++) or_obs_encode(boards + 16 * i, obs + 48 * i);
}

/*
 * Step n independent envs once.  rng_mode: 0 Philox(seed, step, env id = env_base + i),
 * 1 MT19937 (mt_states[i]), 2 injected (inj_k[i], inj_v[i]).  out_i32 is [n, 10]:
 * points, max_tile, invalid, done, mono_b, mono_a, empt_b, empt_a, maxexp_b, maxexp_a.
 * info (may be NULL) is [n,5] deltas.  moved (may be NULL) is the pre-spawn board.
 */
void or_step_batch(int8_t *boards, const int64_t *dirs, int64_t n, int rng_mode, uint64_t seed,
                   uint64_t step, uint32_t env_base, or_mt *mt_states, const int32_t *inj_k,
                   const int32_t *inj_v, int full_info, int64_t *out_i64, double *info, int8_t *moved) {
    for (int64_t i = 0; i < n; i++) {
        or_rng r = {rng_mode, env_base + (uint32_t)i, seed, step, mt_states ? &mt_states[i] : NULL,
                    inj_k ? inj_k[i] : 0, inj_v ? inj_v[i] : 0};
        or_step_out o;
        or_step(boards + 16 * i, (int)dirs[i], &r, full_info, &o);
        int64_t *q = out_i64 + 10 * i;
        q[0] = o.points; q[1] = o.max_tile; q[2] = o.invalid; q[3] = o.done;
        q[4] = o.mono_b; q[5] = o.mono_a; q[6] = o.empt_b; q[7] = o.empt_a;
        q[8] = o.maxexp_b; q[9] = o.maxexp_a;
        if (info) {
            info[5 * i + 0] = o.smooth_d; info[5 * i + 1] = o.corner_d; info[5 * i + 2] = o.adj_d;
            info[5 * i + 3] = o.chain_d; info[5 * i + 4] = o.topo_d;
        }
        if (moved) memcpy(moved + 16 * i, o.moved, 16);
    }
}

void or_reset_batch(int8_t *boards, int64_t n, int rng_mode, uint64_t seed, uint64_t step,
                    uint32_t env_base, or_mt *mt_states) {
    for (int64_t i = 0; i < n; i++) {
        or_rng r = {rng_mode, env_base + (uint32_t)i, seed, step, mt_states ? &mt_states[i] : NULL, 0, 0};
        or_reset(boards + 16 * i, &r);
    }
}

void or_philox_batch(uint64_t seed, uint64_t step, uint32_t env_base, uint32_t stream, uint32_t *out, int64_t n) {
    for (int64_t i = 0; i < n; i++) or_philox_draw(seed, step, env_base + (uint32_t)i, stream, out + 4 * i);
}

/*
 * CPU baseline workload / checker of env_rollout_kernel: `n_envs` independent games stepped
 * `steps` times with the synthetic random-legal policy: step c = step0 + t takes word c & 1 of the
 * stream-1 draw at counter c >> 1 (or_step_word); a game that ends at step c restarts from words 2
 * and 3 of that draw (or_reset_words; a pair of steps holds at most one reset).  A board handed in
 * already finished is first reset with counter step0 + steps, stream 2 (the kernel's convention).  Optional records (time-major [steps][n_envs]):
 * rec_boards [..][16] (board the action was taken on), rec_act, rec_pts, rec_pot [..][4], rec_flags.
 * Returns the number of transitions executed.
 */
int64_t or_random_rollout_rec(int8_t *boards, int64_t n_envs, int64_t steps, uint64_t seed, uint64_t step0,
                              uint32_t env_base, int full_info, int8_t *rec_boards, uint8_t *rec_act,
                              int32_t *rec_pts, int8_t *rec_pot, uint8_t *rec_flags) {
    int64_t count = 0;
    for (int64_t i = 0; i < n_envs; i++) {
        int8_t *b = boards + 16 * i;
        uint32_t env = env_base + (uint32_t)i;
        if (or_legal_mask(b) == 0) {
            or_rng r0 = {OR_RNG_PHILOX, env, seed, step0 + (uint64_t)steps, NULL, 0, 0};
            or_reset(b, &r0);
        }
        for (int64_t t = 0; t < steps; t++) {
            int64_t o = t * n_envs + i;
            if (rec_boards) memcpy(rec_boards + 16 * o, b, 16);
            uint64_t c = step0 + (uint64_t)t;
            uint32_t d[4];
            or_philox_draw(seed, c >> 1, env, 1u, d);
            or_step_out so;
            int dir = or_step_word(b, d[c & 1u], full_info, &so);
            int m = or_legal_mask(b), fl = m;
            if (so.done) {
                or_reset_words(b, d[2], d[3]);
                fl = 0x80 | 0x20 | or_legal_mask(b);
            }
            if (rec_act) rec_act[o] = (uint8_t)dir;
            if (rec_pts) rec_pts[o] = (int32_t)so.points;
            if (rec_pot) {
                rec_pot[4 * o + 0] = (int8_t)so.mono_b; rec_pot[4 * o + 1] = (int8_t)so.mono_a;
                rec_pot[4 * o + 2] = (int8_t)so.empt_b; rec_pot[4 * o + 3] = (int8_t)so.empt_a;
            }
            if (rec_flags) rec_flags[o] = (uint8_t)fl;
            count++;
        }
    }
    return count;
}

int64_t or_random_rollout(int8_t *boards, int64_t n_envs, int64_t steps, uint64_t seed, uint64_t step0,
                          uint32_t env_base, int full_info) {
    return or_random_rollout_rec(boards, n_envs, steps, seed, step0, env_base, full_info, NULL, NULL, NULL, NULL,
                                 NULL);
}

void or_step_random_batch(int8_t *boards, int64_t n, uint64_t seed, uint64_t step, uint32_t env_base,
                          int64_t *out_i64 /* [n,11]: step fields + action */) {
    for (int64_t i = 0; i < n; i++) {
        or_rng r = {OR_RNG_PHILOX, env_base + (uint32_t)i, seed, step, NULL, 0, 0};
        or_step_out o;
        int dir = or_step_random(boards + 16 * i, &r, 0, &o);
        int64_t *q = out_i64 + 11 * i;
        q[0] = o.points; q[1] = o.max_tile; q[2] = o.invalid; q[3] = o.done;
        q[4] = o.mono_b; q[5] = o.mono_a; q[6] = o.empt_b; q[7] = o.empt_a;
        q[8] = o.maxexp_b; q[9] = o.maxexp_a; q[10] = dir;
    }
}
