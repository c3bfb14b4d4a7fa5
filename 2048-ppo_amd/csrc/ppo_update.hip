// ppo_update.hip -- fused kernels of the PPO minibatch step (model_optimize_step, train.py:414-642)
// for GameMLP (game.py:1033-1220): everything of the forward/backward except the GEMMs.
//
//   obs_gather_kernel     boards[idx] -> to_model_format (game.py:92-101), bf16 [m,48]
//   ln_fwd_kernel<J,D>    y = res + Dropout(ReLU(LayerNorm(g)))          (ResidualBlock / stem)
//   ln_bwd_kernel<J,D>    its backward: dg, the residual gradient, dgamma/dbeta partials
//   head_loss_kernel<..>  action/value heads + PPO-clip loss + entropy + smooth-L1 + backward
//   head_kl_kernel<..>    KL(old || new) of the post-step re-forward (train.py:578-601)
//   mlp_fwd_kernel<NT,..> G = X W^T on bf16 MFMA + the LayerNorm/ReLU/dropout/residual epilogue
//   head_fwd_kernel<KS>   rollout policy heads (logits + value) on MFMA
//   wgrad_kernel<BI,BJ>   dW = dG^T X on bf16 MFMA (tall-skinny, K = minibatch rows)
//   colsum1/2             deterministic two-level column sums of per-block partials
//
// One wave per row: lane l owns columns 4(l + 64j), j < J = ceil(h/256), so a row is J
// coalesced 8-B (bf16) or 16-B (fp32) accesses per lane and every row reduction is a wave
// butterfly -- no LDS, no barriers in the row loop.  The kernels are HBM-bound: per row the
// forward moves 6h bytes (g, res in; y out), the backward 12h-14h.  Dropout masks are Philox
// draws regenerated from (row, column group, layer, pass, counter), never stored.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "board.hpp"
#include "ln_row.hpp"
#include "ppo_common.hpp"
#include "../../include/g2048_ppo.h"

using g2048::philox;

namespace {

using namespace g2048::ppo;

constexpr int kWaves = 4;  // waves per block
constexpr int kThreads = 64 * kWaves;
constexpr float kLnEps = 1e-5f;

__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// round-to-nearest-even float -> bf16 pair on the hardware converter (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
    const bf16x2_t v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ uint32_t f2bf(float f) { return pack_bf2(f, 0.0f) & 0xFFFFu; }

__device__ __forceinline__ void load_bf4_lds(const char *p, float v[4]) {
    const uint2 t = *reinterpret_cast<const uint2 *>(p);
    v[0] = __uint_as_float(t.x << 16);
    v[1] = __uint_as_float(t.x & 0xFFFF0000u);
    v[2] = __uint_as_float(t.y << 16);
    v[3] = __uint_as_float(t.y & 0xFFFF0000u);
}

__device__ __forceinline__ void load_bf4(const uint16_t *p, float v[4]) {
    const uint2 q = *reinterpret_cast<const uint2 *>(p);
    v[0] = bf2f(q.x & 0xFFFFu);
    v[1] = bf2f(q.x >> 16);
    v[2] = bf2f(q.y & 0xFFFFu);
    v[3] = bf2f(q.y >> 16);
}

__device__ __forceinline__ void store_bf4(uint16_t *p, const float v[4]) {
    *reinterpret_cast<uint2 *>(p) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
}

__device__ __forceinline__ void store_bf4(uint16_t *p, const __attribute__((ext_vector_type(4))) float &v) {
    const float t[4] = {v[0], v[1], v[2], v[3]};
    store_bf4(p, t);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

__constant__ float kThirds[4] = {0.0f, 1.0f / 3.0f, 2.0f / 3.0f, 1.0f};

// ------------------------------------------------------------------ obs gather ---------------
__global__ __launch_bounds__(256) void obs_gather_kernel(const int8_t *__restrict__ boards,
                                                         const int64_t *__restrict__ idx, uint16_t *__restrict__ obs,
                                                         int64_t m) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // chunk of 4 features
    if (q >= m * 12) return;
    const int64_t r = q / 12;
    const int f0 = (int)(q - r * 12) * 4;
    const int8_t *b = boards + idx[r] * 16;
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int f = f0 + u, cell = f / 3, k = f - cell * 3;
        v[u] = k == 0 ? (float)b[cell] : kThirds[k == 1 ? (cell >> 2) : (cell & 3)];
    }
    store_bf4(obs + q * 4, v);
}

// ------------------------------------------------------------------ LayerNorm forward --------
// RPW rows per wave and iteration: their loads are all in flight before the first reduction.
constexpr int kFwdRows = 4;

template <int J, bool DROP>
__global__ __launch_bounds__(kThreads) void ln_fwd_kernel(const uint16_t *__restrict__ g, const float *__restrict__ gamma,
                                                          const float *__restrict__ beta,
                                                          const uint16_t *__restrict__ res, uint16_t *__restrict__ y,
                                                          float *__restrict__ mean_out, float *__restrict__ rstd_out,
                                                          int64_t m, int h, DropArgs da) {
    constexpr int RPW = kFwdRows;
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * kWaves;
    const Drop d = make_drop(da);
    float gm[J][4], bt[J][4];
    bool ok[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int c = 4 * (lane + 64 * j);
        ok[j] = c < h;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            gm[j][u] = ok[j] ? gamma[c + u] : 0.0f;
            bt[j][u] = ok[j] ? beta[c + u] : 0.0f;
        }
    }
    const float inv_h = 1.0f / (float)h;
    for (int64_t r0 = ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * RPW; r0 < m; r0 += nw * RPW) {
        float x[RPW][J][4], rs[RPW][J][4];
        float s[RPW], v[RPW], mean[RPW], rstd[RPW];
#pragma unroll
        for (int q = 0; q < RPW; q++) {
            const int64_t r = r0 + q;
            s[q] = 0.0f;
#pragma unroll
            for (int j = 0; j < J; j++) {
                const int c = 4 * (lane + 64 * j);
                if (ok[j] && r < m) {
                    load_bf4(g + r * h + c, x[q][j]);
                    if (res) load_bf4(res + r * h + c, rs[q][j]);
                } else {
#pragma unroll
                    for (int u = 0; u < 4; u++) x[q][j][u] = rs[q][j][u] = 0.0f;
                }
                s[q] += (x[q][j][0] + x[q][j][1]) + (x[q][j][2] + x[q][j][3]);
            }
        }
#pragma unroll
        for (int q = 0; q < RPW; q++) mean[q] = wave_sum(s[q]) * inv_h;
#pragma unroll
        for (int q = 0; q < RPW; q++) {
            v[q] = 0.0f;
#pragma unroll
            for (int j = 0; j < J; j++)
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const float t = ok[j] ? x[q][j][u] - mean[q] : 0.0f;
                    v[q] += t * t;
                }
        }
#pragma unroll
        for (int q = 0; q < RPW; q++) rstd[q] = 1.0f / sqrtf(wave_sum(v[q]) * inv_h + kLnEps);
#pragma unroll
        for (int q = 0; q < RPW; q++) {
            const int64_t r = r0 + q;
            if (r >= m) break;
#pragma unroll
            for (int j = 0; j < J; j++) {
                if (!ok[j]) continue;
                const int c = 4 * (lane + 64 * j);
                float o[4], k[4];
                if (DROP) drop_mult(d, (uint32_t)r, (uint32_t)(lane + 64 * j), k);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    float a = fmaxf((x[q][j][u] - mean[q]) * rstd[q] * gm[j][u] + bt[j][u], 0.0f);
                    if (DROP) a *= k[u];
                    o[u] = res ? rs[q][j][u] + a : a;
                }
                store_bf4(y + r * h + c, o);
            }
            if (lane == 0) {
                mean_out[r] = mean[q];
                rstd_out[r] = rstd[q];
            }
        }
    }
}

// ------------------------------------------------------------------ LayerNorm backward -------
// The sources of a block's output gradient: dy = dres + sum_i p[i] + the heads' share, recomputed
// from their output gradient dz [m][8] (4 logits, value, 3 pad) as dz[0:4] wa + dz[4] wv (wv NULL =
// decoupled critic: the value branch is cut).
static_assert(sizeof(g2048_dy) == 64 && offsetof(g2048_dy, dz) == 40, "g2048_dy layout (tests/test_abi.py)");

struct DySrc {
    const float *dres;
    const uint16_t *p[G2048_DY_MAX_P];
    int np;
    const float *dz, *wa, *wv;
};

// Block partials: part[blockIdx][0:h] = sum dz*xhat (dgamma), part[blockIdx][h:2h] = sum dz (dbeta).
// dres_out may alias dres_in (each element is read, then written, by the same lane).
constexpr int kBwdRows = 2;
constexpr int kBwdWaves = 16;  // 1024-thread blocks, <= 256 of them: few partial rows to reduce
constexpr int kBwdThreads = 64 * kBwdWaves;

template <int J, bool DROP, bool HEAD>
__global__ __launch_bounds__(kBwdThreads) void ln_bwd_kernel(
    DySrc src, const uint16_t *__restrict__ g,
    const float *__restrict__ mean_in, const float *__restrict__ rstd_in, const float *__restrict__ gamma,
    const float *__restrict__ beta, uint16_t *__restrict__ dg, float *dres_out, float *__restrict__ part,
    int64_t m, int h, DropArgs da) {
    constexpr int RPW = kBwdRows;
    extern __shared__ float lds[];  // [kBwdWaves][2h]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t nw = (int64_t)gridDim.x * kBwdWaves;
    const Drop d = make_drop(da);
    float gm[J][4], bt[J][4], ag[J][4], ab[J][4], wh[HEAD ? 5 : 1][J][4];
    bool ok[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int c = 4 * (lane + 64 * j);
        ok[j] = c < h;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            gm[j][u] = ok[j] ? gamma[c + u] : 0.0f;
            bt[j][u] = ok[j] ? beta[c + u] : 0.0f;
            ag[j][u] = ab[j][u] = 0.0f;
            if (HEAD) {
#pragma unroll
                for (int k = 0; k < 4; k++) wh[k][j][u] = ok[j] ? src.wa[k * h + c + u] : 0.0f;
                wh[HEAD ? 4 : 0][j][u] = ok[j] && src.wv ? src.wv[c + u] : 0.0f;
            }
        }
    }
    const float inv_h = 1.0f / (float)h;
    for (int64_t r0 = ((int64_t)blockIdx.x * kBwdWaves + wave) * RPW; r0 < m; r0 += nw * RPW) {
        float x[RPW][J][4], dy[RPW][J][4], xh[RPW][J][4], dxh[RPW][J][4];
        float mean[RPW], rstd[RPW], s1[RPW], s2[RPW];
#pragma unroll
        for (int q = 0; q < RPW; q++) {
            const int64_t r = r0 + q;
            const bool rv = r < m;
            mean[q] = rv ? mean_in[r] : 0.0f;
            rstd[q] = rv ? rstd_in[r] : 0.0f;
            float dz[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
            if (HEAD && rv) {  // the heads' output gradient of this row (wave-uniform broadcast loads)
                const float4 d0 = *reinterpret_cast<const float4 *>(src.dz + r * 8);
                dz[0] = d0.x;
                dz[1] = d0.y;
                dz[2] = d0.z;
                dz[3] = d0.w;
                dz[4] = src.dz[r * 8 + 4];
            }
#pragma unroll
            for (int j = 0; j < J; j++) {
                const int c = 4 * (lane + 64 * j);
#pragma unroll
                for (int u = 0; u < 4; u++) x[q][j][u] = dy[q][j][u] = 0.0f;
                if (!(ok[j] && rv)) continue;
                load_bf4(g + r * h + c, x[q][j]);
                if (HEAD) {
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        float t = 0.0f;
#pragma unroll
                        for (int k = 0; k < 5; k++) t += dz[k] * wh[HEAD ? k : 0][j][u];
                        dy[q][j][u] = t;
                    }
                }
                if (src.dres) {
                    const float4 t = *reinterpret_cast<const float4 *>(src.dres + r * h + c);
                    dy[q][j][0] += t.x;
                    dy[q][j][1] += t.y;
                    dy[q][j][2] += t.z;
                    dy[q][j][3] += t.w;
                }
#pragma unroll
                for (int i = 0; i < G2048_DY_MAX_P; i++) {
                    if (i >= src.np) break;
                    float t[4];
                    load_bf4(src.p[i] + r * h + c, t);
#pragma unroll
                    for (int u = 0; u < 4; u++) dy[q][j][u] += t[u];
                }
            }
        }
#pragma unroll
        for (int q = 0; q < RPW; q++) {
            const int64_t r = r0 + q;
            const bool rv = r < m;
            s1[q] = s2[q] = 0.0f;
#pragma unroll
            for (int j = 0; j < J; j++) {
                const bool live = ok[j] && rv;
                const int c = 4 * (lane + 64 * j);
                float k[4];
                if (live && dres_out)
                    *reinterpret_cast<float4 *>(dres_out + r * h + c) =
                        make_float4(dy[q][j][0], dy[q][j][1], dy[q][j][2], dy[q][j][3]);
                if (DROP) drop_mult(d, (uint32_t)r, (uint32_t)(lane + 64 * j), k);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const float xhat = live ? (x[q][j][u] - mean[q]) * rstd[q] : 0.0f;
                    const float z = xhat * gm[j][u] + bt[j][u];
                    float dz = (live && z > 0.0f) ? dy[q][j][u] : 0.0f;
                    if (DROP) dz *= k[u];
                    ag[j][u] += dz * xhat;
                    ab[j][u] += dz;
                    xh[q][j][u] = xhat;
                    dxh[q][j][u] = dz * gm[j][u];
                    s1[q] += dxh[q][j][u];
                    s2[q] += dxh[q][j][u] * xhat;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < RPW; q++) {
            s1[q] = wave_sum(s1[q]) * inv_h;
            s2[q] = wave_sum(s2[q]) * inv_h;
        }
#pragma unroll
        for (int q = 0; q < RPW; q++) {
            const int64_t r = r0 + q;
            if (r >= m) break;
#pragma unroll
            for (int j = 0; j < J; j++) {
                if (!ok[j]) continue;
                float o[4];
#pragma unroll
                for (int u = 0; u < 4; u++) o[u] = rstd[q] * (dxh[q][j][u] - s1[q] - xh[q][j][u] * s2[q]);
                store_bf4(dg + r * h + 4 * (lane + 64 * j), o);
            }
        }
    }
    // block reduction of the dgamma / dbeta accumulators
#pragma unroll
    for (int j = 0; j < J; j++) {
        if (!ok[j]) continue;
        const int c = 4 * (lane + 64 * j);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            lds[wave * 2 * h + c + u] = ag[j][u];
            lds[wave * 2 * h + h + c + u] = ab[j][u];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * h; c += kBwdThreads) {
        float t = 0.0f;
#pragma unroll
        for (int w = 0; w < kBwdWaves; w++) t += lds[w * 2 * h + c];
        part[(int64_t)blockIdx.x * 2 * h + c] = t;
    }
}

// ------------------------------------------------------------------ heads + PPO loss ---------
// B fragments (lane (g, c): k = 32 ks + 8 g + j, column c) of the head matrix [wa (4 rows); wv],
// zero beyond column 4 and row h, split w = hi + mid + lo into three bf16 terms.
template <int KS>
__device__ __forceinline__ void load_head_b3(bf16x8_t fb[3][KS], const float *wa, const float *wv, int h, int g,
                                             int c, int k0 = 0) {
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
        s16x8_t v0, v1, v2;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int k = k0 + 32 * ks + 8 * g + j;
            const float wgt = (c < 5 && k < h) ? (c < 4 ? wa[c * h + k] : wv ? wv[k] : 0.0f) : 0.0f;
            const __bf16 hi = (__bf16)wgt;
            const float r1 = wgt - (float)hi;
            const __bf16 mid = (__bf16)r1;
            const __bf16 lo = (__bf16)(r1 - (float)mid);
            v0[j] = __builtin_bit_cast(short, hi);
            v1[j] = __builtin_bit_cast(short, mid);
            v2[j] = __builtin_bit_cast(short, lo);
        }
        fb[0][ks] = __builtin_bit_cast(bf16x8_t, v0);
        fb[1][ks] = __builtin_bit_cast(bf16x8_t, v1);
        fb[2][ks] = __builtin_bit_cast(bf16x8_t, v2);
    }
}

// z[64 rows][5] = x[r0 .. r0+63] [wa; wv]^T on MFMA, into the wave's LDS tile (without bias).
// KS k-steps of 32 per chunk; with MULTI the weights are re-split per 256-column chunk (h > 256).
// With xs (STAGE), the 64 rows come from the wave's LDS image (row-major, pitch 2h bytes).
template <int KS, bool MULTI, bool STAGE = false>
__device__ __forceinline__ void head_tiles(float (*zt)[5], bf16x8_t fb[3][KS], const uint16_t *xin, const float *wa,
                                           const float *wv, int64_t m, int h, int64_t r0, int g, int c, int nout,
                                           const char *xs = nullptr) {
    f32x4_t z[4];
#pragma unroll
    for (int t = 0; t < 4; t++) z[t] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
    for (int k0 = 0; k0 < h; k0 += 32 * KS) {
        if (MULTI) load_head_b3<KS>(fb, wa, wv, h, g, c, k0);
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int64_t mr = r0 + 16 * t + c;
#pragma unroll
            for (int ks = 0; ks < KS; ks++) {
                const int kl = k0 + 32 * ks + 8 * g;
                uint4 q = make_uint4(0u, 0u, 0u, 0u);
                if (STAGE) {  // rows past m hold stale LDS: they only feed their own (unused) outputs
                    if (kl < h) {
                        const char *src = xs + (16 * t + c) * 2 * h + 2 * kl;
                        const uint2 lo = *reinterpret_cast<const uint2 *>(src);
                        const uint2 hi = kl + 8 <= h ? *reinterpret_cast<const uint2 *>(src + 8) : make_uint2(0u, 0u);
                        q = make_uint4(lo.x, lo.y, hi.x, hi.y);
                    }
                } else if (mr < m && kl < h) {
                    const uint16_t *src = xin + mr * h + kl;
                    const uint2 lo = *reinterpret_cast<const uint2 *>(src);
                    const uint2 hi = kl + 8 <= h ? *reinterpret_cast<const uint2 *>(src + 4) : make_uint2(0u, 0u);
                    q = make_uint4(lo.x, lo.y, hi.x, hi.y);
                }
                const bf16x8_t xa = __builtin_bit_cast(bf16x8_t, q);
                z[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, fb[2][ks], z[t], 0, 0, 0);
                z[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, fb[1][ks], z[t], 0, 0, 0);
                z[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, fb[0][ks], z[t], 0, 0, 0);
            }
        }
        if (!MULTI) break;
    }
    if (c < nout) {
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int r = 0; r < 4; r++) zt[16 * t + 4 * g + r][c] = z[t][r];
    }
}

// Block partials: [dwa 4h | dwv h | dba 4 | dbv 1 | sum ppo, sum H, sum v]  (5h + 8 floats)
//
// 64 rows per wave and iteration, three layouts:
//   heads    logits/value of the 64 rows on MFMA (head_fwd's tiles), through a per-wave LDS
//            transpose to lane = row;
//   loss     lane = row: the scalar loss math runs once per row (not once per lane of a row);
//   backward lane = 4 features: for each row, dx = dz W (20 FMA per lane, row-contiguous float4
//            stores) and the head-weight gradient accumulates dz x in registers.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

// Copies nbytes (a multiple of 8) from global src to the wave's LDS image dst with 16-byte
// LDS-DMA loads (1 KiB per wave instruction, no VGPR staging); an 8-byte tail goes through lane 0.
__device__ __forceinline__ void wave_stage(char *dst, const char *src, int nbytes, int lane) {
    const int n16 = nbytes & ~15;
    for (int off = 0; off < n16; off += 1024) {
        if (off + 16 * lane < n16)
            __builtin_amdgcn_global_load_lds((glb_void_t *)(src + off + 16 * lane), (lds_void_t *)(dst + off), 16, 0, 0);
    }
    if (n16 < nbytes && lane == 0)
        *reinterpret_cast<uint2 *>(dst + n16) = *reinterpret_cast<const uint2 *>(src + n16);
}

template <int J, int KS, bool MULTI, bool DX>
__global__ __launch_bounds__(kThreads) void head_loss_kernel(const uint16_t *__restrict__ xin,
                                                             const float *__restrict__ wa, const float *__restrict__ ba,
                                                             const float *__restrict__ wv, const float *__restrict__ bv,
                                                             int64_t m, int h, HeadLossArgs a,
                                                             float *__restrict__ masked_out, float *__restrict__ dx_out,
                                                             float *__restrict__ dz_out, float *__restrict__ part) {
    // rows >= mv are padding: no loss, zero gradient; the mean is over the mv valid rows
    const int64_t mv = a.rows ? min(*a.rows, m) : m;
    if (a.rows) a.inv_m = 1.0f / (float)max(mv, (int64_t)1);
    // dynamic LDS: per wave the 64-row image of x (h <= 256: STAGE), then the block reduction
    // [kWaves][5h + 8] over the same bytes
    constexpr bool STAGE = !MULTI;
    extern __shared__ float lds[];
    __shared__ float zs[kWaves][64][5], dzs[kWaves][64][5];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
    const int64_t nw = (int64_t)gridDim.x * kWaves;
    const int C = 5 * h + 8;
    char *xs = reinterpret_cast<char *>(lds) + (size_t)wave * 128 * h;
    // MFMA B fragments of the head weights, B[k][n] = W_head n [k] (n < 5), as an exact 3-term bf16
    // split (hi + mid + lo carries all 24 mantissa bits): the logits keep fp32 weights
    bf16x8_t fb[3][KS];
    if (!MULTI) load_head_b3<KS>(fb, wa, wv, h, g, c);
    float w[DX ? 5 : 1][J][4], acc[5][J][4];
    bool ok[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int cc = 4 * (lane + 64 * j);
        ok[j] = cc < h;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (DX) {
#pragma unroll
                for (int k = 0; k < 4; k++) w[DX ? k : 0][j][u] = ok[j] ? wa[k * h + cc + u] : 0.0f;
                w[DX ? 4 : 0][j][u] = ok[j] ? wv[cc + u] : 0.0f;
            }
#pragma unroll
            for (int k = 0; k < 5; k++) acc[k][j][u] = 0.0f;
        }
    }
    const float bsa[4] = {ba[0], ba[1], ba[2], ba[3]}, bsv = bv[0];
    const float beta_c = *a.beta_dev;
    float sb[5] = {0, 0, 0, 0, 0}, s_ppo = 0.0f, s_ent = 0.0f, s_v = 0.0f;

    for (int64_t r0 = ((int64_t)blockIdx.x * kWaves + wave) * 64; r0 < m; r0 += nw * 64) {
        // ---- heads on MFMA: 4 tiles of 16 rows, lane (g, c) gets rows 4g + r, head c
        const int nr = (int)min((int64_t)64, m - r0);
        // the rows' loss inputs and (STAGE) the 64 x rows into LDS, all in flight together
        RowIn in{};
        if (lane < nr) in = load_row_in(a, a.idx[r0 + lane]);
        if (STAGE) {
            wave_stage(xs, reinterpret_cast<const char *>(xin + r0 * h), nr * 2 * h, lane);
            __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0): the image has landed (own wave only)
        }
        // ---- heads on MFMA: 4 tiles of 16 rows, lane (g, c) gets rows 4g + r, head c
        head_tiles<KS, MULTI, STAGE>(zs[wave], fb, xin, wa, wv, m, h, r0, g, c, 5, xs);
        // ---- loss: lane = row (LDS ops of a wave execute in order: the writes above land first)
        {
            const int64_t r = r0 + lane;
            float dz[5] = {0, 0, 0, 0, 0};
            if (lane < nr && r < mv) {
                float z[5], mk[4], ppo, ent, vl;
#pragma unroll
                for (int k = 0; k < 5; k++) z[k] = zs[wave][lane][k] + (k < 4 ? bsa[k] : bsv);
                row_loss(z, in, a, beta_c, dz, mk, ppo, ent, vl);
                *reinterpret_cast<float4 *>(masked_out + r * 4) = make_float4(mk[0], mk[1], mk[2], mk[3]);
                s_ppo += ppo;
                s_ent += ent;
                s_v += vl;
            }
#pragma unroll
            for (int k = 0; k < 5; k++) {
                dzs[wave][lane][k] = dz[k];
                sb[k] += dz[k];
            }
            if (dz_out && lane < nr) {
                *reinterpret_cast<float4 *>(dz_out + r * 8) = make_float4(dz[0], dz[1], dz[2], dz[3]);
                *reinterpret_cast<float4 *>(dz_out + r * 8 + 4) = make_float4(dz[4], 0.0f, 0.0f, 0.0f);
            }
        }
        // ---- backward: lane = 4 features, one row after the other (8 rows' loads in flight)
        constexpr int RB = J == 1 ? 8 : (J == 2 ? 4 : 2);
        for (int q0 = 0; q0 < nr; q0 += RB) {
            float x[RB][J][4];
#pragma unroll
            for (int qq = 0; qq < RB; qq++) {
                const int q = q0 + qq;
#pragma unroll
                for (int j = 0; j < J; j++) {
                    if (ok[j] && q < nr) {
                        if (STAGE) load_bf4_lds(xs + q * 2 * h + 8 * (lane + 64 * j), x[qq][j]);
                        else load_bf4(xin + (r0 + q) * h + 4 * (lane + 64 * j), x[qq][j]);
                    } else {
                        x[qq][j][0] = x[qq][j][1] = x[qq][j][2] = x[qq][j][3] = 0.0f;
                    }
                }
            }
#pragma unroll
            for (int qq = 0; qq < RB; qq++) {
                const int q = q0 + qq;
                if (q >= nr) break;
                float dz[5];
#pragma unroll
                for (int k = 0; k < 5; k++) dz[k] = dzs[wave][q][k];
#pragma unroll
                for (int j = 0; j < J; j++) {
                    if (!ok[j]) continue;
#pragma unroll
                    for (int u = 0; u < 4; u++)
#pragma unroll
                        for (int k = 0; k < 5; k++) acc[k][j][u] += dz[k] * x[qq][j][u];
                    if (!DX) continue;
                    float o[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        float t = 0.0f;
#pragma unroll
                        for (int k = 0; k < 4; k++) t += dz[k] * w[DX ? k : 0][j][u];
                        if (!a.decouple) t += dz[4] * w[DX ? 4 : 0][j][u];
                        o[u] = t;
                    }
                    *reinterpret_cast<float4 *>(dx_out + (r0 + q) * h + 4 * (lane + 64 * j)) =
                        make_float4(o[0], o[1], o[2], o[3]);
                }
            }
        }
    }
    // block reduction: head weight grads (per lane), bias grads and loss sums (per lane -> wave)
#pragma unroll
    for (int k = 0; k < 5; k++) sb[k] = wave_sum(sb[k]);
    s_ppo = wave_sum(s_ppo);
    s_ent = wave_sum(s_ent);
    s_v = wave_sum(s_v);
    if (STAGE) __syncthreads();  // the reduction overwrites the other waves' images
    float *mine = lds + wave * C;
#pragma unroll
    for (int j = 0; j < J; j++) {
        if (!ok[j]) continue;
        const int cc = 4 * (lane + 64 * j);
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int k = 0; k < 5; k++) mine[k * h + cc + u] = acc[k][j][u];
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 5; k++) mine[5 * h + k] = sb[k];
        mine[5 * h + 5] = s_ppo;
        mine[5 * h + 6] = s_ent;
        mine[5 * h + 7] = s_v;
    }
    __syncthreads();
    for (int cc = threadIdx.x; cc < C; cc += kThreads) {
        float t = 0.0f;
#pragma unroll
        for (int w2 = 0; w2 < kWaves; w2++) t += lds[w2 * C + cc];
        part[(int64_t)blockIdx.x * C + cc] = t;
    }
}

// ------------------------------------------------------------------ KL diagnostic ------------
// Block partials: [sum KL, max KL].  Logits of 64 rows per wave on MFMA (fp32 weights as the
// 3-term bf16 split of head_loss), transposed through LDS to lane = row for the KL.
template <int KS, bool MULTI>
__global__ __launch_bounds__(kThreads) void head_kl_kernel(const uint16_t *__restrict__ xin, const float *__restrict__ wa,
                                                           const float *__restrict__ ba, int64_t m, int h,
                                                           const float *__restrict__ old_masked,
                                                           const int64_t *__restrict__ rows, float *__restrict__ part) {
    __shared__ float lds[kWaves][2];
    __shared__ float zs[kWaves][64][5];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
    const int64_t nw = (int64_t)gridDim.x * kWaves;
    bf16x8_t fb[3][KS];
    if (!MULTI) load_head_b3<KS>(fb, wa, nullptr, h, g, c);
    const float bias[4] = {ba[0], ba[1], ba[2], ba[3]};
    float ksum = 0.0f, kmax = -INFINITY;
    const int64_t mv = rows ? min(*rows, m) : m;  // rows >= mv: padding of a ragged minibatch
    for (int64_t r0 = ((int64_t)blockIdx.x * kWaves + wave) * 64; r0 < m; r0 += nw * 64) {
        head_tiles<KS, MULTI>(zs[wave], fb, xin, wa, nullptr, m, h, r0, g, c, 4);
        const int64_t r = r0 + lane;
        if (r < mv) {
            const float4 o4 = *reinterpret_cast<const float4 *>(old_masked + r * 4);
            const float o[4] = {o4.x, o4.y, o4.z, o4.w};
            bool valid[4];
            float mo = -INFINITY, mn = -INFINITY, nz[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                valid[k] = o[k] != -INFINITY;
                nz[k] = valid[k] ? zs[wave][lane][k] + bias[k] : -INFINITY;
                mo = fmaxf(mo, o[k]);
                mn = fmaxf(mn, nz[k]);
            }
            float so = 0.0f, sn = 0.0f;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                so += valid[k] ? expf(o[k] - mo) : 0.0f;
                sn += valid[k] ? expf(nz[k] - mn) : 0.0f;
            }
            const float lso = mo + logf(so), lsn = mn + logf(sn);
            float kl = 0.0f;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (!valid[k]) continue;
                const float lo = o[k] - lso, ln = nz[k] - lsn;
                kl += expf(lo) * (lo - ln);
            }
            ksum += kl;
            kmax = fmaxf(kmax, kl);
        }
    }
    ksum = wave_sum(ksum);
    kmax = wave_max(kmax);
    if (lane == 0) {
        lds[wave][0] = ksum;
        lds[wave][1] = kmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.0f, mx = -INFINITY;
        for (int w2 = 0; w2 < kWaves; w2++) {
            s += lds[w2][0];
            mx = fmaxf(mx, lds[w2][1]);
        }
        part[blockIdx.x * 2] = s;
        part[blockIdx.x * 2 + 1] = mx;
    }
}


// ------------------------------------------------------------------ weight gradient ----------
// C[n1][n2] = sum_m A[m][n1] B[m][n2]  (dW = dG^T X of a Linear layer, A = dG, B = X, both bf16
// row-major [M, n]).  A tall-skinny reduction GEMM on bf16 MFMA (v_mfma_f32_16x16x32_bf16):
// each 256-thread block owns a slab of rows and the WHOLE output (waves tiled WI x WJ, each wave
// BI x BJ 16x16 tiles in registers), stages 64 rows of A and B per step into LDS (two buffers,
// the next step's global loads in flight during the MFMAs) and reads both operands with the
// hardware-transposing ds_read_b64_tr_b16 from the row-major image, so no transpose pass.
// The k order inside a 32-row block is permuted (group g of a half reads rows 4g..4g+3 and
// 16+4g..16+4g+3) identically for both operands; with the row pitch == 32 mod 256 bytes the
// 8 rows a 32-lane half touches fill the 64 banks exactly (conflict-free).  Per-block partial
// outputs are summed in a fixed order by colsum1/2 (deterministic).

constexpr int kWgRows = 64;
constexpr int kWgThreads = 256;  // 4 waves: one 139-KB-LDS block per CU, 512 registers per lane
// 8-B staging chunks per thread per step and operand (n <= 224): 64 rows x 56 chunks / threads
__host__ __device__ constexpr int wg_items(int threads) { return (kWgRows * 56 + threads - 1) / threads; }
// NW = 8 (the h = 196 layers): two waves per tile block split each 64-row step's two 32-row
// k-blocks between them (two waves per SIMD: one's MFMAs overlap the other's fragment reads and
// the staging), and the second half's accumulators are added through LDS before the store.
__host__ __device__ constexpr size_t wg_combine_bytes(int bi, int bj) { return (size_t)4 * bi * bj * 256 * 4; }

__device__ __forceinline__ bf16x8_t wg_frag(const char *buf, int pitch, int kb, int c0, int lane) {
    const int g = (lane >> 4) & 3, q = (lane >> 2) & 3, p = lane & 3;
    const char *a1 = buf + (kb * 32 + 4 * g + q) * pitch + (c0 + 4 * p) * 2;
    const s16x4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)a1);
    const s16x4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(a1 + 16 * pitch));
    // whole-vector reinterpretation (element-wise __bf16 casts of the i16 lanes miscompile)
    const s16x8_t v = __builtin_shufflevector(t1, t2, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, v);
}

// gridDim.z == 2: a second product of the same shape (A2, B2 -> part2) in the same launch.
template <int BI, int BJ, int NW = 4>
__global__ __launch_bounds__(64 * NW) void wgrad_kernel(const uint16_t *__restrict__ A, const uint16_t *__restrict__ B,
                                                        int64_t M, int n1, int n2, int pa, int pb, int wi_n,
                                                        int64_t rows_per_block, int bw, float *__restrict__ part,
                                                        const uint16_t *__restrict__ A2 = nullptr,
                                                        const uint16_t *__restrict__ B2 = nullptr,
                                                        float *__restrict__ part2 = nullptr) {
    if (blockIdx.z == 1) {  // block-uniform
        A = A2;
        B = B2;
        part = part2;
    }
    constexpr int kThr = 64 * NW, kItems = wg_items(kThr), KSPLIT = NW / 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wave = wave_all & 3, sub = wave_all >> 2;  // tile block, k-split half
    const int ti0 = (wave % wi_n) * BI, tj0 = (wave / wi_n) * BJ;  // wave-uniform: scalar branches
    // blockIdx.y picks a band of bw output columns (B columns cb0 .. cb0 + w): more blocks in flight
    const int cb0 = (int)blockIdx.y * bw, w = min(bw, n2 - cb0);
    const int TI = (n1 + 15) >> 4, TJ = (w + 15) >> 4;
    const int stage_bytes = kWgRows * (pa + pb);
    for (int o = tid * 16; o < 2 * stage_bytes; o += kThr * 16) *reinterpret_cast<uint4 *>(smem + o) = make_uint4(0, 0, 0, 0);

    // Staging: the 64 rows of a step are one contiguous span of A (and of B) in HBM, read as
    // 8-byte chunks c = tid + 256u; each chunk's LDS slot (row pitch pa / pb) is fixed per thread.
    const int ga = n1 >> 2, gb = w >> 2, ca = kWgRows * ga, cb = kWgRows * gb;
    const int64_t r_begin = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r_end = min(M, r_begin + rows_per_block);
    int offa[kItems], offb[kItems], srcb[kItems], rowb[kItems];
#pragma unroll
    for (int u = 0; u < kItems; u++) {
        const int c = tid + u * kThr;
        const int ra = c / ga, rb = c / gb, qb = c - rb * gb;
        offa[u] = ra * pa + 8 * (c - ra * ga);
        offb[u] = kWgRows * pa + rb * pb + 8 * qb;
        srcb[u] = rb * n2 + cb0 + 4 * qb;  // element offset of the chunk from the step's first row
        rowb[u] = rb;
    }
    uint2 rega[kItems], regb[kItems];
    auto load = [&](int64_t r0) {
        const char *sa = reinterpret_cast<const char *>(A + r0 * n1);
        const uint16_t *sb = B + r0 * n2;
        const int64_t va = (r_end - r0) * ga, vrows = r_end - r0;  // valid chunks / rows
#pragma unroll
        for (int u = 0; u < kItems; u++) {
            const int c = tid + u * kThr;
            rega[u] = (c < ca && c < va) ? *reinterpret_cast<const uint2 *>(sa + 8 * c) : make_uint2(0, 0);
            regb[u] = (c < cb && rowb[u] < vrows) ? *reinterpret_cast<const uint2 *>(sb + srcb[u]) : make_uint2(0, 0);
        }
    };
    auto store = [&](int s) {
        char *base = smem + s * stage_bytes;
#pragma unroll
        for (int u = 0; u < kItems; u++) {
            const int c = tid + u * kThr;
            if (c < ca) *reinterpret_cast<uint2 *>(base + offa[u]) = rega[u];
            if (c < cb) *reinterpret_cast<uint2 *>(base + offb[u]) = regb[u];
        }
    };
    f32x4_t acc[BI][BJ];
#pragma unroll
    for (int i = 0; i < BI; i++)
#pragma unroll
        for (int j = 0; j < BJ; j++) acc[i][j] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};

    __syncthreads();  // zero fill done before the first tile lands
    if (r_begin < r_end) {
        load(r_begin);
        store(0);
    }
    __syncthreads();
    int s = 0;
    for (int64_t r0 = r_begin; r0 < r_end; r0 += kWgRows) {
        const bool more = r0 + kWgRows < r_end;
        if (more) load(r0 + kWgRows);
        const char *ba = smem + s * stage_bytes, *bb = ba + kWgRows * pa;
        if (ti0 < TI && tj0 < TJ) {  // wave-uniform; inside, every MFMA is unconditional (a guarded
                                     // MFMA makes the compiler copy its accumulator out and wait)
#pragma unroll
            for (int kb = 0; kb < 2; kb++) {
                if (KSPLIT == 2 && kb != sub) continue;  // wave-uniform
                bf16x8_t fb[BJ];
#pragma unroll
                for (int j = 0; j < BJ; j++) fb[j] = wg_frag(bb, pb, kb, 16 * (tj0 + j), lane);
#pragma unroll
                for (int i = 0; i < BI; i++) {
                    const bf16x8_t fa = wg_frag(ba, pa, kb, 16 * (ti0 + i), lane);
#pragma unroll
                    for (int j = 0; j < BJ; j++)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
                }
            }
        }
        if (more) store(s ^ 1);
        __syncthreads();
        s ^= 1;
    }
    if (KSPLIT == 2) {  // the second k half's accumulators join the first's through LDS
        f32x4_t *cmb = reinterpret_cast<f32x4_t *>(smem) + (size_t)wave * BI * BJ * 64;
        if (sub == 1 && ti0 < TI && tj0 < TJ)
#pragma unroll
            for (int i = 0; i < BI; i++)
#pragma unroll
                for (int j = 0; j < BJ; j++) cmb[(i * BJ + j) * 64 + lane] = acc[i][j];
        __syncthreads();
        if (sub == 1) return;
        if (ti0 < TI && tj0 < TJ)
#pragma unroll
            for (int i = 0; i < BI; i++)
#pragma unroll
                for (int j = 0; j < BJ; j++) acc[i][j] = acc[i][j] + cmb[(i * BJ + j) * 64 + lane];
    }
    float *out = part + (int64_t)blockIdx.x * n1 * n2;
    const int col = lane & 15, rowq = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < BI; i++)
#pragma unroll
        for (int j = 0; j < BJ; j++) {
            const int ii = 16 * (ti0 + i) + rowq, jj = cb0 + 16 * (tj0 + j) + col;
            if (ti0 + i < TI && tj0 + j < TJ && jj < cb0 + w)
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (ii + r < n1) out[(int64_t)(ii + r) * n2 + jj] = acc[i][j][r];
        }
}


// ------------------------------------------------------------------ fused Linear + LN block --
// One ResidualBlock (or the stem) forward in one kernel:
//     G = X W^T (bf16, kept for the backward),  Y = [X +] Dropout(ReLU(LayerNorm(G)))
// computed as Y^T = W X^T on v_mfma_f32_16x16x32_bf16 so that a lane ends up holding 4
// consecutive features of one row per 16-feature tile: the LayerNorm row reductions are two
// cross-lane steps and every G / Y / residual access is an 8-byte vector.  W (<= 256 x 256 bf16)
// is staged once per block in LDS; X is read from HBM exactly once, straight into MFMA fragments.
// Per 65536 x 196 layer this moves X + G + Y (+ X again for the residual): ~77-103 MB, instead
// of the GEMM's X + G plus the separate LayerNorm pass's G + X + Y.
constexpr int kMfWaves = 4;
constexpr int kMfThreads = 64 * kMfWaves;
constexpr int kMfRows = 16 * kMfWaves;  // rows per slab: a 16-row MFMA tile per wave
constexpr int kMfItems = 16;            // 8-byte staging chunks per thread per slab (K <= 256)

// LDS row pitch (bytes) of a bf16 image with kp columns: 16 rows read at the same column by a
// 16-byte fragment load fall into 16 distinct 4-bank groups when pitch/4 is an odd multiple of 4.
__host__ __device__ inline int mf_pitch(int kp) {
    int dw = (kp + 1) / 2;
    dw = (dw + 3) & ~3;
    if (((dw >> 2) & 1) == 0) dw += 4;
    return dw * 4;
}

// KS > 0: the fixed-shape path (KS k-steps of 32 columns: the h = 196 blocks KS = 7, the stem KS = 2):
// both LDS images are zero-padded to NT * 16 W rows and KS * 32 columns at a compile-time pitch, so
// the MFMA loop is fully unrolled with immediate LDS offsets and no per-fragment address arithmetic
// or range selects.
__host__ __device__ constexpr int mf_fixed_pitch(int ks) { return 64 * ks + 16; }  // 16 B x odd

template <int NT, int KS, bool RES, bool DROP>
__global__ __launch_bounds__(kMfThreads) void mlp_fwd_kernel(const uint16_t *__restrict__ X,
                                                             const uint16_t *__restrict__ W,
                                                             const float *__restrict__ gamma,
                                                             const float *__restrict__ beta, uint16_t *__restrict__ G,
                                                             uint16_t *__restrict__ Y, float *__restrict__ mean_out,
                                                             float *__restrict__ rstd_out, int64_t M, int N, int K,
                                                             DropArgs da) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // W image: N rows (fixed path: NT * 16, the extra rows zero), zero K padding
    const int kp = (K + 7) & ~7, pw = KS ? mf_fixed_pitch(KS) : mf_pitch(kp);
    const int wrows = KS ? 16 * NT : N;
    char *sW = smem;
    char *sX0 = smem + ((wrows * pw + 15) & ~15);   // two 64-row X slabs (double buffer)
    const int xbytes = kMfRows * pw;
    char *zero = sX0 + 2 * xbytes;
    float *sgb = reinterpret_cast<float *>(zero + 64);  // gamma[N], beta[N]
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, col = lane & 15;
    // zero everything once (K padding of W and of both X buffers must read as zero)
    for (int o = tid * 16; o < (int)(zero - smem) + 64; o += kMfThreads * 16)
        *reinterpret_cast<uint4 *>(smem + o) = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    {  // W is one contiguous span: 8-byte chunks, 16 loads in flight per thread per batch
        const int q4w = K >> 2, nw = N * q4w;
        for (int c0 = 0; c0 < nw; c0 += 16 * kMfThreads) {
            uint2 v[16];
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const int c = c0 + tid + u * kMfThreads;
                v[u] = c < nw ? *reinterpret_cast<const uint2 *>(W + 4 * (int64_t)c) : make_uint2(0u, 0u);
            }
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const int c = c0 + tid + u * kMfThreads;
                if (c < nw) {
                    const int r = c / q4w;
                    *reinterpret_cast<uint2 *>(sW + r * pw + 8 * (c - r * q4w)) = v[u];
                }
            }
        }
    }
    for (int e = tid; e < N; e += kMfThreads) {
        sgb[e] = gamma[e];
        sgb[N + e] = beta[e];
    }
    const Drop d = make_drop(da);
    const float inv_n = 1.0f / (float)N;
    const int64_t nslab = (M + kMfRows - 1) / kMfRows;

    // staging of a slab: its rows are one contiguous span of X, read as 8-byte chunks
    const int q4 = K >> 2, nchunk = kMfRows * q4;
    int off[kMfItems];
#pragma unroll
    for (int u = 0; u < kMfItems; u++) {
        const int c = tid + u * kMfThreads, r = c / q4;
        off[u] = r * pw + 8 * (c - r * q4);
    }
    uint2 reg[kMfItems];
    auto load = [&](int64_t slab) {
        const uint16_t *src = X + slab * kMfRows * K;
        const int64_t valid = (M - slab * kMfRows) * q4;  // chunks inside the matrix
#pragma unroll
        for (int u = 0; u < kMfItems; u++) {
            const int c = tid + u * kMfThreads;
            reg[u] = (c < nchunk && c < valid) ? *reinterpret_cast<const uint2 *>(src + 4 * c) : make_uint2(0u, 0u);
        }
    };
    auto store = [&](char *buf) {
#pragma unroll
        for (int u = 0; u < kMfItems; u++) {
            const int c = tid + u * kMfThreads;
            if (c < nchunk) *reinterpret_cast<uint2 *>(buf + off[u]) = reg[u];
        }
    };
    int64_t slab = blockIdx.x;
    if (slab < nslab) {
        load(slab);
        store(sX0);
    }
    __syncthreads();
    int cur = 0;
    for (; slab < nslab; slab += gridDim.x) {
        const bool more = slab + gridDim.x < nslab;
        if (more) load(slab + gridDim.x);  // next slab's HBM reads in flight during this slab
        const char *sx = sX0 + cur * xbytes;
        const char *xrow = sx + (wave * 16 + col) * pw;
        f32x4_t acc[NT];
#pragma unroll
        for (int n = 0; n < NT; n++) acc[n] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (KS > 0) {  // every fragment in range: unrolled, immediate offsets
            const char *xb = xrow + 16 * g, *wb = sW + col * pw + 16 * g;
#pragma unroll
            for (int ks = 0; ks < KS; ks++) {
                const bf16x8_t fx = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4 *>(xb + 64 * ks));
#pragma unroll
                for (int n = 0; n < NT; n++) {
                    const bf16x8_t fw =
                        __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4 *>(wb + n * 16 * pw + 64 * ks));
                    acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw, fx, acc[n], 0, 0, 0);
                }
            }
        } else
        for (int k0 = 0; k0 < kp; k0 += 32) {
            const int kl = k0 + 8 * g;
            const bf16x8_t fx =
                __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4 *>(kl < kp ? xrow + 2 * kl : zero));
#pragma unroll
            for (int n = 0; n < NT; n++) {  // A operand: W[n][k .. k+7]
                const int row = 16 * n + col;
                const char *pp = (row < N && kl < kp) ? sW + row * pw + 2 * kl : zero;
                const bf16x8_t fw = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4 *>(pp));
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw, fx, acc[n], 0, 0, 0);
            }
        }
        // epilogue: lane holds row m = slab*64 + 16*wave + col, features 16n + 4g + r.  The
        // LayerNorm arithmetic is ln_row.hpp's (shared bitwise with the fused rollout kernel).
        namespace R = g2048::lnrow;
        const int64_t m = slab * kMfRows + wave * 16 + col;
        R::f32x2 v[NT][2];
        uint2 gb[NT];
        R::round_g<NT>(acc, v, gb);
        float mean, rstd;
        R::stats<NT>(v, [&](int n) { return 16 * n + 4 * g < N; }, inv_n, mean, rstd);
        if (m < M) {
            if (g == 0 && mean_out) {
                mean_out[m] = mean;
                rstd_out[m] = rstd;
            }
            uint4 dpair = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int n = 0; n < NT; n++) {
                const int f0 = 16 * n + 4 * g;
                if (f0 >= N) continue;
                const float4 ga = *reinterpret_cast<const float4 *>(sgb + f0);
                const float4 be = *reinterpret_cast<const float4 *>(sgb + N + f0);
                R::f32x2 y0 = R::affine_relu(v[n][0], rstd, R::f32x2{ga.x, ga.y}, R::f32x2{be.x, be.y});
                R::f32x2 y1 = R::affine_relu(v[n][1], rstd, R::f32x2{ga.z, ga.w}, R::f32x2{be.z, be.w});
                if (DROP) {  // tiles n, n+1 hold column groups 4n+g, 4n+4+g: one Philox call
                    float k[4];
                    if ((n & 1) == 0) dpair = drop_draw4(d, (uint32_t)m, (uint32_t)(f0 >> 2));
                    drop_mult_bits(d, drop_half(dpair, (uint32_t)(f0 >> 2)), k);
                    y0 = y0 * R::f32x2{k[0], k[1]};
                    y1 = y1 * R::f32x2{k[2], k[3]};
                }
                if (RES) {  // the residual is this layer's input, already in LDS
                    const uint2 w = *reinterpret_cast<const uint2 *>(xrow + 2 * f0);
                    y0 = R::f32x2{R::bf_lo(w.x), R::bf_hi(w.x)} + y0;
                    y1 = R::f32x2{R::bf_lo(w.y), R::bf_hi(w.y)} + y1;
                }
                if (G) *reinterpret_cast<uint2 *>(G + m * N + f0) = gb[n];
                *reinterpret_cast<uint2 *>(Y + m * N + f0) = make_uint2(R::pack_bf2(y0.x, y0.y), R::pack_bf2(y1.x, y1.y));
            }
        }
        if (more) store(sX0 + (cur ^ 1) * xbytes);  // the other buffer: last read one slab ago
        __syncthreads();
        cur ^= 1;
    }
}

// The h = 196 layers (the README model: blocks 196 -> 196, stem 48 -> 196).  One image of W per CU
// in LDS (conflict-free swizzled pitch), 8 waves, each owning 16-row tiles with no barrier after
// the staging: the wave reads its X^T B fragments straight from HBM into registers (the first
// tile's reads are issued before the W image is written, so they overlap the staging; later tiles'
// reads go out as soon as the previous fragments are consumed), runs the 91 MFMAs, and the
// LayerNorm / ReLU / dropout / residual epilogue of ln_row.hpp.  G and Y leave through a per-wave
// LDS tile: the 16 rows of a tile are one contiguous 6 272-B span of the output, written as 16-B
// lanes (the MFMA layout would scatter 32-B pieces over 16 rows).  Per accumulator the MFMA
// sequence (k-steps in order, same fragments) and the epilogue are mlp_fwd_kernel's, so both
// compute bitwise the same G / Y / statistics.  The residual is re-read in the epilogue's layout
// (an L2 hit: the wave read the same rows moments before).  N and K are compile-time, so every
// range test outside the last W tile / k-step folds away.
//
// Measured alternatives (tools/time_mlp.py, 65 536 rows): 32-row tiles per wave (two MFMAs per W
// fragment) +8-30 % (registers: the dropout variant spills), 16 waves per CU (128-VGPR cap, spills)
// +50 %, the slab kernel +40 %; removing any one of X reads, MFMAs or epilogue arithmetic from
// this kernel saves only ~4 us each: it is latency-bound on the per-wave chain, not on one unit.
constexpr int kMwWaves = 8;
constexpr int kMwThreads = 64 * kMwWaves;
constexpr int kMwNT = 13;
constexpr int kMwN = 196;
constexpr int kMwOut = 16 * kMwN * 2;  // bytes of one 16-row output tile (6 272)

__host__ __device__ constexpr int mw_ks(int k) { return (k + 31) / 32; }
// W image row pitch: 16 B x P with P = 4 or 12 mod 16 (>= 4 KS slots), and 16-B slot q of row r
// stored at slot q ^ mw_swz(r).  A ds_read_b128 fragment read (lane (g, c) reads slot 4 ks + g of
// row 16 n + c) then puts each of the instruction's four 16-lane bank groups ({0-3, 12-15, 20-27},
// ... MI355X_MICROARCH.md, LDS) on 16 distinct slots of the 256-B bank row: conflict-free.
__host__ __device__ constexpr int mw_pitch(int ks) {
    return 16 * ((4 * ks) % 16 == 4 || (4 * ks) % 16 == 12 ? 4 * ks : 4 * ks + 4);
}
__device__ __forceinline__ int mw_swz(int r) { return (0x1230 >> (4 * ((r >> 2) & 3))) & 3; }  // 0, 3, 2, 1
__host__ __device__ constexpr size_t mw_w_bytes(int k) { return (size_t)16 * kMwNT * mw_pitch(mw_ks(k)); }
__host__ __device__ constexpr size_t mw_lds_bytes(int k, bool kl = false) {
    return mw_w_bytes(k) + (size_t)8 * kMwN + (size_t)kMwWaves * kMwOut + (kl ? (size_t)4 * 4 * 16 * kMwNT : 0);
}

// one 16-row output tile from the wave's LDS tile to HBM as contiguous 16-B lanes: `rows` valid
// rows (a row is 392 B, so an odd count ends in the middle of a 16-B chunk: that chunk goes as 8 B)
__device__ __forceinline__ void mw_flush(const char *t, uint16_t *dst, int rows, int lane) {
    const int bytes = rows * 2 * kMwN;
#pragma unroll
    for (int i = 0; i < (kMwOut + 1023) / 1024; i++) {
        const int o = 16 * (lane + 64 * i);
        if (o + 16 <= bytes) {
            *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(dst) + o) = *reinterpret_cast<const uint4 *>(t + o);
        } else if (o < bytes) {
            *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(dst) + o) = *reinterpret_cast<const uint2 *>(t + o);
        }
    }
}

// KL (the post-step re-forward's last block, train.py:578-601): instead of storing Y, the block
// output (bf16-rounded, as the stored H would be) goes straight into the action head (fp32 Wa in
// LDS) and the KL(old || new) of each row is summed / maxed into the block's partial pair, the
// layout of head_kl_kernel: no H write, no H re-read, no head launch.
struct KlArgs {
    const float *wa, *ba, *old_masked;
    const int64_t *rows;
    float *part;
};

template <int K, bool RES, bool DROP, bool KL = false>
__global__ __launch_bounds__(kMwThreads) void mlp_fwd_wide_kernel(const uint16_t *__restrict__ X,
                                                                  const uint16_t *__restrict__ W,
                                                                  const float *__restrict__ gamma,
                                                                  const float *__restrict__ beta,
                                                                  uint16_t *__restrict__ G, uint16_t *__restrict__ Y,
                                                                  float *__restrict__ mean_out,
                                                                  float *__restrict__ rstd_out, int64_t M,
                                                                  DropArgs da, KlArgs ka = KlArgs{}) {
    constexpr int N = kMwN, NT = kMwNT, KS = mw_ks(K), PW = mw_pitch(KS);
    constexpr int CPR = 8 * KS;                                 // 8-byte chunks per padded W row (<= 64)
    constexpr int RPW = (16 * NT + kMwWaves - 1) / kMwWaves;    // padded W rows staged per wave
    static_assert(K % 4 == 0 && CPR <= 64 && 16 * NT >= N, "shape");
    static_assert((PW / 16) % 16 == 4 || (PW / 16) % 16 == 12, "pitch");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char *sW = smem;
    float *sgb = reinterpret_cast<float *>(smem + mw_w_bytes(K));  // gamma[N], beta[N]
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    char *sO = smem + mw_w_bytes(K) + 8 * N + wave * kMwOut;         // this wave's output tile
    const int g = lane >> 4, col = lane & 15;
    const int64_t ntile = (M + 15) >> 4, stride = (int64_t)gridDim.x * kMwWaves;
    int64_t tile = (int64_t)blockIdx.x * kMwWaves + wave;

    // the padded W image: wave w stages rows w, w + 8, ..., lane q its 8-byte chunk q; every
    // global load in flight before the first LDS write
    const bool qin = lane < CPR, qk = 4 * lane < K;
    uint2 wv[RPW];
#pragma unroll
    for (int u = 0; u < RPW; u++) {
        const int r = wave + kMwWaves * u;  // wave-uniform
        const uint2 t = *reinterpret_cast<const uint2 *>(W + (int64_t)(r < N ? r : 0) * K + (qk ? 4 * lane : 0));
        wv[u] = (r < N && qk) ? t : make_uint2(0u, 0u);
    }
    // B fragments of a tile: lane (g, col) holds row 16 t + col, columns 32 ks + 8 g .. + 7 (zero
    // past K; K % 4 == 0 so a partial chunk is 4 columns).  Loads are unconditional from clamped
    // addresses: a row past M reads row 0, which only feeds that row's own (never stored) outputs.
    bf16x8_t fx[KS];
    auto load_x = [&](int64_t t) {
        const int64_t row = 16 * t + col;
        const uint16_t *xr = X + (row < M ? row : 0) * K;
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            const int k0 = 32 * ks + 8 * g;
            uint2 lo, hi;
            if (32 * ks + 32 <= K) {  // the whole k-step inside K (folds after unrolling)
                lo = *reinterpret_cast<const uint2 *>(xr + k0);
                hi = *reinterpret_cast<const uint2 *>(xr + k0 + 4);
            } else {
                const uint2 a = *reinterpret_cast<const uint2 *>(xr + (k0 < K ? k0 : 0));
                const uint2 b = *reinterpret_cast<const uint2 *>(xr + (k0 + 4 < K ? k0 + 4 : 0));
                lo = k0 < K ? a : make_uint2(0u, 0u);
                hi = k0 + 4 < K ? b : make_uint2(0u, 0u);
            }
            fx[ks] = __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
        }
    };
    if (tile < ntile) load_x(tile);  // in flight across the W image's LDS writes and the barrier
    if (qin)
#pragma unroll
        for (int u = 0; u < RPW; u++) {
            const int r = wave + kMwWaves * u;
            if (r < 16 * NT)  // 8-byte chunk lane of 16-B slot lane / 2, swizzled
                *reinterpret_cast<uint2 *>(sW + r * PW + 16 * ((lane >> 1) ^ mw_swz(r)) + 8 * (lane & 1)) = wv[u];
        }
    for (int e = tid; e < N; e += kMwThreads) {
        sgb[e] = gamma[e];
        sgb[N + e] = beta[e];
    }
    // KL: Wa [4][208] fp32 (zero past N) after this block's output tiles
    float *swa = reinterpret_cast<float *>(smem + mw_w_bytes(K) + 8 * N + (size_t)kMwWaves * kMwOut);
    if (KL)
        for (int e = tid; e < 4 * 16 * NT; e += kMwThreads) {
            const int k = e / (16 * NT), f = e - k * 16 * NT;
            swa[e] = f < N ? ka.wa[k * N + f] : 0.0f;
        }
    __syncthreads();
    const Drop d = make_drop(da);
    constexpr float inv_n = 1.0f / (float)N;
    float ksum = 0.0f, kmax = -INFINITY;
    const int64_t mv = KL ? (ka.rows ? min(*ka.rows, M) : M) : M;
    const char *wb = sW + col * PW + 16 * (g ^ mw_swz(col));  // rows 16 n + col share the swizzle
    const bool lastok = 16 * (NT - 1) + 4 * g < N;           // this lane's 4-group of the last W tile is real
    auto valid = [&](int n) { return n < NT - 1 || lastok; };
    char *orow = sO + col * 2 * N + 8 * g;                    // lane's spot in the LDS output tile
    namespace R = g2048::lnrow;
    for (; tile < ntile; tile += stride) {
        f32x4_t acc[NT];
#pragma unroll
        for (int n = 0; n < NT; n++)  // W tile-row outer: its KS fragments are the only ones in flight
#pragma unroll
            for (int ks = 0; ks < KS; ks++) {
                const bf16x8_t fw =
                    __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4 *>(wb + n * 16 * PW + 64 * ks));
                const f32x4_t z = {0.0f, 0.0f, 0.0f, 0.0f};  // k-step 0 starts from the inline zero
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw, fx[ks], ks ? acc[n] : z, 0, 0, 0);
            }
        const int64_t m = 16 * tile + col;
        const int rows = (int)(M - 16 * tile < 16 ? M - 16 * tile : 16);  // valid rows of this tile
        // the residual rows first, then (the fragments are consumed) the next tile's reads: loads
        // complete in issue order, so the epilogue's wait for the residual never waits for them
        uint2 xres[NT];
        if (RES) {
            const int64_t mc = m < M ? m : 0;
#pragma unroll
            for (int n = 0; n < NT; n++)
                xres[n] = *reinterpret_cast<const uint2 *>(X + mc * K + 16 * n + 4 * g * valid(n));
        }
        if (tile + stride < ntile) load_x(tile + stride);
        R::f32x2 v[NT][2];
        {
            uint2 gb[NT];
            R::round_g<NT>(acc, v, gb);
            if (G) {  // G through the LDS tile at once: its bits need no register past this point
#pragma unroll
                for (int n = 0; n < NT; n++)
                    if (valid(n)) *reinterpret_cast<uint2 *>(orow + 32 * n) = gb[n];
                mw_flush(sO, G + 16 * tile * N, rows, lane);
            }
        }
        float mean, rstd;
        R::stats<NT>(v, valid, inv_n, mean, rstd);
        if (g == 0 && mean_out && m < M) {
            mean_out[m] = mean;
            rstd_out[m] = rstd;
        }
        uint4 dpair = make_uint4(0u, 0u, 0u, 0u);
        R::f32x2 lg01 = {0.0f, 0.0f}, lg23 = {0.0f, 0.0f};  // KL: this lane's share of the 4 logits
#pragma unroll
        for (int n = 0; n < NT; n++) {
            const int f0 = 16 * n + 4 * g;
            if (!valid(n)) continue;
            const float4 ga = *reinterpret_cast<const float4 *>(sgb + f0);
            const float4 be = *reinterpret_cast<const float4 *>(sgb + N + f0);
            R::f32x2 y0 = R::affine_relu(v[n][0], rstd, R::f32x2{ga.x, ga.y}, R::f32x2{be.x, be.y});
            R::f32x2 y1 = R::affine_relu(v[n][1], rstd, R::f32x2{ga.z, ga.w}, R::f32x2{be.z, be.w});
            if (DROP) {
                float k[4];
                if ((n & 1) == 0) dpair = drop_draw4(d, (uint32_t)m, (uint32_t)(f0 >> 2));
                drop_mult_bits(d, drop_half(dpair, (uint32_t)(f0 >> 2)), k);
                y0 = y0 * R::f32x2{k[0], k[1]};
                y1 = y1 * R::f32x2{k[2], k[3]};
            }
            if (RES) {
                y0 = R::f32x2{R::bf_lo(xres[n].x), R::bf_hi(xres[n].x)} + y0;
                y1 = R::f32x2{R::bf_lo(xres[n].y), R::bf_hi(xres[n].y)} + y1;
            }
            const uint2 yb = make_uint2(R::pack_bf2(y0.x, y0.y), R::pack_bf2(y1.x, y1.y));
            if (KL) {  // logits of the bf16 output: feature f contributes yb[f] * Wa[k][f] to logit k
                const float yv[4] = {R::bf_lo(yb.x), R::bf_hi(yb.x), R::bf_lo(yb.y), R::bf_hi(yb.y)};
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const R::f32x2 y2 = {yv[u], yv[u]};
                    lg01 = R::fma2(y2, R::f32x2{swa[f0 + u], swa[16 * NT + f0 + u]}, lg01);
                    lg23 = R::fma2(y2, R::f32x2{swa[2 * 16 * NT + f0 + u], swa[3 * 16 * NT + f0 + u]}, lg23);
                }
            } else {
                *reinterpret_cast<uint2 *>(orow + 32 * n) = yb;
            }
        }
        if (!KL) {
            mw_flush(sO, Y + 16 * tile * N, rows, lane);
        } else {  // the row's logits (all 4 lanes of the row), then its KL on lane g == 0
            const float z[4] = {R::xor32_add(R::xor16_add(lg01.x)) + ka.ba[0], R::xor32_add(R::xor16_add(lg01.y)) + ka.ba[1],
                                R::xor32_add(R::xor16_add(lg23.x)) + ka.ba[2], R::xor32_add(R::xor16_add(lg23.y)) + ka.ba[3]};
            if (g == 0 && m < mv) {
                const float4 o4 = *reinterpret_cast<const float4 *>(ka.old_masked + m * 4);
                const float o[4] = {o4.x, o4.y, o4.z, o4.w};
                bool ok4[4];
                float mo = -INFINITY, mn = -INFINITY, nz[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    ok4[k] = o[k] != -INFINITY;
                    nz[k] = ok4[k] ? z[k] : -INFINITY;
                    mo = fmaxf(mo, o[k]);
                    mn = fmaxf(mn, nz[k]);
                }
                float so = 0.0f, sn = 0.0f;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    so += ok4[k] ? expf(o[k] - mo) : 0.0f;
                    sn += ok4[k] ? expf(nz[k] - mn) : 0.0f;
                }
                const float lso = mo + logf(so), lsn = mn + logf(sn);
                float kl = 0.0f;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (!ok4[k]) continue;
                    const float lo = o[k] - lso, ln = nz[k] - lsn;
                    kl += expf(lo) * (lo - ln);
                }
                ksum += kl;
                kmax = fmaxf(kmax, kl);
            }
        }
    }
    if (KL) {  // per block: (sum, max) of the rows' KL -> ka.part[blockIdx] (head_kl_kernel's layout)
        ksum = wave_sum(ksum);
        kmax = wave_max(kmax);
        float *red = reinterpret_cast<float *>(sgb);  // gamma / beta are no longer read
        __syncthreads();
        if (lane == 0) {
            red[2 * wave] = ksum;
            red[2 * wave + 1] = kmax;
        }
        __syncthreads();
        if (tid == 0) {
            float s2 = 0.0f, mx = -INFINITY;
            for (int w2 = 0; w2 < kMwWaves; w2++) {
                s2 += red[2 * w2];
                mx = fmaxf(mx, red[2 * w2 + 1]);
            }
            ka.part[blockIdx.x * 2] = s2;
            ka.part[blockIdx.x * 2 + 1] = mx;
        }
    }
}

// ------------------------------------------------------------------ h = 196 LayerNorm backward
// ln_bwd_kernel for the README model's blocks (h = 196, dy = heads' share + up to 2 matmul
// gradients, no fp32 residual gradient) in the MFMA epilogue layout of mlp_fwd_wide_kernel: a wave
// owns 16-row tiles, lane (g, c) holds row 16 t + c, features 16 n + 4 g .. + 3 (n < 13), so a row
// reduction is two cross-lane swaps, all 64 lanes are busy (208 slots for 196 features instead of
// 256) and one dropout Philox call serves two tiles n, n + 1 (the forward's draw, drop_draw4).
// The heads' share of dy, dz W_heads (rank 5), comes out of two v_mfma_f32_16x16x4_f32 per tile n
// already in this layout (A = the head weights, held as fragments for the whole launch; B = the
// tile's dz rows).  Pass 1 forms the masked gradient dzr (kept: 52 registers), the dgamma / dbeta
// accumulators and the row sums; pass 2 recomputes xhat from the raw G bits and writes dG through
// the wave's LDS tile as contiguous 16-B stores.  dgamma / dbeta: each lane accumulates its
// features over its rows across tiles; one 16-lane rotate-sum per wave and one LDS sum per block
// at the end give the same [block][2 h] partial rows as ln_bwd_kernel.
constexpr int kLbWaves = 8;
constexpr int kLbThreads = 64 * kLbWaves;
constexpr int kLbPad = 16 * kMwNT;  // 208 feature slots

__host__ __device__ constexpr size_t lb_lds_bytes() {
    return (size_t)4 * 10 * kLbPad + (size_t)kLbWaves * (kMwOut > 4 * 2 * kLbPad ? kMwOut : 4 * 2 * kLbPad);
}

__device__ __forceinline__ float row16_sum(float v) {  // sum over the 16 lanes of a DPP row (every lane)
    v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), 0x128, 0xF, 0xF, false));  // row_ror:8
    v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), 0x124, 0xF, 0xF, false));  // row_ror:4
    v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), 0x122, 0xF, 0xF, false));  // row_ror:2
    v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), 0x121, 0xF, 0xF, false));  // row_ror:1
    return v;
}

template <bool DROP, bool HEAD, int NP>
__global__ __launch_bounds__(kLbThreads) void ln_bwd196_kernel(DySrc src, const uint16_t *__restrict__ g,
                                                                const float *__restrict__ mean_in,
                                                                const float *__restrict__ rstd_in,
                                                                const float *__restrict__ gamma,
                                                                const float *__restrict__ beta,
                                                                uint16_t *__restrict__ dg, float *__restrict__ part,
                                                                int64_t m, DropArgs da) {
    constexpr int N = kMwN, NT = kMwNT;
    namespace R = g2048::lnrow;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *sgm = reinterpret_cast<float *>(smem), *sbt = sgm + kLbPad;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int gq = lane >> 4, col = lane & 15;
    char *sO = smem + 4 * 10 * kLbPad + wave * (kMwOut > 4 * 2 * kLbPad ? kMwOut : 4 * 2 * kLbPad);
    for (int e = tid; e < kLbPad; e += kLbThreads) {
        sgm[e] = e < N ? gamma[e] : 0.0f;
        sbt[e] = e < N ? beta[e] : 0.0f;
    }
    // head weights W_heads^T [208][8] (rows 5-7 and features past N zero) for the A fragments of
    // v_mfma_f32_16x16x4_f32: lane (f = l & 15, k = l >> 4) reads swh[k][16 n + f], swh[4 + k][..]
    float *swh = sbt + kLbPad;
    for (int e = tid; e < 8 * kLbPad; e += kLbThreads) {
        const int k = e / kLbPad, f = e - k * kLbPad;
        float v = 0.0f;
        if (HEAD && f < N) v = k < 4 ? src.wa[k * N + f] : (k == 4 && src.wv ? src.wv[f] : 0.0f);
        swh[e] = v;
    }
    __syncthreads();
    const Drop d = make_drop(da);
    constexpr float inv_h = 1.0f / (float)N;
    const bool lastok = 16 * (NT - 1) + 4 * gq < N;
    auto valid = [&](int n) { return n < NT - 1 || lastok; };
    char *orow = sO + col * 2 * N + 8 * gq;
    R::f32x2 ag[NT][2], ab[NT][2];
#pragma unroll
    for (int n = 0; n < NT; n++) ag[n][0] = ag[n][1] = ab[n][0] = ab[n][1] = R::f32x2{0.0f, 0.0f};
    const int64_t ntile = (m + 15) >> 4;
    for (int64_t tile = (int64_t)blockIdx.x * kLbWaves + wave; tile < ntile; tile += (int64_t)gridDim.x * kLbWaves) {
        const int64_t row = 16 * tile + col;
        const bool live = row < m;
        const int64_t rc = live ? row : 0;
        const int rows = (int)(m - 16 * tile < 16 ? m - 16 * tile : 16);
        uint2 gr[NT], pr[NP > 0 ? NP : 1][NT];
#pragma unroll
        for (int n = 0; n < NT; n++) {
            const int f0 = 16 * n + 4 * gq * valid(n);  // an invalid lane re-reads an in-row group
            gr[n] = *reinterpret_cast<const uint2 *>(g + rc * N + f0);
#pragma unroll
            for (int i = 0; i < NP; i++) pr[i][n] = *reinterpret_cast<const uint2 *>(src.p[i] + rc * N + f0);
        }
        const float mu = mean_in[rc], rs = rstd_in[rc];
        // heads' share, B: lane (k = l >> 4, j = l & 15) holds dz[16 t + j][k] (value column 4 for k == 0)
        const float b0 = HEAD ? src.dz[rc * 8 + gq] : 0.0f;
        const float b1 = (HEAD && gq == 0) ? src.dz[rc * 8 + 4] : 0.0f;
        // pass 1: dzr = dy * [z > 0] * keep, dgamma / dbeta accumulators, row sums
        R::f32x2 dzr[NT][2];
        R::f32x2 s1 = {0.0f, 0.0f}, s2 = {0.0f, 0.0f};
        const R::f32x2 nmu = {-mu, -mu}, rs2 = {rs, rs};
        uint4 dpair = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int n = 0; n < NT; n++) {
            const int f0 = 16 * n + 4 * gq;
            f32x4_t dy = {0.0f, 0.0f, 0.0f, 0.0f};
            if (HEAD) {
                dy = __builtin_amdgcn_mfma_f32_16x16x4f32(swh[gq * kLbPad + 16 * n + col], b0, dy, 0, 0, 0);
                dy = __builtin_amdgcn_mfma_f32_16x16x4f32(swh[(4 + gq) * kLbPad + 16 * n + col], b1, dy, 0, 0, 0);
            }
            float t[4] = {dy[0], dy[1], dy[2], dy[3]};
#pragma unroll
            for (int i = 0; i < NP; i++) {
                t[0] += R::bf_lo(pr[i][n].x);
                t[1] += R::bf_hi(pr[i][n].x);
                t[2] += R::bf_lo(pr[i][n].y);
                t[3] += R::bf_hi(pr[i][n].y);
            }
            const float4 gm = *reinterpret_cast<const float4 *>(sgm + f0);
            const float4 bt = *reinterpret_cast<const float4 *>(sbt + f0);
            const R::f32x2 xh0 = (R::f32x2{R::bf_lo(gr[n].x), R::bf_hi(gr[n].x)} + nmu) * rs2;
            const R::f32x2 xh1 = (R::f32x2{R::bf_lo(gr[n].y), R::bf_hi(gr[n].y)} + nmu) * rs2;
            const R::f32x2 z0 = R::fma2(xh0, R::f32x2{gm.x, gm.y}, R::f32x2{bt.x, bt.y});
            const R::f32x2 z1 = R::fma2(xh1, R::f32x2{gm.z, gm.w}, R::f32x2{bt.z, bt.w});
            const bool on = live && valid(n);
            float k[4] = {1.0f, 1.0f, 1.0f, 1.0f};
            if (DROP) {
                if ((n & 1) == 0) dpair = drop_draw4(d, (uint32_t)rc, (uint32_t)(f0 >> 2));
                drop_mult_bits(d, drop_half(dpair, (uint32_t)(f0 >> 2)), k);
            }
            const R::f32x2 d0 = {(on && z0.x > 0.0f) ? t[0] * k[0] : 0.0f, (on && z0.y > 0.0f) ? t[1] * k[1] : 0.0f};
            const R::f32x2 d1 = {(on && z1.x > 0.0f) ? t[2] * k[2] : 0.0f, (on && z1.y > 0.0f) ? t[3] * k[3] : 0.0f};
            dzr[n][0] = d0;
            dzr[n][1] = d1;
            ag[n][0] = R::fma2(d0, xh0, ag[n][0]);
            ag[n][1] = R::fma2(d1, xh1, ag[n][1]);
            ab[n][0] = ab[n][0] + d0;
            ab[n][1] = ab[n][1] + d1;
            const R::f32x2 x0 = d0 * R::f32x2{gm.x, gm.y}, x1 = d1 * R::f32x2{gm.z, gm.w};  // dxhat
            s1 = s1 + x0 + x1;
            s2 = R::fma2(x1, xh1, R::fma2(x0, xh0, s2));
        }
        const float m1 = R::xor32_add(R::xor16_add(s1.x + s1.y)) * inv_h;
        const float m2 = R::xor32_add(R::xor16_add(s2.x + s2.y)) * inv_h;
        // pass 2: dG = rstd (dxhat - mean(dxhat) - xhat mean(dxhat xhat)) into the LDS tile
        const R::f32x2 nm1 = {-m1, -m1}, nm2 = {-m2, -m2};
#pragma unroll
        for (int n = 0; n < NT; n++) {
            if (!valid(n)) continue;
            const int f0 = 16 * n + 4 * gq;
            const float4 gm = *reinterpret_cast<const float4 *>(sgm + f0);
            const R::f32x2 xh0 = (R::f32x2{R::bf_lo(gr[n].x), R::bf_hi(gr[n].x)} + nmu) * rs2;
            const R::f32x2 xh1 = (R::f32x2{R::bf_lo(gr[n].y), R::bf_hi(gr[n].y)} + nmu) * rs2;
            const R::f32x2 o0 = R::fma2(xh0, nm2, R::fma2(dzr[n][0], R::f32x2{gm.x, gm.y}, nm1)) * rs2;
            const R::f32x2 o1 = R::fma2(xh1, nm2, R::fma2(dzr[n][1], R::f32x2{gm.z, gm.w}, nm1)) * rs2;
            *reinterpret_cast<uint2 *>(orow + 32 * n) = make_uint2(R::pack_bf2(o0.x, o0.y), R::pack_bf2(o1.x, o1.y));
        }
        mw_flush(sO, dg + 16 * tile * N, rows, lane);
    }
    // dgamma / dbeta: the 16 rows of a lane group, then the block's waves (LDS), one partial row
    float *red = reinterpret_cast<float *>(sO);  // this wave's [2][208] (its output tile is drained)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int n = 0; n < NT; n++)
#pragma unroll
        for (int h2 = 0; h2 < 2; h2++) {
            const float a0 = row16_sum(ag[n][h2].x), a1 = row16_sum(ag[n][h2].y);
            const float b0 = row16_sum(ab[n][h2].x), b1 = row16_sum(ab[n][h2].y);
            if (col == 0) {
                const int f = 16 * n + 4 * gq + 2 * h2;
                red[f] = a0;
                red[f + 1] = a1;
                red[kLbPad + f] = b0;
                red[kLbPad + f + 1] = b1;
            }
        }
    __syncthreads();
    const int stride_w = (kMwOut > 4 * 2 * kLbPad ? kMwOut : 4 * 2 * kLbPad) / 4;  // floats between wave regions
    const float *red0 = reinterpret_cast<const float *>(smem + 4 * 10 * kLbPad);
    for (int c = tid; c < 2 * N; c += kLbThreads) {
        const int o = c < N ? c : kLbPad + (c - N);
        float t = 0.0f;
#pragma unroll
        for (int w = 0; w < kLbWaves; w++) t += red0[w * stride_w + o];
        part[(int64_t)blockIdx.x * 2 * N + c] = t;
    }
}

// ------------------------------------------------------------------ policy / value heads -----
// logits = x Wa^T + ba, value = x Wv^T + bv for the rollout policy (GameMLP.forward, game.py:
// 1208-1219): one v_mfma_f32_16x16x32_bf16 tile per 16 rows with the 5 head rows as the 16-wide
// N (columns 5..15 zero), head weights held as bf16 B fragments in registers for the whole launch.
template <int KS>
__global__ __launch_bounds__(256) void head_fwd_kernel(const uint16_t *__restrict__ X, const float *__restrict__ wa,
                                                       const float *__restrict__ ba, const float *__restrict__ wv,
                                                       const float *__restrict__ bv, int64_t M, int K,
                                                       float *__restrict__ logits, int64_t lstride,
                                                       float *__restrict__ value) {
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    bf16x8_t fb[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
        s16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int k = 32 * ks + 8 * g + j;
            const float wgt = (c < 5 && k < K) ? (c < 4 ? wa[c * K + k] : wv[k]) : 0.0f;
            v[j] = __builtin_bit_cast(short, (__bf16)wgt);
        }
        fb[ks] = __builtin_bit_cast(bf16x8_t, v);
    }
    const float bias = c < 4 ? ba[c] : (c == 4 ? bv[0] : 0.0f);
    const int64_t tiles = (M + 15) >> 4;
    for (int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); tile < tiles; tile += (int64_t)gridDim.x * 4) {
        const int64_t m0 = tile * 16, mr = m0 + c;
        bf16x8_t fa[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            const int kl = 32 * ks + 8 * g;
            uint4 w = make_uint4(0u, 0u, 0u, 0u);
            if (mr < M && kl < K) {
                const uint16_t *src = X + mr * K + kl;
                const uint2 lo = *reinterpret_cast<const uint2 *>(src);
                const uint2 hi = kl + 8 <= K ? *reinterpret_cast<const uint2 *>(src + 4) : make_uint2(0u, 0u);
                w = make_uint4(lo.x, lo.y, hi.x, hi.y);
            }
            fa[ks] = __builtin_bit_cast(bf16x8_t, w);
        }
        f32x4_t acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ks = 0; ks < KS; ks++) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks], fb[ks], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int64_t row = m0 + 4 * g + r;
            if (row >= M) continue;
            if (c < 4)
                logits[row * lstride + c] = acc[r] + bias;
            else if (c == 4)
                value[row] = acc[r] + bias;
        }
    }
}


// ------------------------------------------------------------------ minibatch statistics -----
// The per-minibatch accumulation of model_optimize_step's returned statistics (train.py:603-642)
// in one thread: stats[0..8] += {loss, policy_loss, entropy_loss, value_loss, grad_norm, entropy,
// kl_total, kl_average}, stats[8] = max(stats[8], kl_max); optionally bumps a device counter.
__global__ __launch_bounds__(256) void ppo_stats_kernel(const float *__restrict__ sums, const float *__restrict__ kl,
                                                        int kl_rows, const float *__restrict__ gn,
                                                        const float *__restrict__ beta, float critic, float m,
                                                        const int64_t *__restrict__ rows, float *__restrict__ stats,
                                                        uint64_t *__restrict__ counter) {
    __shared__ float red[2][256];
    float ks = 0.0f, km = -INFINITY;
    if (kl_rows > 0) {  // the KL kernel's partial rows: fixed-order sums
        for (int b = threadIdx.x; b < kl_rows; b += 256) {
            ks += kl[2 * b];
            km = fmaxf(km, kl[2 * b + 1]);
        }
        red[0][threadIdx.x] = ks;
        red[1][threadIdx.x] = km;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) {
                red[0][threadIdx.x] += red[0][threadIdx.x + w];
                red[1][threadIdx.x] = fmaxf(red[1][threadIdx.x], red[1][threadIdx.x + w]);
            }
            __syncthreads();
        }
        ks = red[0][0];
        km = red[1][0];
    } else {
        ks = kl[0];
        km = kl[1];
    }
    if (threadIdx.x != 0) return;
    if (rows) m = (float)max(*rows, (int64_t)1);
    const float s_ppo = sums[0] / m, s_ent = sums[1] / m, s_v = sums[2] / m, b = *beta;
    stats[0] += -(s_ppo - critic * s_v + b * s_ent);
    stats[1] += -s_ppo;
    stats[2] += -b * s_ent;
    stats[3] += critic * s_v;
    stats[4] += *gn;
    stats[5] += s_ent;
    stats[6] += ks;
    stats[7] += ks / m;
    stats[8] = fmaxf(stats[8], km);
    if (counter) *counter += 1ull;
}

// ------------------------------------------------------------------ column sums --------------
// Stage 1: grid (ceil(C/64), kSlices); block (64 columns x 4 row groups) sums rows of slice y.
constexpr int kSlices = 32;

__global__ __launch_bounds__(256) void colsum1_kernel(const float *__restrict__ part, int nb, int C,
                                                      float *__restrict__ part2, int max_col) {
    __shared__ float lds[4][64];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
    const int per = (nb + kSlices - 1) / kSlices;
    const int b0 = blockIdx.y * per, b1 = min(nb, b0 + per);
    float t = 0.0f, mx = -INFINITY;
    if (c < C)
        for (int b = b0 + rg; b < b1; b += 4) {
            const float v = part[(int64_t)b * C + c];
            t += v;
            mx = fmaxf(mx, v);
        }
    lds[rg][threadIdx.x & 63] = c == max_col ? mx : t;
    __syncthreads();
    if (rg == 0 && c < C) {
        const int l = threadIdx.x;
        part2[blockIdx.y * C + c] = c == max_col ? fmaxf(fmaxf(lds[0][l], lds[1][l]), fmaxf(lds[2][l], lds[3][l]))
                                                 : (lds[0][l] + lds[1][l]) + (lds[2][l] + lds[3][l]);
    }
}

struct Segs {
    float *dst[5];
    int len[5];
    int n;
};

__global__ __launch_bounds__(256) void colsum2_kernel(const float *__restrict__ part2, int C, Segs segs, int max_col) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    float t = 0.0f, mx = -INFINITY;
#pragma unroll 8
    for (int s = 0; s < kSlices; s++) {
        const float v = part2[s * C + c];
        t += v;
        mx = fmaxf(mx, v);
    }
    int off = 0;
    for (int k = 0; k < segs.n; k++) {
        if (c < off + segs.len[k]) {
            segs.dst[k][c - off] = c == max_col ? mx : t;
            return;
        }
        off += segs.len[k];
    }
}

// All deferred column sums in one launch: block = 64 columns x 16 row groups of one job (the job
// found from the block index); each thread sums its rows in order, then a fixed-order LDS combine.
static_assert(sizeof(g2048_colsum_job) == 88, "g2048_colsum_job layout (tests/test_abi.py)");
struct ColsumBatch {
    g2048_colsum_job job[G2048_COLSUM_MAX_JOBS];
    int first[G2048_COLSUM_MAX_JOBS + 1];
    int njobs;
    int nsq;      // sq: per-block sums of squares of the gradient segments (pad_ bit k: segment k)
    float *sq;
    float *tick;  // += 1 by block 0 (the optimizer's step count)
};

// a job whose partial rows are whole float2s runs 2 columns per lane (128 per block: 8-byte loads);
// every column is summed in the same order either way (rows rg, rg + 16, ... per group, then the
// 16 groups in order), so the two forms give the same bits.  (Round 6: 2 columns per lane, not 4 --
// the bench minibatch's 27.8 MB of partials then spread over 706 blocks instead of 353, i.e. ~2.8
// blocks per CU instead of 1 or 2.)
constexpr int kColsumW = 2;
__host__ __device__ inline bool colsum_vec(const g2048_colsum_job &jb) {
    return jb.cols % kColsumW == 0 && ((uintptr_t)jb.part % (4 * kColsumW)) == 0;
}

__global__ __launch_bounds__(1024) void colsum_batch_kernel(const ColsumBatch cb) {
    __shared__ float2 lds[16][64];
    int j = 0;
    while (j + 1 < cb.njobs && (int)blockIdx.x >= cb.first[j + 1]) j++;
    const g2048_colsum_job &jb = cb.job[j];
    const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const bool vec = colsum_vec(jb);  // block-uniform
    const int W = vec ? kColsumW : 1;
    const int c0 = ((int)blockIdx.x - cb.first[j]) * 64 * W + cl * W;
    float t[kColsumW];
#pragma unroll
    for (int u = 0; u < kColsumW; u++) t[u] = c0 + u == jb.max_col ? -INFINITY : 0.0f;
    if (c0 < jb.cols) {
        const float *p = jb.part + c0;
        if (vec) {
#pragma unroll 4
            for (int b = rg; b < jb.nb; b += 16) {
                const float2 v = *reinterpret_cast<const float2 *>(p + (int64_t)b * jb.cols);
                const float vv[kColsumW] = {v.x, v.y};
#pragma unroll
                for (int u = 0; u < kColsumW; u++) t[u] = c0 + u == jb.max_col ? fmaxf(t[u], vv[u]) : t[u] + vv[u];
            }
        } else {
#pragma unroll 4
            for (int b = rg; b < jb.nb; b += 16) {
                const float v = p[(int64_t)b * jb.cols];
                t[0] = c0 == jb.max_col ? fmaxf(t[0], v) : t[0] + v;
            }
        }
    }
    lds[rg][cl] = make_float2(t[0], t[1]);
    __syncthreads();
    if (cb.sq) {  // block 0: the step count and the zero tail of the partials
        if (blockIdx.x == 0 && threadIdx.x == 0 && cb.tick) *cb.tick += 1.0f;
        if (blockIdx.x == 0)
            for (int b = (int)gridDim.x + (int)threadIdx.x; b < cb.nsq; b += 1024) cb.sq[b] = 0.0f;
    }
    if (rg != 0) return;
    if (c0 >= jb.cols) {
        if (cb.sq) {  // this wave still joins the block's sum of squares
            float z = 0.0f;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) z += __shfl_xor(z, o);
            if (cl == 0) cb.sq[blockIdx.x] = z;
        }
        return;
    }
    float acc[kColsumW];
    {
        const float2 a0 = lds[0][cl];
        acc[0] = a0.x;
        acc[1] = a0.y;
    }
#pragma unroll
    for (int g = 1; g < 16; g++) {
        const float2 a = lds[g][cl];
        const float av[kColsumW] = {a.x, a.y};
#pragma unroll
        for (int u = 0; u < kColsumW; u++) acc[u] = c0 + u == jb.max_col ? fmaxf(acc[u], av[u]) : acc[u] + av[u];
    }
    float ss = 0.0f;
    for (int u = 0; u < W; u++) {
        const int c = c0 + u;
        if (c >= jb.cols) break;
        int off = 0;
        for (int k = 0; k < jb.nseg; k++) {
            if (c < off + jb.len[k]) {
                jb.dst[k][c - off] = acc[u];
                if ((jb.pad_ >> k) & 1) ss += acc[u] * acc[u];
                break;
            }
            off += jb.len[k];
        }
    }
    if (cb.sq) {  // rg == 0: one wave holds the block's outputs
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
        if (cl == 0) cb.sq[blockIdx.x] = ss;
    }
}

__global__ __launch_bounds__(256) void dropout_mask_kernel(int64_t m, int h, DropArgs da, uint8_t *__restrict__ mask) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int groups = h / 4;
    if (q >= m * groups) return;
    const int64_t r = q / groups;
    const int cg = (int)(q - r * groups);
    const Drop d = make_drop(da);
    float k[4];
    drop_mult(d, (uint32_t)r, (uint32_t)cg, k);
    for (int u = 0; u < 4; u++) mask[r * h + 4 * cg + u] = k[u] != 0.0f ? 1 : 0;
}

// ------------------------------------------------------------------ host helpers -------------
inline int status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}

inline bool shape_ok(int64_t m, int32_t h) { return m >= 0 && h > 0 && h % 4 == 0 && h <= 1024 && m < (1ll << 31); }

inline bool al(const void *p, unsigned a) { return ((uintptr_t)p % a) == 0u; }

// blocks of the head kernels: one 64-row group per wave and step, <= 256 blocks (<= partial_blocks)
inline int head_blocks(int64_t m) {
    const int64_t b = (m + 64 * kWaves - 1) / (64 * kWaves);
    return (int)(b < 1 ? 1 : (b > 256 ? 256 : b));
}

// blocks of ln_bwd: 1024 threads, >= 4 rows per wave, <= 256 blocks (<= partial_blocks)
inline int bwd_blocks(int64_t m) {
    const int64_t b = (m + 4 * kBwdWaves - 1) / (4 * kBwdWaves);
    return (int)(b < 1 ? 1 : (b > 256 ? 256 : b));
}

// blocks of a partial-producing kernel: >= 4 rows per wave, <= 2048 blocks
inline int partial_blocks(int64_t m) {
    const int64_t b = (m + 4 * kWaves - 1) / (4 * kWaves);
    return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

int colsum(hipStream_t s, const float *part, int nb, int C, float *scratch2, const Segs &segs, int max_col,
           g2048_colsum_job *defer = nullptr) {
    if (defer) {  // described, summed later by g2048_colsum_batch
        *defer = g2048_colsum_job{};
        defer->part = part;
        defer->nb = nb;
        defer->cols = C;
        defer->max_col = max_col;
        defer->nseg = segs.n;
        for (int k = 0; k < segs.n; k++) {
            defer->dst[k] = segs.dst[k];
            defer->len[k] = segs.len[k];
        }
        return status();
    }
    hipLaunchKernelGGL(colsum1_kernel, dim3((C + 63) / 64, kSlices), dim3(256), 0, s, part, nb, C, scratch2, max_col);
    hipLaunchKernelGGL(colsum2_kernel, dim3((C + 255) / 256), dim3(256), 0, s, scratch2, C, segs, max_col);
    return status();
}


// weight-gradient launch geometry
struct WgPlan {
    int bi, bj, wi, nb, pa, pb, bw, ny;
    int64_t rows;
    size_t lds;
};

inline int wg_pitch(int n) {  // LDS row bytes: >= 2 * pad16(n) and == 32 (mod 256)
    const int b = ((n + 15) / 16) * 32;
    return b + (((32 - b) % 256) + 256) % 256;
}

inline bool wg_plan(int64_t m, int n1, int n2, WgPlan &p, int64_t rows_target = 512) {
    if (n1 <= 0 || n2 <= 0 || n1 % 4 || n2 % 4 || n1 > 224 || n2 > 224 || m <= 0) return false;
    const int TI = (n1 + 15) / 16, TJ0 = (n2 + 15) / 16;
    // split the output columns into ny bands of whole 16-column tiles when there are enough
    // tiles: twice the blocks, each staging its band of B only
    const int ny = TJ0 >= 4 ? 2 : 1;
    const int TJ = (TJ0 + ny - 1) / ny;
    static const int menu[3][2] = {{2, 2}, {4, 4}, {7, 4}};  // n <= 224: TI <= 14, TJ <= 7 after the split
    static const int arr[3][2] = {{2, 2}, {4, 1}, {1, 4}};
    for (auto &mb : menu)
        for (auto &a : arr)
            if (a[0] * mb[0] >= TI && a[1] * mb[1] >= TJ) {
                p.bi = mb[0];
                p.bj = mb[1];
                p.wi = a[0];
                p.ny = ny;
                p.bw = 16 * TJ;
                int64_t nb = m / rows_target;
                nb = nb < 1 ? 1 : (nb > 256 ? 256 : nb);
                int64_t rows = (m + nb - 1) / nb;
                rows = (rows + kWgRows - 1) / kWgRows * kWgRows;
                p.nb = (int)((m + rows - 1) / rows);
                p.rows = rows;
                p.pa = wg_pitch(n1);
                p.pb = wg_pitch(p.bw < n2 ? p.bw : n2);
                p.lds = (size_t)2 * kWgRows * (p.pa + p.pb);
                return true;
            }
    return false;
}

#define G2048_DISPATCH_J(h, BODY)            \
    do {                                     \
        const int jj_ = ((h) + 255) / 256;  \
        if (jj_ == 1) { constexpr int J = 1; BODY; } \
        else if (jj_ == 2) { constexpr int J = 2; BODY; } \
        else if (jj_ == 3) { constexpr int J = 3; BODY; } \
        else { constexpr int J = 4; BODY; }  \
    } while (0)

}  // namespace

// ------------------------------------------------------------------ input gradient -----------
// P = dG W  (the Linear input gradient, dG bf16 [m, n], W bf16 [n, k] = the layer weight [out, in],
// P bf16 [m, k]) on bf16 MFMA in the forward kernels' orientation: P^T = W^T dG^T, so a lane's B
// fragment is 16 contiguous bytes of one dG row and its result is 4 consecutive columns of one P
// row (one 8-byte store).  W^T is staged once per block into LDS with a row pitch of 16 KS + 4
// dwords (4 (4KS + 1), 4KS + 1 odd): the 16 rows a fragment read touches start on 16 distinct
// 4-bank groups, so the ds_read_b128 of a wave is conflict-free.  A wave owns 32 rows of dG (two
// B-fragment sets), so every W^T fragment read feeds two MFMAs.  KS = ceil(n / 32) k-steps,
// CT = ceil(k / 16) output column tiles; m unbounded (persistent over row blocks).
constexpr int kDgThreads = 512;

template <int KS, int CT, int NH>  // NH 16-row halves of dG per wave (2 while the accumulators fit)
__global__ __launch_bounds__(kDgThreads) void dgrad_kernel(const uint16_t *__restrict__ dg,
                                                           const uint16_t *__restrict__ w,
                                                           uint16_t *__restrict__ out, int64_t m, int n, int k) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int kPitch = 32 * KS + 8;  // bf16 elements per W^T row (16 KS + 4 dwords)
    constexpr int kRowsT = 16 * CT;
    uint16_t *wt = reinterpret_cast<uint16_t *>(smem);
    const int tid = threadIdx.x;
    // zero the padding (rows c >= k, columns j >= n), then W^T[c][j] = W[j][c] from 8-byte reads of
    // W rows (k % 4 == 0), all of a thread's reads issued before its LDS writes
    for (int e = tid; e < kRowsT * kPitch / 8; e += kDgThreads) reinterpret_cast<uint4 *>(smem)[e] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    {
        const int k4 = k >> 2, total = n * k4;
        constexpr int kU = 8;
        for (int e0 = tid; e0 < total; e0 += kU * kDgThreads) {
            uint2 v[kU];
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int e = e0 + u * kDgThreads;
                v[u] = e < total ? reinterpret_cast<const uint2 *>(w)[e] : make_uint2(0u, 0u);
            }
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int e = e0 + u * kDgThreads;
                if (e >= total) break;
                const int j = e / k4, c = 4 * (e - j * k4);
                wt[(c + 0) * kPitch + j] = (uint16_t)(v[u].x & 0xFFFFu);
                wt[(c + 1) * kPitch + j] = (uint16_t)(v[u].x >> 16);
                wt[(c + 2) * kPitch + j] = (uint16_t)(v[u].y & 0xFFFFu);
                wt[(c + 3) * kPitch + j] = (uint16_t)(v[u].y >> 16);
            }
        }
    }
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6, rt = lane & 15, g = lane >> 4;
    const int64_t stride = (int64_t)gridDim.x * (kDgThreads / 64) * 16 * NH;
    for (int64_t rb = ((int64_t)blockIdx.x * (kDgThreads / 64) + wave) * 16 * NH; rb < m; rb += stride) {
        bf16x8_t fb[NH][KS];
#pragma unroll
        for (int h = 0; h < NH; h++) {
            const int64_t r = rb + 16 * h + rt;
            const uint16_t *row = dg + (r < m ? r : 0) * (int64_t)n;
#pragma unroll
            for (int s = 0; s < KS; s++) {
                const int kk = 32 * s + 8 * g;
                uint4 v = make_uint4(0u, 0u, 0u, 0u);
                if (r < m) {
                    if (kk + 8 <= n) {
                        v = *reinterpret_cast<const uint4 *>(row + kk);
                    } else if (kk < n) {  // n % 4 == 0: a 4-element tail
                        const uint2 t = *reinterpret_cast<const uint2 *>(row + kk);
                        v = make_uint4(t.x, t.y, 0u, 0u);
                    }
                }
                fb[h][s] = __builtin_bit_cast(bf16x8_t, v);
            }
        }
        f32x4_t acc[NH][CT];
#pragma unroll
        for (int h = 0; h < NH; h++)
#pragma unroll
            for (int ct = 0; ct < CT; ct++) acc[h][ct] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
        // W^T fragments one column tile ahead of the MFMAs; the empty asm with a memory clobber keeps
        // the compiler from hoisting every tile's LDS reads to the top (which spills)
        const char *base = smem + (rt * kPitch + 8 * g) * 2;
        bf16x8_t fa[2][KS];
#pragma unroll
        for (int s = 0; s < KS; s++) fa[0][s] = *reinterpret_cast<const bf16x8_t *>(base + 64 * s);
#pragma unroll
        for (int ct = 0; ct < CT; ct++) {
            if (ct + 1 < CT) {
#pragma unroll
                for (int s = 0; s < KS; s++)
                    fa[(ct + 1) & 1][s] = *reinterpret_cast<const bf16x8_t *>(base + (16 * (ct + 1) * kPitch) * 2 + 64 * s);
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int s = 0; s < KS; s++)
#pragma unroll
                for (int h = 0; h < NH; h++)
                    acc[h][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ct & 1][s], fb[h][s], acc[h][ct], 0, 0, 0);
        }
        // lane (col = row rt of half h, rows 4g .. 4g+3 of tile ct): P[r][16 ct + 4g .. +3]
#pragma unroll
        for (int h = 0; h < NH; h++) {
            const int64_t r = rb + 16 * h + rt;
            if (r >= m) continue;
            uint16_t *orow = out + r * (int64_t)k;
#pragma unroll
            for (int ct = 0; ct < CT; ct++) {
                const int c = 16 * ct + 4 * g;
                if (c < k)
                    *reinterpret_cast<uint2 *>(orow + c) = make_uint2(pack_bf2(acc[h][ct][0], acc[h][ct][1]),
                                                                     pack_bf2(acc[h][ct][2], acc[h][ct][3]));
            }
        }
    }
}

template <int KS, int CT, int NH>
int launch_dgrad(hipStream_t s, const uint16_t *dg, const uint16_t *w, uint16_t *out, int64_t m, int n, int k) {
    const size_t lds = (size_t)16 * CT * (32 * KS + 8) * 2;
    const int64_t rows_per_block = (kDgThreads / 64) * 16 * NH;
    int64_t blocks = (m + rows_per_block - 1) / rows_per_block;
    blocks = blocks > 256 ? 256 : blocks;  // persistent: one block per CU holds W^T
    hipLaunchKernelGGL((dgrad_kernel<KS, CT, NH>), dim3((unsigned)blocks), dim3(kDgThreads), lds, s, dg, w, out, m, n, k);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : (int)e;
}

extern "C" {

int g2048_obs_gather(g2048_stream_t stream, const int8_t *boards, const int64_t *idx, int64_t m, uint16_t *obs) {
    if (m < 0 || (m > 0 && (!boards || !idx || !obs || !al(obs, 8)))) return G2048_EINVAL;
    if (m == 0) return G2048_OK;
    hipLaunchKernelGGL(obs_gather_kernel, dim3((unsigned)((m * 12 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       boards, idx, obs, m);
    return status();
}

int g2048_ln_act_fwd(g2048_stream_t stream, const uint16_t *g, const float *gamma, const float *beta,
                     const uint16_t *res, uint16_t *y, float *mean, float *rstd, int64_t m, int32_t h,
                     const g2048_dropout *drop) {
    if (!shape_ok(m, h)) return G2048_EINVAL;
    if (m == 0) return G2048_OK;
    if (!g || !gamma || !beta || !y || !mean || !rstd || !al(g, 8) || !al(y, 8) || (res && !al(res, 8)))
        return G2048_EINVAL;
    const DropArgs da = drop_args(drop);
    const int64_t blocks64 = (m + kWaves * kFwdRows - 1) / (kWaves * kFwdRows);
    const dim3 grid((unsigned)(blocks64 > 2048 ? 2048 : blocks64)), blk(kThreads);
    const hipStream_t s = (hipStream_t)stream;
    if (drop_on(drop))
        G2048_DISPATCH_J(h, hipLaunchKernelGGL((ln_fwd_kernel<J, true>), grid, blk, 0, s, g, gamma, beta, res, y, mean,
                                               rstd, m, h, da));
    else
        G2048_DISPATCH_J(h, hipLaunchKernelGGL((ln_fwd_kernel<J, false>), grid, blk, 0, s, g, gamma, beta, res, y,
                                               mean, rstd, m, h, da));
    return status();
}

size_t g2048_ln_act_bwd_partials(int64_t m, int32_t h) {
    if (!shape_ok(m, h)) return 0;
    return (size_t)partial_blocks(m) * 2 * h + (size_t)kSlices * 2 * h;
}

int g2048_ln_act_bwd(g2048_stream_t stream, const g2048_dy *dy, const uint16_t *g, const float *mean,
                     const float *rstd, const float *gamma, const float *beta, uint16_t *dg, float *dres_out,
                     float *partials, float *dgamma, float *dbeta, int64_t m, int32_t h, const g2048_dropout *drop,
                     g2048_colsum_job *defer) {
    if (!shape_ok(m, h) || !dy) return G2048_EINVAL;
    if (!g || !mean || !rstd || !gamma || !beta || !dg || !partials || !dgamma || !dbeta) return G2048_EINVAL;
    if (!al(g, 8) || !al(dg, 8) || (dy->dres && !al(dy->dres, 16)) || (dres_out && !al(dres_out, 16)))
        return G2048_EINVAL;
    DySrc src{};
    src.dres = dy->dres;
    for (int i = 0; i < G2048_DY_MAX_P; i++) {
        if (!dy->p[i]) continue;  // the non-NULL entries, packed
        if (!al(dy->p[i], 8)) return G2048_EINVAL;
        src.p[src.np++] = dy->p[i];
    }
    const bool head = dy->dz != nullptr;
    if (head && (!dy->wa || !al(dy->dz, 16))) return G2048_EINVAL;
    src.dz = dy->dz;
    src.wa = dy->wa;
    src.wv = dy->wv;
    const hipStream_t s = (hipStream_t)stream;
    if (m == 0) {
        if (defer) *defer = g2048_colsum_job{};  // an empty job: g2048_colsum_batch skips it
        (void)hipMemsetAsync(dgamma, 0, sizeof(float) * h, s);
        (void)hipMemsetAsync(dbeta, 0, sizeof(float) * h, s);
        return status();
    }
    const DropArgs da = drop_args(drop);
    if (h == kMwN && src.np <= 2 && !src.dres && !dres_out && al(dg, 16)) {  // the h = 196 tile kernel
        const int64_t nwg = ((m + 15) / 16 + kLbWaves - 1) / kLbWaves;
        int nb = (int)(nwg < 256 ? nwg : 256);
        nb = nb < partial_blocks(m) ? nb : partial_blocks(m);
        const size_t lds = lb_lds_bytes();
#define G2048_LB196(D_, H_, P_)                                                                                    \
    hipLaunchKernelGGL((ln_bwd196_kernel<D_, H_, P_>), dim3(nb), dim3(kLbThreads), lds, s, src, g, mean, rstd, gamma, \
                       beta, dg, partials, m, da)
#define G2048_LB196_P(D_, H_)                        \
    do {                                             \
        if (src.np == 0) G2048_LB196(D_, H_, 0);     \
        else if (src.np == 1) G2048_LB196(D_, H_, 1); \
        else G2048_LB196(D_, H_, 2);                 \
    } while (0)
        if (drop_on(drop)) {
            if (head) G2048_LB196_P(true, true);
            else G2048_LB196_P(true, false);
        } else {
            if (head) G2048_LB196_P(false, true);
            else G2048_LB196_P(false, false);
        }
#undef G2048_LB196_P
#undef G2048_LB196
        Segs segs{};
        segs.n = 2;
        segs.dst[0] = dgamma;
        segs.len[0] = h;
        segs.dst[1] = dbeta;
        segs.len[1] = h;
        return colsum(s, partials, nb, 2 * h, partials + (size_t)nb * 2 * h, segs, -1, defer);
    }
    const int nb = bwd_blocks(m);
    const size_t lds = sizeof(float) * kBwdWaves * 2 * h;
#define G2048_LB(D_, H_)                                                                                             \
    G2048_DISPATCH_J(h, hipLaunchKernelGGL((ln_bwd_kernel<J, D_, H_>), dim3(nb), dim3(kBwdThreads), lds, s, src, g, \
                                           mean, rstd, gamma, beta, dg, dres_out, partials, m, h, da))
    if (drop_on(drop)) {
        if (head) G2048_LB(true, true);
        else G2048_LB(true, false);
    } else {
        if (head) G2048_LB(false, true);
        else G2048_LB(false, false);
    }
#undef G2048_LB
    Segs segs{};
    segs.n = 2;
    segs.dst[0] = dgamma;
    segs.len[0] = h;
    segs.dst[1] = dbeta;
    segs.len[1] = h;
    return colsum(s, partials, nb, 2 * h, partials + (size_t)nb * 2 * h, segs, -1, defer);
}

size_t g2048_ppo_head_partials(int64_t m, int32_t h) {
    if (!shape_ok(m, h)) return 0;
    return (size_t)partial_blocks(m) * (5 * h + 8) + (size_t)kSlices * (5 * h + 8);
}

int g2048_ppo_head_loss(g2048_stream_t stream, const uint16_t *x, const float *wa, const float *ba, const float *wv,
                        const float *bv, int64_t m, int32_t h, const g2048_ppo_batch *batch, const float *beta_dev,
                        float critic, float clip_eps, int32_t decouple_critic, float *masked, float *dx, float *dz,
                        float *partials, float *dwa, float *dba, float *dwv, float *dbv, float *sums,
                        g2048_colsum_job *defer) {
    if (!shape_ok(m, h) || m == 0 || !batch) return G2048_EINVAL;
    if (!x || !wa || !ba || !wv || !bv || !beta_dev || !masked || (!dx && !dz) || !partials || !dwa || !dba || !dwv ||
        !dbv || !sums || !batch->idx || !batch->action || !batch->legal || !batch->old_logp || !batch->adv ||
        !batch->ret)
        return G2048_EINVAL;
    if (!al(x, 8) || !al(masked, 16) || (dx && !al(dx, 16)) || (dz && !al(dz, 16))) return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    HeadLossArgs a{batch->idx, batch->action, batch->legal, batch->old_logp, batch->adv, batch->ret, beta_dev,
                   batch->rows, critic, 1.0f - clip_eps, 1.0f + clip_eps, 1.0f / (float)m, decouple_critic};
    const int nb = head_blocks(m);
    const int C = 5 * h + 8;
    const size_t red = sizeof(float) * kWaves * C, img = (size_t)kWaves * 128 * h;
    const size_t lds = h <= 256 && img > red ? img : red;
    // h <= 256: J = 1 and all KS = ceil(h/32) k-steps of the heads in registers; wider: 256-column chunks
#define G2048_HL(J_, KS_, MULTI_)                                                                                  \
    do {                                                                                                          \
        if (dx)                                                                                                   \
            hipLaunchKernelGGL((head_loss_kernel<J_, KS_, MULTI_, true>), dim3(nb), dim3(kThreads), lds, s, x, wa, \
                               ba, wv, bv, m, h, a, masked, dx, dz, partials);                                    \
        else                                                                                                      \
            hipLaunchKernelGGL((head_loss_kernel<J_, KS_, MULTI_, false>), dim3(nb), dim3(kThreads), lds, s, x, wa, \
                               ba, wv, bv, m, h, a, masked, dx, dz, partials);                                    \
    } while (0)
    switch ((h + 31) / 32) {
        case 1: G2048_HL(1, 1, false); break;
        case 2: G2048_HL(1, 2, false); break;
        case 3: G2048_HL(1, 3, false); break;
        case 4: G2048_HL(1, 4, false); break;
        case 5: G2048_HL(1, 5, false); break;
        case 6: G2048_HL(1, 6, false); break;
        case 7: G2048_HL(1, 7, false); break;
        case 8: G2048_HL(1, 8, false); break;
        default:
            if (h <= 512) G2048_HL(2, 8, true);
            else if (h <= 768) G2048_HL(3, 8, true);
            else G2048_HL(4, 8, true);
            break;
    }
#undef G2048_HL
    Segs segs{};
    segs.n = 5;
    segs.dst[0] = dwa; segs.len[0] = 4 * h;
    segs.dst[1] = dwv; segs.len[1] = h;
    segs.dst[2] = dba; segs.len[2] = 4;
    segs.dst[3] = dbv; segs.len[3] = 1;
    segs.dst[4] = sums; segs.len[4] = 3;
    return colsum(s, partials, nb, C, partials + (size_t)nb * C, segs, -1, defer);
}

int g2048_ppo_head_kl(g2048_stream_t stream, const uint16_t *x, const float *wa, const float *ba, int64_t m,
                      int32_t h, const float *old_masked, const int64_t *rows, float *partials, float *out,
                      g2048_colsum_job *defer) {
    if (!shape_ok(m, h) || m == 0 || !x || !wa || !ba || !old_masked || !partials || !out) return G2048_EINVAL;
    if (!al(x, 8) || !al(old_masked, 16)) return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    const int nb = head_blocks(m);
    switch ((h + 31) / 32) {
#define G2048_HK(KS_, MULTI_) \
    hipLaunchKernelGGL((head_kl_kernel<KS_, MULTI_>), dim3(nb), dim3(kThreads), 0, s, x, wa, ba, m, h, old_masked, rows, \
                       partials)
        case 1: G2048_HK(1, false); break;
        case 2: G2048_HK(2, false); break;
        case 3: G2048_HK(3, false); break;
        case 4: G2048_HK(4, false); break;
        case 5: G2048_HK(5, false); break;
        case 6: G2048_HK(6, false); break;
        case 7: G2048_HK(7, false); break;
        case 8: G2048_HK(8, false); break;
        default: G2048_HK(8, true); break;
#undef G2048_HK
    }
    Segs segs{};
    segs.n = 1;
    segs.dst[0] = out;
    segs.len[0] = 2;
    return colsum(s, partials, nb, 2, partials + (size_t)nb * 2, segs, 1, defer);
}


size_t g2048_wgrad_partials(int64_t m, int32_t n1, int32_t n2) {
    WgPlan p;
    if (!wg_plan(m, n1, n2, p)) return 0;
    return (size_t)p.nb * n1 * n2 + (size_t)kSlices * n1 * n2;
}

// one launch of wgrad_kernel for plan p (nz = 2: the pair (a, b) and (a2, b2))
static int wg_launch(hipStream_t s, const WgPlan &p, int nz, const uint16_t *a, const uint16_t *b, float *part,
                     const uint16_t *a2, const uint16_t *b2, float *part2, int64_t m, int n1, int n2) {
    const dim3 grid(p.nb, p.ny, nz), blk(kWgThreads);
    if (p.bi == 2)
        hipLaunchKernelGGL((wgrad_kernel<2, 2>), grid, blk, p.lds, s, a, b, m, n1, n2, p.pa, p.pb, p.wi, p.rows, p.bw,
                           part, a2, b2, part2);
    else if (p.bi == 4)
        hipLaunchKernelGGL((wgrad_kernel<4, 4>), grid, blk, p.lds, s, a, b, m, n1, n2, p.pa, p.pb, p.wi, p.rows, p.bw,
                           part, a2, b2, part2);
    else if (p.wi == 2 && !getenv("G2048_WGRAD_NW4")) {  // 2 x 2 blocks of 7 x 4 tiles: the k-split 8-wave kernel
        const size_t lds = p.lds > wg_combine_bytes(7, 4) ? p.lds : wg_combine_bytes(7, 4);
        hipLaunchKernelGGL((wgrad_kernel<7, 4, 8>), grid, dim3(512), lds, s, a, b, m, n1, n2, p.pa, p.pb, p.wi, p.rows,
                           p.bw, part, a2, b2, part2);
    } else
        hipLaunchKernelGGL((wgrad_kernel<7, 4>), grid, blk, p.lds, s, a, b, m, n1, n2, p.pa, p.pb, p.wi, p.rows, p.bw,
                           part, a2, b2, part2);
    return status();
}

int g2048_wgrad(g2048_stream_t stream, const uint16_t *a, const uint16_t *b, int64_t m, int32_t n1, int32_t n2,
                float *partials, float *out, g2048_colsum_job *defer) {
    WgPlan p;
    if (!a || !b || !partials || !out || !al(a, 8) || !al(b, 8)) return G2048_EINVAL;
    if (!wg_plan(m, n1, n2, p)) return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    const int st = wg_launch(s, p, 1, a, b, partials, nullptr, nullptr, nullptr, m, n1, n2);
    if (st) return st;
    Segs segs{};
    segs.n = 1;
    segs.dst[0] = out;
    segs.len[0] = n1 * n2;
    return colsum(s, partials, p.nb, n1 * n2, partials + (size_t)p.nb * n1 * n2, segs, -1, defer);
}

size_t g2048_wgrad_pair_partials(int64_t m, int32_t n1, int32_t n2) {
    WgPlan p;
    if (!wg_plan(m, n1, n2, p, 1024)) return 0;
    return (size_t)p.nb * n1 * n2 + (size_t)kSlices * n1 * n2;
}

int g2048_wgrad_pair(g2048_stream_t stream, const uint16_t *a0, const uint16_t *b0, const uint16_t *a1,
                     const uint16_t *b1, int64_t m, int32_t n1, int32_t n2, float *partials0, float *partials1,
                     float *out0, float *out1, g2048_colsum_job *defer) {
    WgPlan p;
    if (!a0 || !b0 || !a1 || !b1 || !partials0 || !partials1 || !out0 || !out1 || !al(a0, 8) || !al(b0, 8) ||
        !al(a1, 8) || !al(b1, 8))
        return G2048_EINVAL;
    if (!wg_plan(m, n1, n2, p, 1024)) return G2048_EINVAL;  // twice the rows per block: half the partial rows
    const hipStream_t s = (hipStream_t)stream;
    const int st = wg_launch(s, p, 2, a0, b0, partials0, a1, b1, partials1, m, n1, n2);
    if (st) return st;
    float *part[2] = {partials0, partials1}, *out[2] = {out0, out1};
    for (int k = 0; k < 2; k++) {
        Segs segs{};
        segs.n = 1;
        segs.dst[0] = out[k];
        segs.len[0] = n1 * n2;
        const int rc = colsum(s, part[k], p.nb, n1 * n2, part[k] + (size_t)p.nb * n1 * n2, segs, -1,
                              defer ? defer + k : nullptr);
        if (rc) return rc;
    }
    return G2048_OK;
}


size_t g2048_mlp_fwd_lds_bytes(int32_t n, int32_t k) {
    if (n <= 0 || k <= 0 || n > 256 || k > 256 || n % 4 || k % 4) return 0;
    const int kp = (k + 7) & ~7, pw = mf_pitch(kp);
    const size_t b = (size_t)((n * pw + 15) & ~15) + (size_t)2 * kMfRows * pw + 64 + (size_t)8 * n;
    return b <= 160 * 1024 ? b : 0;
}

// the fixed-shape fast path of mlp_fwd_kernel: the h = 196 model's blocks (KS = 7) and stem (KS = 2)
static size_t mf_fixed_lds(int n, int ks) {
    const int pw = mf_fixed_pitch(ks);
    return (size_t)((16 * 13 * pw + 15) & ~15) + (size_t)2 * kMfRows * pw + 64 + (size_t)8 * n;
}
static int mf_fixed_ks(int n, int k) {
    if ((n + 15) / 16 != 13) return 0;
    const int ks = (((k + 7) & ~7) + 31) / 32;
    if (ks != 7 && ks != 2) return 0;
    return mf_fixed_lds(n, ks) <= 160 * 1024 ? ks : 0;
}

int g2048_mlp_fwd(g2048_stream_t stream, const uint16_t *x, const uint16_t *w, const float *gamma, const float *beta,
                  int32_t residual, uint16_t *g, uint16_t *y, float *mean, float *rstd, int64_t m, int32_t n, int32_t k,
                  const g2048_dropout *drop) {
    const size_t lds_generic = g2048_mlp_fwd_lds_bytes(n, k);
    if (!lds_generic || m < 0 || !x || !w || !gamma || !beta || !y || (!mean) != (!rstd)) return G2048_EINVAL;
    const int fks = mf_fixed_ks(n, k);
    const size_t lds = fks ? mf_fixed_lds(n, fks) : lds_generic;
    if (residual && n != k) return G2048_EINVAL;
    if (!al(x, 8) || !al(w, 8) || (g && !al(g, 8)) || !al(y, 8) || !al(gamma, 16) || !al(beta, 16)) return G2048_EINVAL;
    if (m == 0) return G2048_OK;
    const hipStream_t s = (hipStream_t)stream;
    const DropArgs da = drop_args(drop);
    const int64_t nslab = (m + kMfRows - 1) / kMfRows;
    const dim3 grid((unsigned)(nslab > 256 ? 256 : nslab)), blk(kMfThreads);  // one persistent block per CU
    const bool dr = drop_on(drop);
    const int nt = (n + 15) / 16;
#define G2048_MF_LAUNCH_KS(NT_, KS_)                                                                               \
    do {                                                                                                           \
        if (residual && dr)                                                                                        \
            hipLaunchKernelGGL((mlp_fwd_kernel<NT_, KS_, true, true>), grid, blk, lds, s, x, w, gamma, beta, g, y,  \
                               mean, rstd, m, n, k, da);                                                           \
        else if (residual)                                                                                         \
            hipLaunchKernelGGL((mlp_fwd_kernel<NT_, KS_, true, false>), grid, blk, lds, s, x, w, gamma, beta, g, y, \
                               mean, rstd, m, n, k, da);                                                           \
        else if (dr)                                                                                               \
            hipLaunchKernelGGL((mlp_fwd_kernel<NT_, KS_, false, true>), grid, blk, lds, s, x, w, gamma, beta, g, y, \
                               mean, rstd, m, n, k, da);                                                           \
        else                                                                                                       \
            hipLaunchKernelGGL((mlp_fwd_kernel<NT_, KS_, false, false>), grid, blk, lds, s, x, w, gamma, beta, g,   \
                               y, mean, rstd, m, n, k, da);                                                        \
    } while (0)
#define G2048_MF_LAUNCH(NT_) G2048_MF_LAUNCH_KS(NT_, 0)
    // the h = 196 shapes: mlp_fwd_wide_kernel (W-only LDS, 8 waves); G2048_MLP_FWD_SLAB set in the
    // environment selects the slab kernel instead (bitwise the same outputs: A/B timing and tests)
    if (n == kMwN && (k == kMwN || k == 48) && al(y, 16) && (!g || al(g, 16)) && !getenv("G2048_MLP_FWD_SLAB")) {
        const int64_t ntile = (m + 15) / 16, nwg = (ntile + kMwWaves - 1) / kMwWaves;
        const dim3 wgrid((unsigned)(nwg > 256 ? 256 : nwg)), wblk(kMwThreads);
#define G2048_MW_LAUNCH(K_)                                                                                      \
    do {                                                                                                         \
        const size_t wl = mw_lds_bytes(K_);                                                                      \
        if (residual && dr)                                                                                      \
            hipLaunchKernelGGL((mlp_fwd_wide_kernel<K_, true, true>), wgrid, wblk, wl, s, x, w, gamma, beta, g, y, \
                               mean, rstd, m, da);                                                               \
        else if (residual)                                                                                       \
            hipLaunchKernelGGL((mlp_fwd_wide_kernel<K_, true, false>), wgrid, wblk, wl, s, x, w, gamma, beta, g,  \
                               y, mean, rstd, m, da);                                                            \
        else if (dr)                                                                                             \
            hipLaunchKernelGGL((mlp_fwd_wide_kernel<K_, false, true>), wgrid, wblk, wl, s, x, w, gamma, beta, g,  \
                               y, mean, rstd, m, da);                                                            \
        else                                                                                                     \
            hipLaunchKernelGGL((mlp_fwd_wide_kernel<K_, false, false>), wgrid, wblk, wl, s, x, w, gamma, beta, g, \
                               y, mean, rstd, m, da);                                                            \
    } while (0)
        if (k == kMwN) G2048_MW_LAUNCH(kMwN);
        else G2048_MW_LAUNCH(48);
#undef G2048_MW_LAUNCH
        return status();
    }
    if (fks == 7) {
        G2048_MF_LAUNCH_KS(13, 7);
        return status();
    }
    if (fks == 2) {
        G2048_MF_LAUNCH_KS(13, 2);
        return status();
    }
    switch (nt) {
        case 1: G2048_MF_LAUNCH(1); break;
        case 2: G2048_MF_LAUNCH(2); break;
        case 3: G2048_MF_LAUNCH(3); break;
        case 4: G2048_MF_LAUNCH(4); break;
        case 5: case 6: G2048_MF_LAUNCH(6); break;
        case 7: case 8: G2048_MF_LAUNCH(8); break;
        case 9: case 10: G2048_MF_LAUNCH(10); break;
        case 11: case 12: G2048_MF_LAUNCH(12); break;
        case 13: G2048_MF_LAUNCH(13); break;
        default: G2048_MF_LAUNCH(16); break;
    }
#undef G2048_MF_LAUNCH
#undef G2048_MF_LAUNCH_KS
    return status();
}


int g2048_mlp_fwd_kl(g2048_stream_t stream, const uint16_t *x, const uint16_t *w, const float *gamma,
                     const float *beta, int64_t m, int32_t n, int32_t k, const g2048_dropout *drop, const float *wa,
                     const float *ba, const float *old_masked, const int64_t *rows, float *partials, float *out,
                     g2048_colsum_job *defer) {
    if (n != kMwN || k != kMwN || m <= 0 || !x || !w || !gamma || !beta || !wa || !ba || !old_masked || !partials ||
        !out)
        return G2048_EINVAL;
    if (!al(x, 8) || !al(w, 8) || !al(gamma, 16) || !al(beta, 16) || !al(old_masked, 16)) return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    const DropArgs da = drop_args(drop);
    const int64_t ntile = (m + 15) / 16, nwg = (ntile + kMwWaves - 1) / kMwWaves;
    const int nb = (int)(nwg > 256 ? 256 : nwg);
    const KlArgs ka{wa, ba, old_masked, rows, partials};
    const size_t lds = mw_lds_bytes(kMwN, true);
    if (drop_on(drop))
        hipLaunchKernelGGL((mlp_fwd_wide_kernel<kMwN, true, true, true>), dim3(nb), dim3(kMwThreads), lds, s, x, w, gamma,
                           beta, nullptr, nullptr, nullptr, nullptr, m, da, ka);
    else
        hipLaunchKernelGGL((mlp_fwd_wide_kernel<kMwN, true, false, true>), dim3(nb), dim3(kMwThreads), lds, s, x, w,
                           gamma, beta, nullptr, nullptr, nullptr, nullptr, m, da, ka);
    const int st = status();
    if (st) return st;
    Segs segs{};  // as g2048_ppo_head_kl: out = {sum KL, max KL} over the nb partial pairs
    segs.n = 1;
    segs.dst[0] = out;
    segs.len[0] = 2;
    return colsum(s, partials, nb, 2, partials + (size_t)nb * 2, segs, 1, defer);
}

int g2048_head_fwd(g2048_stream_t stream, const uint16_t *x, const float *wa, const float *ba, const float *wv,
                   const float *bv, int64_t m, int32_t h, float *logits, int64_t logits_stride, float *value) {
    if (m < 0 || h <= 0 || h % 4 || h > 256 || !x || !wa || !ba || !wv || !bv || !logits || !value) return G2048_EINVAL;
    if (!al(x, 8) || logits_stride < 4) return G2048_EINVAL;
    if (m == 0) return G2048_OK;
    const int64_t tiles = (m + 15) / 16;
    const int64_t blocks = (tiles + 3) / 4;
    const dim3 grid((unsigned)(blocks > 2048 ? 2048 : blocks)), blk(256);
    const hipStream_t s = (hipStream_t)stream;
    switch ((h + 31) / 32) {
#define G2048_HF(KS_) case KS_: hipLaunchKernelGGL((head_fwd_kernel<KS_>), grid, blk, 0, s, x, wa, ba, wv, bv, m, h, \
                                                  logits, logits_stride, value); break;
        G2048_HF(1) G2048_HF(2) G2048_HF(3) G2048_HF(4) G2048_HF(5) G2048_HF(6) G2048_HF(7) G2048_HF(8)
#undef G2048_HF
    }
    return status();
}


int g2048_ppo_stats(g2048_stream_t stream, const float *sums, const float *kl, int32_t kl_rows, const float *grad_norm,
                    const float *beta_dev, float critic, int64_t m, const int64_t *rows, float *stats,
                    uint64_t *counter) {
    if (!sums || !kl || kl_rows < 0 || !grad_norm || !beta_dev || !stats || m <= 0) return G2048_EINVAL;
    hipLaunchKernelGGL(ppo_stats_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, sums, kl, kl_rows, grad_norm,
                       beta_dev, critic, (float)m, rows, stats, counter);
    return status();
}

static int colsum_batch_build(const g2048_colsum_job *jobs, int32_t njobs, ColsumBatch &cb, int &blocks);

int g2048_colsum_batch(g2048_stream_t stream, const g2048_colsum_job *jobs, int32_t njobs) {
    ColsumBatch cb{};
    int blocks = 0;
    const int st = colsum_batch_build(jobs, njobs, cb, blocks);
    if (st || !blocks) return st;
    hipLaunchKernelGGL(colsum_batch_kernel, dim3(blocks), dim3(1024), 0, (hipStream_t)stream, cb);
    return status();
}

int g2048_colsum_batch_blocks(const g2048_colsum_job *jobs, int32_t njobs) {
    ColsumBatch cb{};
    int blocks = 0;
    const int st = colsum_batch_build(jobs, njobs, cb, blocks);
    return st ? -1 : blocks;
}

int g2048_colsum_batch_sq(g2048_stream_t stream, const g2048_colsum_job *jobs, int32_t njobs, float *sq, int32_t nsq,
                          float *tick) {
    ColsumBatch cb{};
    int blocks = 0;
    const int st = colsum_batch_build(jobs, njobs, cb, blocks);
    if (st) return st;
    if (!sq || nsq < 1 || nsq > G2048_COLSUM_SQ_MAX || blocks > nsq || ((uintptr_t)sq & 3u)) return G2048_EINVAL;
    cb.sq = sq;
    cb.nsq = nsq;
    cb.tick = tick;
    if (!blocks) blocks = 1;  // (an empty batch still ticks and zeroes the partials)
    hipLaunchKernelGGL(colsum_batch_kernel, dim3(blocks), dim3(1024), 0, (hipStream_t)stream, cb);
    return status();
}

static int colsum_batch_build(const g2048_colsum_job *jobs, int32_t njobs, ColsumBatch &cb, int &blocks) {
    if (njobs < 0 || njobs > G2048_COLSUM_MAX_JOBS || (njobs && !jobs)) return G2048_EINVAL;
    blocks = 0;
    for (int j = 0; j < njobs; j++) {
        const g2048_colsum_job &jb = jobs[j];
        if (!jb.part && jb.cols == 0) continue;  // empty (m = 0) job
        if (!jb.part || jb.nb <= 0 || jb.cols <= 0 || jb.nseg <= 0 || jb.nseg > G2048_COLSUM_SEGS) return G2048_EINVAL;
        int64_t tot = 0;
        for (int k = 0; k < jb.nseg; k++) {
            if (!jb.dst[k] || jb.len[k] <= 0) return G2048_EINVAL;
            tot += jb.len[k];
        }
        if (tot != jb.cols) return G2048_EINVAL;
        cb.job[cb.njobs] = jb;
        cb.first[cb.njobs] = blocks;
        cb.njobs++;
        blocks += colsum_vec(jb) ? (jb.cols + 64 * kColsumW - 1) / (64 * kColsumW) : (jb.cols + 63) / 64;
    }
    cb.first[cb.njobs] = blocks;
    return G2048_OK;
}

int g2048_dropout_mask(g2048_stream_t stream, int64_t m, int32_t h, const g2048_dropout *drop, uint8_t *mask) {
    if (!shape_ok(m, h) || !mask) return G2048_EINVAL;
    if (m == 0) return G2048_OK;
    DropArgs da = drop_args(drop);
    hipLaunchKernelGGL(dropout_mask_kernel, dim3((unsigned)((m * (h / 4) + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, m, h, da, mask);
    return status();
}


int g2048_linear_dgrad_supported(int32_t n, int32_t k) {
    // the shapes where it beats the library GEMM (m = 65 536: 7.8 / 15.0 / 25.0 us vs 19.9 / 19.8 /
    // 42.5 us; at h = 256 hipBLASLt's power-of-two tiles win, 20.9 vs 34.9 us -- tools/time_dgrad.py)
    auto ok = [](int32_t x) { return x == 64 || x == 128 || x == 196; };
    return n == k && ok(n) ? 1 : 0;
}

int g2048_linear_dgrad(g2048_stream_t stream, const uint16_t *dg, const uint16_t *w, uint16_t *out, int64_t m,
                       int32_t n, int32_t k) {
    if (m < 0 || !g2048_linear_dgrad_supported(n, k)) return G2048_EINVAL;
    if (m == 0) return G2048_OK;
    if (!dg || !w || !out || ((uintptr_t)dg | (uintptr_t)out) % 8 || (uintptr_t)w % 2) return G2048_EINVAL;
    const hipStream_t s = (hipStream_t)stream;
    switch (n) {
        case 64: return launch_dgrad<2, 4, 2>(s, dg, w, out, m, n, k);
        case 128: return launch_dgrad<4, 8, 2>(s, dg, w, out, m, n, k);
        default: return launch_dgrad<7, 13, 1>(s, dg, w, out, m, n, k);
    }
}

}  // extern "C"
