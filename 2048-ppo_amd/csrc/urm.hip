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
//   residual_rms     one wave per row: x = rms_norm(x + y) [+ emb], bf16 copy for the next GEMM
//   swiglu_conv      one thread per (board, channel): SiLU(gate)*up, the kernel-2 depthwise conv
//                    along the board's 16 tokens carried in a register, SiLU
//   pool_heads       one wave per board: mean over the 16 tokens, action / value heads
//
// fp32 arithmetic throughout (bf16 only as GEMM operands / attention probabilities, like torch's
// bf16 autocast of the same module); parity vs the fp32 module in tests/test_gpu_urm.py.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/g2048_urm.h"

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kMaxPerLane = 8;  // h <= 512 over 64 lanes

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even (finite inputs)
    const uint32_t u = __float_as_uint(f);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
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

__global__ __launch_bounds__(kThreads) void urm_attn_kernel(const uint16_t *__restrict__ qkv,
                                                            uint16_t *__restrict__ out, int64_t tasks, int h,
                                                            int heads) {
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
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
            const int d = d0 + 4 * g + jj;
            ka[jj] = d < hd ? (short)krow[d] : (short)0;
            qb[jj] = d < hd ? (short)qrow[d] : (short)0;
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
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float sum = 0.0f;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        p[r] = __expf(p[r] - m);
        sum += p[r];
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.0f / sum;
    s16x4 pb;  // B operand of O^T = V^T P^T: B[k = key 4g + jj][n = query i]
#pragma unroll
    for (int r = 0; r < 4; r++) pb[r] = (short)f2bf(p[r] * inv);
    // A operand: V^T[row = dim d0 + i][k = key 4g + jj] = V[4g + jj][d0 + i]
    const uint16_t *vcol = base + 2 * h + hh * hd;
    uint16_t *orow = out + (b * 16 + i) * (int64_t)h + hh * hd;
    for (int d0 = 0; d0 < hd; d0 += 16) {
        s16x4 va;
        const int d = d0 + i;
#pragma unroll
        for (int jj = 0; jj < 4; jj++)
            va[jj] = d < hd ? (short)vcol[(int64_t)(4 * g + jj) * (3 * h) + d] : (short)0;
        f32x4 o = {0.0f, 0.0f, 0.0f, 0.0f};
        o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, pb, o, 0, 0, 0);
        // lane (i, g): o[r] = O^T[d0 + 4g + r][i] = O[i][d0 + 4g + r]
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int dd = d0 + 4 * g + r;
            if (dd < hd) orow[dd] = f2bf(o[r]);
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

}  // namespace

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

int g2048_urm_attention(g2048_stream_t stream, const uint16_t *qkv, uint16_t *out, int64_t n, int32_t h,
                        int32_t heads) {
    if (n < 0 || !h_ok(h) || heads <= 0 || h % heads != 0 || h / heads > 64) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!qkv || !out) return G2048_EINVAL;
    const int64_t tasks = n * heads;
    hipLaunchKernelGGL(urm_attn_kernel, dim3(blocks(tasks, kThreads / 64)), dim3(kThreads), 0, (hipStream_t)stream,
                       qkv, out, tasks, (int)h, (int)heads);
    return launch_status();
}

int g2048_urm_residual_rms(g2048_stream_t stream, float *x, const uint16_t *y, const float *emb, uint16_t *xb,
                           int64_t rows, int32_t h, float eps) {
    if (rows < 0 || !h_ok(h)) return G2048_EINVAL;
    if (rows == 0) return G2048_OK;
    if (!x || !y || !xb) return G2048_EINVAL;
    hipLaunchKernelGGL(urm_residual_rms_kernel, dim3(blocks(rows, kThreads / 64)), dim3(kThreads), 0,
                       (hipStream_t)stream, x, y, emb, xb, rows, (int)h, eps);
    return launch_status();
}

int g2048_urm_swiglu_conv(g2048_stream_t stream, const uint16_t *gu, const float *w, const float *b, uint16_t *out,
                          int64_t n, int32_t inter) {
    if (n < 0 || inter <= 0) return G2048_EINVAL;
    if (n == 0) return G2048_OK;
    if (!gu || !w || !b || !out) return G2048_EINVAL;
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

}  // extern "C"
