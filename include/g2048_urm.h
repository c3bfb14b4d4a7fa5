/*
 * g2048_urm.h -- C ABI of the GameURM policy forward (game.py:1223-1458) in libg2048.so: the
 * Universal-Reasoning-Model transformer over the 16 cell tokens, as fused HIP kernels for gfx950:
 * the four projections of a block (qkv_proj, o_proj, gate_up_proj, down_proj) on the MFMA
 * projection kernel with their epilogues fused (g2048_urm_linear*), everything between them one of
 * the kernels below, the whole rollout forward also as one persistent launch (g2048_urm_forward);
 * for training, the autograd Functions of g2048/urm.py run the forwards, input gradients and weight
 * gradients on these kernels (no library GEMM at the default config).
 *
 * Token layout: board b's 16 cells are rows 16 b .. 16 b + 15 of every [rows, .] activation
 * (row-major, cell order of to_model_format, game.py:92-101), so a board's sequence is contiguous.
 * The residual stream x is fp32 [16 n, h]; GEMM operands are bf16 (raw uint16 bits).  h % 4 == 0,
 * h <= 512, heads | h, head_dim = h / heads <= 64.
 *
 * Conventions: as g2048.h (device pointers, asynchronous on `stream`, no allocation, no host
 * synchronisation; 0 / G2048_EINVAL / hipError_t).
 */
#ifndef G2048_URM_H
#define G2048_URM_H

#include <stddef.h>
#include <stdint.h>

#include "g2048.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Stem and first loop input (game.py:1376-1380, 1425-1431, 1441):
 *   emb = SiLU(LayerNorm(Linear(3 -> h, no bias)(cell features)))      fp32 [16 n, h]
 *   x   = init_hidden + emb;  xb = bf16(x)                              (loop 1's input)
 * obs [n, 48] fp32 (obs_dtype 0) or bf16 (1); w [h, 3], ln_w / ln_b [h], init_hidden [16, h]
 * fp32; LayerNorm eps 1e-5 (nn.LayerNorm default). */
int g2048_urm_stem(g2048_stream_t stream, const void *obs, int32_t obs_dtype, const float *w, const float *ln_w,
                   const float *ln_b, const float *init_hidden, float *emb, float *x, uint16_t *xb, int64_t n,
                   int32_t h);

/* Bidirectional multi-head attention core of GameURMAttention (game.py:1296-1317,
 * scaled_dot_product_attention with scale 1/sqrt(head_dim), no mask, eval mode):
 * qkv bf16 [16 n, 3 h] = x W_qkv^T viewed as (3, heads, head_dim) per token -> out bf16 [16 n, h]
 * (heads concatenated, the o_proj operand).  One wave per (board, head) on
 * v_mfma_f32_16x16x16_bf16: S^T = K Q^T (head_dim zero-padded to 16), masked-free softmax over the
 * 16 keys in registers (fp32), O^T = V^T P^T. */
int g2048_urm_attention(g2048_stream_t stream, const uint16_t *qkv, uint16_t *out, int64_t n, int32_t h,
                        int32_t heads);

/* Backward of g2048_urm_attention for head_dim 16 (h = 16 heads): dout bf16 [16 n, h] (the
 * gradient of the attention output) -> dqkv bf16 [16 n, 3 h] (dq, dk, dv in the qkv layout), P
 * recomputed in fp32 from q, k (autograd path of GameURMAttention, game.py:1296-1317). */
int g2048_urm_attention_bwd(g2048_stream_t stream, const uint16_t *qkv, const uint16_t *dout, uint16_t *dqkv,
                            int64_t n, int32_t h, int32_t heads);

/* Training-mode attention dropout (GameURMAttention, game.py:1314: dropout_p = config.dropout while
 * training): the forward / backward above with P replaced by P * keep / (1 - p) before O = P V.
 * keep: 16-bit Philox4x32-10 uniform >= round(p 2^16), one draw per (board, head, query, group of 4
 * keys) keyed by `seed` with the device call counter *counter (read at launch, so a captured graph
 * draws a new mask per replay once the caller bumps it); the backward regenerates the same mask from
 * the same seed / counter value.  p = 0 is the plain path (counter may be NULL).  The mask is the
 * same distribution as torch's, not its stream. */
int g2048_urm_attention_drop(g2048_stream_t stream, const uint16_t *qkv, uint16_t *out, int64_t n, int32_t h,
                             int32_t heads, float p, uint64_t seed, const uint64_t *counter);
int g2048_urm_attention_bwd_drop(g2048_stream_t stream, const uint16_t *qkv, const uint16_t *dout, uint16_t *dqkv,
                                 int64_t n, int32_t h, int32_t heads, float p, uint64_t seed, const uint64_t *counter);
/* The same with the mask keyed by *counter + offset (round 5: the forward's k-th attention application
 * passes offset k and the caller bumps the counter once per forward by the number of applications,
 * instead of a counter snapshot and a bump per application -- the same masks). */
int g2048_urm_attention_drop_at(g2048_stream_t stream, const uint16_t *qkv, uint16_t *out, int64_t n, int32_t h,
                                int32_t heads, float p, uint64_t seed, const uint64_t *counter, uint64_t offset);
int g2048_urm_attention_bwd_drop_at(g2048_stream_t stream, const uint16_t *qkv, const uint16_t *dout,
                                    uint16_t *dqkv, int64_t n, int32_t h, int32_t heads, float p, uint64_t seed,
                                    const uint64_t *counter, uint64_t offset);

/* The post-norm residual RMSNorm for autograd training (GameURMBlock, game.py:1346-1350, h = 64):
 *   forward  out = (h + a) * rsqrt(mean((h + a)^2) + eps), rstd [rows] saved; h, out fp32, a fp32
 *            (a_dtype 0) or bf16 (1, the autocast projection output)
 *   backward ds = rstd (dout - out mean(dout out)); dh = ds fp32, da = ds in a's dtype. */
int g2048_urm_rms_res_fwd(g2048_stream_t stream, const float *h, const void *a, int32_t a_dtype, float *out,
                          float *rstd, int64_t rows, int32_t hidden, float eps);
int g2048_urm_rms_res_bwd(g2048_stream_t stream, const float *dout, const float *out, const float *rstd, float *dh,
                          void *da, int32_t a_dtype, int64_t rows, int32_t hidden);
/* The same with the output's bf16 copy fused in (the next projection's autocast operand):
 *   fwd2  also outb = bf16(out) [rows, 64] when outb != NULL
 *   bwd2  the output gradient is dout (fp32, may be NULL) + doutb (bf16, may be NULL: the bf16
 *         copy's gradient, converted and added like autocast's cast backward) */
int g2048_urm_rms_res_fwd2(g2048_stream_t stream, const float *h, const void *a, int32_t a_dtype, float *out,
                           uint16_t *outb, float *rstd, int64_t rows, int32_t hidden, float eps);
int g2048_urm_rms_res_bwd2(g2048_stream_t stream, const float *dout, const uint16_t *doutb, const float *out,
                           const float *rstd, float *dh, void *da, int32_t a_dtype, int64_t rows, int32_t hidden);
/*   bwd3  bwd2, or with dpool (fp32 [rows / 16, 64], instead of dout) as the output gradient broadcast
 *         over each board's 16 token rows: the backward of GameURM's token mean-pool (game.py:1450,
 *         dpooled / 16 expanded over the tokens) read without materialising [rows, 64]. */
int g2048_urm_rms_res_bwd3(g2048_stream_t stream, const float *dout, const float *dpool, const uint16_t *doutb,
                           const float *out, const float *rstd, float *dh, void *da, int32_t a_dtype, int64_t rows,
                           int32_t hidden);

/* A GameURM loop start for autograd training (game.py:1441, hidden_states + emb under bf16
 * autocast): out fp32 [rows, hidden] = a + e and outb = bf16(out) (the first block's qkv operand) in
 * one pass; a has rows rows, or a_rows rows broadcast over groups of a_rows (init_hidden [16, h]
 * over the boards; a_rows 0 = rows).  Backward: dx fp32 = dout + float(doutb) (the fp32 and bf16
 * gradient halves; either may be NULL). */
int g2048_urm_add_cast(g2048_stream_t stream, const float *a, int64_t a_rows, const float *e, float *out, uint16_t *outb,
                       int64_t rows, int32_t hidden);
int g2048_urm_add_cast_bwd(g2048_stream_t stream, const float *dout, const uint16_t *doutb, float *dx, int64_t rows,
                           int32_t hidden);
/* The same, with the loops' emb gradient accumulated in the pass: acc_out = acc_in + dx (acc_in NULL:
 * dx), the order autograd sums a tensor's incoming gradients in (the last loop's first); dx may be
 * NULL (h needs no gradient) when acc_out is given. */
int g2048_urm_add_cast_bwd_acc(g2048_stream_t stream, const float *dout, const uint16_t *doutb, float *dx,
                               const float *acc_in, float *acc_out, int64_t rows, int32_t hidden);

/* SwiGLU + depthwise conv (kernel 2) for autograd training (GameConvSwiGLU, game.py:1264-1276),
 * n boards of 16 tokens, inter <= 128 channels, the reference's autocast dtypes:
 *   forward  y = bf16(bf16(silu(gate)) up), y2 = y_{t-1} w[c][0] + y_t w[c][1] + b[c] (fp32),
 *            act = bf16(silu(y2)) [16 n, inter];  gu bf16 [16 n, 2 inter] (gate | up)
 *   backward dgu bf16 [16 n, 2 inter], dw fp32 [inter][2], db fp32 [inter] (deterministic column
 *            sums over g2048_urm_swiglu_conv_partials(n, inter) floats of scratch). */
size_t g2048_urm_swiglu_conv_partials(int64_t n, int32_t inter);
/* The SwiGLU-conv backward with gu RECOMPUTED from gate_up's operand (round 5; the training forward
 * then stores act only): gu = bf16(x W^T) on MFMA with the fused forward's fragments and k order
 * (bitwise the gu g2048_urm_linear_swiglu_train would have stored), then the backward above: dgu
 * bf16 [16 n, 2 inter], dw fp32 [inter][2], db fp32 [inter] (deterministic; the partial scratch of
 * g2048_urm_swiglu_conv_partials).  x bf16 [16 n, h], w bf16 [2 inter, h] (gate rows, then up rows),
 * conv_w fp32 [inter][2], conv_b fp32 [inter] (any 4-byte alignment), dact bf16 [16 n, inter].
 * h 64 (inter 72..128) or h 32 (inter 40..64), inter % 8 == 0. */
int g2048_urm_gate_up_swiglu_bwd_supported(int32_t h, int32_t inter);
int g2048_urm_gate_up_swiglu_bwd(g2048_stream_t stream, const uint16_t *x, const uint16_t *w, const float *conv_w,
                                 const float *conv_b, const uint16_t *dact, uint16_t *dgu, float *dw, float *db,
                                 float *partials, int64_t n, int32_t h, int32_t inter);
/* accumulate != 0: dw / db are ADDED to (dw += its sum, db += its sum) -- the conv parameters' gradient
 * summed over the loop applications in autograd's order, straight into the parameters' .grad (round 5) */
int g2048_urm_gate_up_swiglu_bwd_acc(g2048_stream_t stream, const uint16_t *x, const uint16_t *w, const float *conv_w,
                                     const float *conv_b, const uint16_t *dact, uint16_t *dgu, float *dw, float *db,
                                     float *partials, int64_t n, int32_t h, int32_t inter, int32_t accumulate);
int g2048_urm_swiglu_conv_fwd(g2048_stream_t stream, const uint16_t *gu, const float *w, const float *b, uint16_t *act,
                              int64_t n, int32_t inter);
int g2048_urm_swiglu_conv_bwd(g2048_stream_t stream, const uint16_t *gu, const float *w, const float *b,
                              const uint16_t *dact, uint16_t *dgu, float *dw, float *db, float *partials, int64_t n,
                              int32_t inter);

/* The stem for autograd training (GameURM.stem under bf16 autocast, game.py:1376-1380, h = 64):
 *   forward  emb = SiLU(LayerNorm(bf16(x W^T))) fp32 [16 n, 64]; obs [n, 48] fp32 (obs_dtype 0,
 *            rounded to bf16 like autocast) or bf16 (1); w [64, 3], ln_w / ln_b [64] fp32
 *   backward demb fp32 [16 n, 64] -> grads fp32 [320] = dW [64][3] | d ln_w [64] | d ln_b [64]
 *            (deterministic: per-block partials over g2048_urm_stem_partials(n) floats of scratch
 *            summed in a fixed order); the observation gets no gradient. */
size_t g2048_urm_stem_partials(int64_t n);
int g2048_urm_stem_fwd(g2048_stream_t stream, const void *obs, int32_t obs_dtype, const float *w, const float *ln_w,
                       const float *ln_b, float *emb, int64_t n, int32_t h, float eps);
int g2048_urm_stem_bwd(g2048_stream_t stream, const void *obs, int32_t obs_dtype, const float *w, const float *ln_w,
                       const float *ln_b, const float *demb, float *grads, float *partials, int64_t n, int32_t h,
                       float eps);
/* The same with the three gradients at their own addresses (dw [64][3], dln_w [64], dln_b [64]: the
 * parameters' .grad) and, with accumulate, added to (round 5: no copies / accumulation kernels). */
int g2048_urm_stem_bwd3(g2048_stream_t stream, const void *obs, int32_t obs_dtype, const float *w, const float *ln_w,
                        const float *ln_b, const float *demb, float *dw, float *dln_w, float *dln_b, int32_t accumulate,
                        float *partials, int64_t n, int32_t h, float eps);

/* Weight gradient of a projection y = x W^T for autograd training: dw fp32 [n, k] = dy^T x over m
 * rows, dy bf16 [m, n], x bf16 [m, k] (the shapes g2048_urm_wgrad_supported(n, k) accepts: n % 16 == 0,
 * k % 8 == 0, n, k <= 256 and at most 64 output tiles of 16 x 16 -- the default GameURM's qkv / o /
 * gate_up / down), deterministic (per-block partials over g2048_urm_wgrad_partials(m, n, k) floats of
 * scratch, summed in a fixed order).  Replaces the K = 16 n weight-gradient GEMMs of autocast's
 * nn.Linear backward for GameURMAttention / GameConvSwiGLU (game.py:1264-1352). */
int g2048_urm_wgrad_supported(int32_t n, int32_t k);
size_t g2048_urm_wgrad_partials(int64_t m, int32_t n, int32_t k);
int g2048_urm_wgrad(g2048_stream_t stream, const uint16_t *dy, const uint16_t *x, float *dw, float *partials,
                    int64_t m, int32_t n, int32_t k);
/* accumulate != 0: dw += dy^T x (the sum rounded once, then added: the bits of autograd's accumulation of
 * a returned gradient into the weight's .grad, round 5) */
int g2048_urm_wgrad_acc(g2048_stream_t stream, const uint16_t *dy, const uint16_t *x, float *dw, float *partials,
                        int64_t m, int32_t n, int32_t k, int32_t accumulate);

/* The whole backward of the residual-RMSNorm projection out = rms_norm(h + bf16(x W^T)) (o_proj /
 * down_proj of GameURMBlock, game.py:1346-1350; LinResRMSFn) in one pass (round 5), for hidden 64
 * and input width k 64 / 120 (g2048_urm_linres_bwd_supported):
 *   g  = dout [or dpool broadcast over each board's 16 rows] [+ doutb as fp32]   (any may be NULL)
 *   dh = rstd (g - out mean(g out))                  fp32 [rows, 64]  (the residual's gradient)
 *   dx = bf16(dh) W                                  bf16 [rows, k]   (NULL: not computed)
 *   dw = bf16(dh)^T x   (accumulate: dw += ...)      fp32 [64, k]
 * out fp32 [rows, 64] and rstd [rows] as the forward wrote them, w bf16 [64, k], x bf16 [rows, k];
 * rows % 16 == 0; every row pointer 16-byte aligned; partials: g2048_urm_linres_bwd_partials(rows, k)
 * floats of scratch.  = g2048_urm_rms_res_bwd2 + g2048_urm_linear_t + g2048_urm_wgrad_acc without
 * the bf16 dh round trip through HBM (dx bitwise g2048_urm_linear_t of the same bf16 dh; dh and dw
 * within fp32 rounding of them: the row mean and the row sum are added in another order). */
int g2048_urm_linres_bwd_supported(int32_t hidden, int32_t k);
size_t g2048_urm_linres_bwd_partials(int64_t rows, int32_t k);
int g2048_urm_linres_bwd(g2048_stream_t stream, const float *dout, const float *dpool, const uint16_t *doutb,
                         const float *out, const float *rstd, const uint16_t *w, const uint16_t *x, float *dh,
                         uint16_t *dx, float *dw, float *partials, int32_t accumulate, int64_t rows, int32_t hidden,
                         int32_t k);

/* Post-norm residual (game.py:1346, 1350 with rms_norm :1223-1229):
 *   x = x + y;  x = x * rsqrt(mean(x^2) + eps)  [+ emb, the next loop's input, game.py:1447];
 *   xb = bf16(x).
 * x fp32 [rows, h] in place, y bf16 [rows, h] (a projection output), emb fp32 or NULL. */
int g2048_urm_residual_rms(g2048_stream_t stream, float *x, const uint16_t *y, const float *emb, uint16_t *xb,
                           int64_t rows, int32_t h, float eps);

/* GameConvSwiGLU between its two projections (game.py:1264-1276): gu bf16 [16 n, 2 inter] =
 * x W_gate_up^T -> a = SiLU(gate) * up; depthwise Conv1d(kernel 2, padding 1, trimmed to 16
 * tokens) over each board's sequence: c_t = w[ch][0] a_{t-1} + w[ch][1] a_t + b[ch] (a_{-1} = 0);
 * out = bf16(SiLU(c)) [16 n, inter] (the down_proj operand).  w fp32 [inter, 2], b fp32 [inter]. */
int g2048_urm_swiglu_conv(g2048_stream_t stream, const uint16_t *gu, const float *w, const float *b, uint16_t *out,
                          int64_t n, int32_t inter);

/* Mean pooling over the 16 tokens and the two heads (game.py:1452-1456): logits fp32 [n, 4] =
 * pooled wa^T + ba, value fp32 [n] = pooled wv^T + bv;  x fp32 [16 n, h], wa [4, h], wv [1, h]. */
int g2048_urm_pool_heads(g2048_stream_t stream, const float *x, const float *wa, const float *ba, const float *wv,
                         const float *bv, float *logits, float *value, int64_t n, int32_t h);

/* The projections with their epilogues fused (small hidden sizes; g2048_urm_linear_supported says
 * which): y = in W^T on bf16 MFMA, W bf16 [n, k] (nn.Linear weight), in bf16 [rows, k], rows % 16
 * == 0 (whole boards), fp32 accumulate, and
 *   g2048_urm_linear          out bf16 [rows, n] = y                                 (qkv_proj)
 *   g2048_urm_linear_rms      x = rms_norm(x + y) [+ emb], xb = bf16(x), n = h       (o_proj, down_proj)
 *   g2048_urm_linear_swiglu   out bf16 [rows, inter] = SiLU(conv(SiLU(gate) * up))  (gate_up_proj,
 *                             w [2 inter, h]; the conv as g2048_urm_swiglu_conv)
 * The projection output never goes through HBM.  epilogue: 0 / 1 / 2 as listed.
 * g2048_urm_linear also serves the training Functions' plain GEMMs (game.py:1279-1352 under bf16
 * autocast, in place of torch.mm / hipBLASLt): the o_proj / down_proj forwards and every input
 * gradient dX = dY W, called with W^T [k_in, n_out] as `w` (h 64: k x n in {64x64, 120x64, 192x64,
 * 64x120, 240x64}; h 32 the same shapes halved). */
int g2048_urm_linear_supported(int32_t epilogue, int32_t k, int32_t n, int32_t inter);
int g2048_urm_linear(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, uint16_t *out, int64_t rows,
                     int32_t k, int32_t n);
/* out [rows, n] = in [rows, k] w with w given as [k, n] row-major: the input gradient dX = dY W of a
 * projection W [k = out features, n = in features] without a transposed copy of W (the kernel
 * stages W^T itself).  Same MFMA order as g2048_urm_linear on W^T (bitwise equal). */
int g2048_urm_linear_t(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, uint16_t *out, int64_t rows,
                       int32_t k, int32_t n);
/* g2048_urm_linear with an fp32 bias [n] added to the fp32 accumulator before the one bf16 rounding
 * (autocast's biased Linear: bf16 operands and bias, one rounding of x W^T + b; bias 16-byte aligned). */
int g2048_urm_linear_bias(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, const float *bias, uint16_t *out,
                          int64_t rows, int32_t k, int32_t n);
int g2048_urm_linear_rms(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, float *x, const float *emb,
                         uint16_t *xb, int64_t rows, int32_t k, int32_t h, float eps);
int g2048_urm_linear_swiglu(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, const float *conv_w,
                            const float *conv_b, uint16_t *out, int64_t rows, int32_t h, int32_t inter);

/* Training variant of g2048_urm_linear_swiglu (epilogue 3 of g2048_urm_linear_supported) for the
 * autograd GateUpSwiGLUFn: also stores gu = bf16(x W_gu^T) [rows, 2 inter] (gate | up: the backward's
 * input) and computes act from those bf16 values with g2048_urm_swiglu_conv_fwd's arithmetic, so the
 * result equals gate_up Linear (autocast bf16) + g2048_urm_swiglu_conv_fwd up to the GEMM's fp32
 * summation order.  in bf16 [rows, h], w bf16 [2 inter, h], conv_w fp32 [inter][2], conv_b [inter];
 * inter % 8 == 0 and gu / act 16-byte aligned (8 features per lane per store).  gu may be NULL (round
 * 4: the no-grad truncated loops, act with the training arithmetic and nothing else stored). */
int g2048_urm_linear_swiglu_train(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, const float *conv_w,
                                  const float *conv_b, uint16_t *gu, uint16_t *act, int64_t rows, int32_t h,
                                  int32_t inter);

/* Training variant of g2048_urm_linear_rms (epilogue 4 of g2048_urm_linear_supported) for the autograd
 * LinResRMSFn -- o_proj / down_proj + residual + post-norm of GameURMBlock (game.py:1346-1350) under bf16
 * autocast: a = bf16(in W^T) (the projection's autocast output), s = h + a, out = s rsqrt(mean(s^2) +
 * eps) -> out fp32 [rows, n], outb bf16 copy (optional, the next projection's operand), rstd fp32
 * [rows] (the backward's g2048_urm_rms_res_bwd2 input); h is read only.  Replaces g2048_urm_linear +
 * g2048_urm_rms_res_fwd2 (the projection output's HBM round trip).  h / out 16-byte aligned. */
int g2048_urm_linear_res_rms(g2048_stream_t stream, const uint16_t *in, const uint16_t *w, const float *h, float *out,
                             uint16_t *outb, float *rstd, int64_t rows, int32_t k, int32_t n, float eps);

/* The whole forward in one persistent kernel (the default GameURMConfig: hidden 64, 4 heads,
 * inter 120, conv kernel 2, 1 or 2 layers, any loop count): obs [n, 48] (fp32 / bf16) -> logits
 * fp32 [n, 4], value fp32 [n]; every activation stays in registers / LDS, the weights of the layer
 * being applied are streamed through LDS.  Weights: bf16 matrices in nn.Linear layout (qkv [192, 64],
 * o [64, 64], gate_up [240, 64], down [64, 120]); conv_w fp32 [120, 2], conv_b fp32 [120]; stem,
 * LayerNorm, init_hidden [16, 64] and head parameters fp32; the matrices and conv arrays 16-byte
 * aligned. */
typedef struct g2048_urm_weights {
    int32_t hidden, heads, inter, num_layers, num_loops;
    float eps;
    const float *stem_w, *ln_w, *ln_b, *init_hidden, *wa, *ba, *wv, *bv;
    const uint16_t *qkv[2], *o[2], *gate_up[2], *down[2];
    const float *conv_w[2], *conv_b[2];
} g2048_urm_weights;

int g2048_urm_forward_supported(int32_t hidden, int32_t heads, int32_t inter, int32_t num_layers, int32_t conv_kernel);
int g2048_urm_forward(g2048_stream_t stream, const g2048_urm_weights *w, const void *obs, int32_t obs_dtype,
                      float *logits, float *value, int64_t n);

/* g2048_urm_forward in training mode (the model's attention dropout, game.py:1314): block
 * application `app` (0 .. num_loops * num_layers - 1) draws the mask of g2048_urm_attention_drop at
 * counter *counter + app (the caller bumps the counter by that many afterwards).  Used for the PPO
 * update's no-grad KL re-forward (train.py:577-582, model still in train mode).  p = 0: g2048_urm_forward. */
int g2048_urm_forward_drop(g2048_stream_t stream, const g2048_urm_weights *w, const void *obs, int32_t obs_dtype,
                           float *logits, float *value, int64_t n, float p, uint64_t seed, const uint64_t *counter);

/* GameURM's PPO minibatch loss on device kernels (model_optimize_step, train.py:491-601, with GameURM's
 * heads, game.py:1451-1456), replacing the ~50 small torch kernels of the heads' autocast projection,
 * the loss expression, its autograd backward, the KL's masked softmaxes and the statistics stack:
 *   g2048_urm_head_loss      pooled [m, h] (fp32: pooled_dtype 0, or bf16: 1) -> z = bf16(bf16(pooled)
 *                            bf16(W)^T + bf16(b)) for W = [Wa; Wv] (autocast's rounding points), the
 *                            per-row PPO-clip / entropy / smooth-L1 loss of g2048_ppo_head_loss
 *                            (batch: the trajectory columns at idx; rows must be NULL), dz fp32 [m, 8]
 *                            (d mean-loss / d(logits, value), columns 5..7 zero), masked fp32 [m, 4]
 *                            (logits with -inf at illegal actions), sums[3] = {sum ppo, sum H, sum v},
 *                            loss[1] = -(mean ppo - critic mean v + beta mean H)
 *   g2048_urm_head_loss_bwd  dy = bf16(grad_out dz) -> dpooled = bf16(dy W) in pooled's dtype, dWa [4, h],
 *                            dba [4], dWv [h], dbv [1] = dy^T bf16(pooled), column sums of dy (overwritten,
 *                            or added to with accumulate)
 *   g2048_urm_kl_stats       KL(old || new) per row from masked and the re-forward's logits fp32 [m, 4],
 *                            then stats[9] += the minibatch's loss / entropy / value / grad-norm / KL
 *                            statistics (g2048_ppo_stats' update: sums, gn, beta_dev, critic, m)
 * h 64 or 32; partials: g2048_urm_head_loss_partials(m, h) floats; sync: a device uint32 ticket word,
 * zero at the first call (each kernel's last block puts it back to zero).  Deterministic: fixed-order
 * block trees and a last-block pass over the block partials. */
struct g2048_ppo_batch;
size_t g2048_urm_head_loss_partials(int64_t m, int32_t h);
int g2048_urm_head_loss(g2048_stream_t stream, const void *pooled, int32_t pooled_dtype, const float *wa,
                        const float *ba, const float *wv, const float *bv, int64_t m, int32_t h,
                        const struct g2048_ppo_batch *batch, const float *beta_dev, float critic, float clip_eps,
                        float *dz, float *masked, float *partials, uint32_t *sync, float *sums, float *loss);
int g2048_urm_head_loss_bwd(g2048_stream_t stream, const void *pooled, int32_t pooled_dtype, const float *wa,
                            const float *wv, const float *dz, const float *grad_out, void *dpooled, float *partials,
                            uint32_t *sync, float *dwa, float *dba, float *dwv, float *dbv, int32_t accumulate,
                            int64_t m, int32_t h);
int g2048_urm_kl_stats(g2048_stream_t stream, const float *old_masked, const float *logits, int64_t m,
                       const float *sums, const float *gn, const float *beta_dev, float critic, float *stats,
                       float *partials, uint32_t *sync);

#ifdef __cplusplus
}
#endif

#endif /* G2048_URM_H */
