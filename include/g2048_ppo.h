/*
 * g2048_ppo.h -- C ABI of the PPO-update kernels in libg2048.so: the GameMLP forward/backward and
 * the PPO-clip loss of model_optimize_step (train.py:414-642) around the model's GEMMs.
 *
 * The reference runs this step through torch autograd (agent GameMLP, game.py:1033-1220; loss
 * train.py:497-568).  Here the minibatch step is explicit: the GEMMs X W^T / dG W / dG^T X go to
 * the platform BLAS (hipBLASLt through torch), everything between them is one of the fused kernels
 * below, and the whole step is captured in a hipGraph by the caller (g2048/fastmlp.py).
 *
 * Conventions: as g2048.h (device pointers, asynchronous on `stream`, no allocation, no host
 * synchronisation, 0 / G2048_EINVAL / hipError_t).  Activations are bf16 (raw uint16 bits),
 * row-major [m, h] with h % 4 == 0 and h <= 1024; LayerNorm statistics, gradients and all
 * reductions are fp32.  Reductions over rows go through per-block partials in a fixed order, so
 * every entry point is deterministic run to run.
 */
#ifndef G2048_PPO_H
#define G2048_PPO_H

#include <stddef.h>
#include <stdint.h>

#include "g2048.h"

#ifdef __cplusplus
extern "C" {
#endif

/* nn.Dropout(p) of a ResidualBlock (game.py:1033-1046), train mode.  Element (row, col) of column
 * group cg = col / 4 = 8a + 4h + b is kept iff its 16-bit uniform >= round(p 2^16), the uniforms
 * being the 8 halves of one Philox4x32-10 draw keyed by `seed` with counter
 * {row, (4a + b) | layer << 12 | pass << 20, *counter_dev + counter} (h picks words {x,y} or {z,w},
 * col % 4 the half-word) -- regenerated, never stored, so the backward pass sees exactly the
 * forward's mask.  p == 0 disables it. */
typedef struct g2048_dropout {
    float p;
    uint32_t layer;
    uint32_t pass;
    uint32_t pad_;
    uint64_t seed;
    uint64_t counter;
    const uint64_t *counter_dev; /* optional device counter base (graph replays advance it) */
} g2048_dropout;

/* to_model_format (game.py:92-101) of boards[idx[r]] for r < m -> bf16 [m, 48]: the gather of a
 * minibatch out of the flat trajectory fused with the encoding. */
int g2048_obs_gather(g2048_stream_t stream, const int8_t *boards, const int64_t *idx, int64_t m, uint16_t *obs);

/* y = res + Dropout(ReLU(LayerNorm(g)))  (res == NULL: the stem, y = ReLU(LayerNorm(g))).
 * LayerNorm eps 1e-5 with affine gamma/beta (nn.LayerNorm defaults); writes the per-row mean and
 * 1/sqrt(var + eps) for the backward pass. */
int g2048_ln_act_fwd(g2048_stream_t stream, const uint16_t *g, const float *gamma, const float *beta,
                     const uint16_t *res, uint16_t *y, float *mean, float *rstd, int64_t m, int32_t h,
                     const g2048_dropout *drop);

/* Dynamic LDS bytes of g2048_mlp_fwd for an [n, k] weight (0 = unsupported: n, k % 4 != 0 or > 256). */
size_t g2048_mlp_fwd_lds_bytes(int32_t n, int32_t k);

/* A whole Linear(bias=False) + LayerNorm + ReLU [+ Dropout + residual] layer forward on MFMA:
 *   g = x w^T (bf16 [m, n], kept for the backward);  y = [x +] Dropout(ReLU(LayerNorm(g)))
 * x bf16 [m, k], w bf16 [n, k]; residual requires n == k (ResidualBlock); mean / rstd as
 * g2048_ln_act_fwd.  Same results as a bf16 GEMM followed by g2048_ln_act_fwd, up to fp32
 * summation order.  Inference (the rollout policy) passes g = mean = rstd = NULL. */
int g2048_mlp_fwd(g2048_stream_t stream, const uint16_t *x, const uint16_t *w, const float *gamma, const float *beta,
                  int32_t residual, uint16_t *g, uint16_t *y, float *mean, float *rstd, int64_t m, int32_t n, int32_t k,
                  const g2048_dropout *drop);

/* Rollout policy heads (GameMLP.forward, game.py:1208-1219) on MFMA: logits[r * logits_stride + a]
 * = x[r] . wa[a] + ba[a] (a < 4), value[r] = x[r] . wv + bv; x bf16 [m, h], weights fp32 (used as
 * bf16), fp32 accumulate. */
int g2048_head_fwd(g2048_stream_t stream, const uint16_t *x, const float *wa, const float *ba, const float *wv,
                   const float *bv, int64_t m, int32_t h, float *logits, int64_t logits_stride, float *value);

/* The fused persistent policy rollout (play_game_for_episode's loop body, train.py:240-337, for
 * every env at once; replaces one Rollout._step per step = g2048_obs_encode + FusedPolicy (three
 * g2048_mlp_fwd + g2048_head_fwd) + g2048_sample_actions + g2048_env_step).  Steps t0 .. t1-1 of
 * all n envs in ONE launch: boards / flags rows t0 are the start state, rows t0+1 .. t1 and the
 * per-step records of rows t0 .. t1-1 are written exactly as the per-step path writes them -- the
 * same time-major [T(+1)][n] layouts as g2048_env_step / g2048_sample_actions, the same Philox
 * streams (action uniform: stream 1 at counter c + 2t; spawns: stream 0, resets: stream 2, at
 * c + 2t + 1; c = counter + *counter_dev) and the same arithmetic (bitwise equal records).
 * GameMLP eval mode with num_layers == 2 and hidden % 4 == 0 whose two h x h block weights fit
 * LDS (g2048_policy_rollout_supported; h = 196 and 192 do).  Weights: the bf16 copies
 * FusedPolicy keeps (w_stem [h][48], w_block[l] [h][h], 8-byte aligned, stem 16-byte), the fp32
 * LayerNorm affines, the heads as bf16 head_bf16 [5][32 ceil(h / 32)] (action_head rows 0..3,
 * value_head row 4, zero padded, 16-byte aligned) and the fp32 biases.  opts: G2048_OPT_AUTO_RESET
 * (fixed horizon) or G2048_OPT_SKIP_DONE (episodic).  Philox spawns only. */
typedef struct g2048_policy_rollout_args {
    int8_t *boards;          /* [T+1][n][16] */
    uint8_t *flags;          /* [T+1][n] legal mask | done / reset / invalid / inactive bits */
    uint8_t *actions;        /* [T][n] */
    float *logp;             /* [T][n][4] log_softmax of the masked logits (-inf where illegal) */
    float *entropy;          /* [T][n] */
    float *value;            /* [T][n] */
    int32_t *points;         /* [T][n] */
    int8_t *max_tile;        /* [T][n] */
    int8_t *pot;             /* [T][n][4] mono_b, mono_a, empt_b, empt_a */
    int64_t n, t0, t1;
    int32_t hidden, num_layers;
    uint32_t opts, env_base;
    const void *w_stem;
    const void *w_block[2];
    const float *ln_gamma[3], *ln_beta[3];
    const void *head_bf16;
    const float *head_bias_action, *head_bias_value;
    uint64_t seed, counter;
    const uint64_t *counter_dev; /* optional device counter base */
    float *debug;            /* optional test hook (NULL): step t0's layer outputs [3][n][16 ceil(h/16)]
                                followed by its head outputs [n][5] (4 logits, value) */
} g2048_policy_rollout_args;

/* 1 when g2048_policy_rollout handles a GameMLP of this shape. */
int g2048_policy_rollout_supported(int32_t hidden, int32_t num_layers);
/* Dynamic LDS bytes the rollout kernel uses for hidden size h (0 = does not fit). */
size_t g2048_policy_rollout_lds_bytes(int32_t h);
int g2048_policy_rollout(g2048_stream_t stream, const g2048_policy_rollout_args *args);

/* Scratch floats of g2048_ln_act_bwd for (m, h). */
size_t g2048_ln_act_bwd_partials(int64_t m, int32_t h);

/* A deferred column reduction.  Every kernel below that reduces over the minibatch rows writes
 * per-block partial rows part[nb][cols] and, by default, sums them itself (two extra launches).
 * Given a non-NULL `defer`, it instead describes that sum here and g2048_colsum_batch performs any
 * number of them in ONE launch: dst <- the fixed-order (deterministic) column sums of part, the
 * column max_col (>= 0) taking the max instead, split into nseg segments of len[i] columns. */
#define G2048_COLSUM_SEGS 5
typedef struct g2048_colsum_job {
    const float *part;
    int32_t nb, cols, max_col, nseg;
    float *dst[G2048_COLSUM_SEGS];
    int32_t len[G2048_COLSUM_SEGS];
    int32_t pad_;
} g2048_colsum_job;

#define G2048_COLSUM_MAX_JOBS 16
int g2048_colsum_batch(g2048_stream_t stream, const g2048_colsum_job *jobs, int32_t njobs);
/* g2048_colsum_batch that also prices the gradient norm: bit k of a job's pad_ marks segment k as
 * gradient; sq[b] = the sum of squares of block b's gradient outputs (b < nsq: the blocks past the
 * launch's grid are zeroed), *tick += 1 (the optimizer's step count) -- the partials the fused
 * optimizer step reads instead of a g2048_grad_sumsq_tick pass over the bucket (single process: the
 * gradient is final when summed).  nsq >= g2048_colsum_batch_blocks(jobs, njobs). */
#define G2048_COLSUM_SQ_MAX 1024
int g2048_colsum_batch_blocks(const g2048_colsum_job *jobs, int32_t njobs);
int g2048_colsum_batch_sq(g2048_stream_t stream, const g2048_colsum_job *jobs, int32_t njobs, float *sq, int32_t nsq,
                          float *tick);

#define G2048_DY_MAX_P 4

/* The sources of a residual block's output gradient dy (each optional):
 *   dres  fp32 [m,h]  a residual-stream gradient accumulated above;
 *   p[i]  bf16 [m,h]  matmul gradients dG_j W_j of the blocks above (NULL entries are skipped);
 *   dz    fp32 [m,8]  the policy/value heads' output gradient as g2048_ppo_head_loss writes it
 *                     (columns 0..4); their share dz[:,0:4] wa + dz[:,4] wv is recomputed in the
 *                     kernel, so no [m,h] head gradient goes through HBM; wa fp32 [4,h]; wv fp32 [h]
 *                     or NULL when the critic is decoupled (game.py:1213-1219).
 * dy = dres + sum_i p[i] + heads, summed in fp32. */
typedef struct g2048_dy {
    const float *dres;
    const uint16_t *p[G2048_DY_MAX_P];
    const float *dz;
    const float *wa;
    const float *wv;
} g2048_dy;

/* Backward of g2048_ln_act_fwd for the output gradient *dy (above).  Writes dg (bf16 [m,h], gradient
 * of the pre-norm activation), dy itself to dres_out (fp32, optional: a residual gradient passed
 * further down), and dgamma / dbeta (fp32 [h], overwritten). */
int g2048_ln_act_bwd(g2048_stream_t stream, const g2048_dy *dy, const uint16_t *g, const float *mean,
                     const float *rstd, const float *gamma, const float *beta, uint16_t *dg, float *dres_out,
                     float *partials, float *dgamma, float *dbeta, int64_t m, int32_t h, const g2048_dropout *drop,
                     g2048_colsum_job *defer);

/* Per-minibatch inputs of the PPO loss, gathered on the fly through idx from the flat trajectory
 * (train.py:466-496). */
typedef struct g2048_ppo_batch {
    const int64_t *idx;    /* [m] rows of the flat trajectory */
    const uint8_t *action; /* [M] */
    const uint8_t *legal;  /* [M] bit a = action a legal */
    const float *old_logp; /* [M, 4] log_softmax of the masked rollout logits */
    const float *adv;      /* [M] */
    const float *ret;      /* [M] normalised return-to-go (value target) */
    const int64_t *rows;   /* nullable device count n <= m: rows >= n of the minibatch are padding (the
                              ragged last minibatch of an epoch run at full size): zero loss and
                              gradient, left out of every sum, and the loss mean is over n rows */
} g2048_ppo_batch;

/* Scratch floats of g2048_ppo_head_loss / g2048_ppo_head_kl for (m, h). */
size_t g2048_ppo_head_partials(int64_t m, int32_t h);

/* Policy/value heads + PPO-clip loss + their backward for one minibatch (train.py:497-568):
 *   logits = x Wa^T + ba, value = x Wv^T + bv;  masked = logits with -inf at illegal actions;
 *   ratio = exp(clamp(logpi(a) - old_logp(a), -20, 20));  ppo = min(A ratio, A clip(ratio, 1-eps, 1+eps));
 *   H = -sum_legal softmax(clamp(masked,-20,20)) log_softmax(...);  v = smooth_l1(value, ret);
 *   loss = -mean(ppo - critic v + beta H)
 * Writes masked (fp32 [m,4], for the KL diagnostic), dx = dloss/dx (fp32 [m,h], optional; the value
 * branch is excluded when decouple_critic, game.py:1213-1219) and/or dz = dloss/d(logits, value)
 * (fp32 [m,8], optional: columns 0..4, for g2048_dy.dz), the head gradients dwa [4,h], dba [4],
 * dwv [h], dbv [1] (overwritten) and sums[3] = {sum ppo, sum H, sum v} over the minibatch.
 * beta_dev: device float (the entropy coefficient, a device scalar so replays see updates). */
int g2048_ppo_head_loss(g2048_stream_t stream, const uint16_t *x, const float *wa, const float *ba, const float *wv,
                        const float *bv, int64_t m, int32_t h, const g2048_ppo_batch *batch, const float *beta_dev,
                        float critic, float clip_eps, int32_t decouple_critic, float *masked, float *dx, float *dz,
                        float *partials, float *dwa, float *dba, float *dwv, float *dbv, float *sums,
                        g2048_colsum_job *defer);

/* KL(old || new) diagnostic after the optimizer step (train.py:578-601): new logits x Wa^T + ba
 * against the stored masked logits (illegal = -inf).  out[2] = {sum KL, max KL} (overwritten).
 * rows (nullable): device count of the valid rows (g2048_ppo_batch.rows). */
int g2048_ppo_head_kl(g2048_stream_t stream, const uint16_t *x, const float *wa, const float *ba, int64_t m,
                      int32_t h, const float *old_masked, const int64_t *rows, float *partials, float *out,
                      g2048_colsum_job *defer);

/* The KL re-forward's last block and heads in one launch (h = 196 ResidualBlock: n = k = 196):
 * Y = x + Dropout(ReLU(LN(x W^T))) as g2048_mlp_fwd (residual, no G / statistics), then instead
 * of storing Y its bf16 values go through the action head (wa [4, 196], ba [4]) and KL(old || new)
 * of every row is reduced like g2048_ppo_head_kl (same partial pairs, out, defer and rows).
 * G2048_EINVAL for any other shape (callers then use g2048_mlp_fwd + g2048_ppo_head_kl). */
int g2048_mlp_fwd_kl(g2048_stream_t stream, const uint16_t *x, const uint16_t *w, const float *gamma,
                     const float *beta, int64_t m, int32_t n, int32_t k, const g2048_dropout *drop, const float *wa,
                     const float *ba, const float *old_masked, const int64_t *rows, float *partials, float *out,
                     g2048_colsum_job *defer);

/* ---- fused forward passes of the minibatch step (csrc/ppo_fused.hip) --------------------------
 * GameMLP (num_layers 2, hidden in {32, 64, 128, 192, 196}) over the minibatch boards[idx[r]] in ONE
 * persistent launch each, on the fused rollout's register hand-off (weights in LDS):
 *   g2048_ppo_forward_loss  the train pass (train.py:491-546): to_model_format -> stem -> 2 blocks with
 *       Dropout(p) of pass 0 -> heads -> the PPO-clip / entropy / smooth-L1 loss and dz.  Replaces
 *       g2048_obs_gather + 3 x g2048_mlp_fwd + g2048_ppo_head_loss (the logits keep the fp32 head weights
 *       through g2048_head_split); its G / H / mean / rstd are bitwise
 *       those of g2048_mlp_fwd.  Writes x0 (bf16 [m,48], optional), g[l] / h[l] (bf16 [m,h], optional
 *       each: h[2] is the head weight-gradient operand), mean[l] / rstd[l] (optional pairs), masked
 *       (fp32 [m,4]), dz (fp32 [m,8], g2048_dy.dz) and dz_bf16 (bf16 [m,16]: dz as two bf16 terms,
 *       hi = bf16(dz) in columns 0..4 and lo = bf16(dz - hi) in 8..12, zeros elsewhere: the operand of
 *       dW_heads = hi^T h[2] + lo^T h[2] on g2048_wgrad, whose [16][h] partial rows summed as 2 nb rows
 *       of 8 h give the fp32-accurate head gradient), and reduces dba [4], dbv [1] and sums [3] =
 *       {sum ppo, sum H, sum v} through g2048_mlp_pass_partials(m, 1) floats of partials.
 *   g2048_ppo_forward_kl  the KL re-forward (train.py:578-601) with the updated weights and the
 *       dropout draw of pass 1 (drop[].pass): KL(old || new) against `masked` (the train pass's
 *       output, read), out[2] = {sum KL, max KL} through g2048_mlp_pass_partials(m, 0) floats.
 * Both take the g2048_ppo_batch conventions (rows: padded ragged minibatch) and the deferred
 * column-sum job (defer, nullable). */
typedef struct g2048_mlp_pass_args {
    const int8_t *boards;          /* [M][16] the flat trajectory's boards (16-byte aligned) */
    g2048_ppo_batch batch;         /* idx (both passes), rows; the loss inputs (train pass) */
    int64_t m;                     /* minibatch rows */
    int32_t hidden, decouple_critic;
    const void *w_stem;            /* bf16 [h][48], 16-byte aligned */
    const void *w_block[2];        /* bf16 [h][h] */
    const float *ln_gamma[3], *ln_beta[3];
    const void *head_frag;         /* g2048_head_split of the current head weights */
    const float *ba, *bv;          /* fp32 head biases (bv: train pass only) */
    g2048_dropout drop[2];         /* blocks 1 and 2 (p == 0: eval-mode blocks) */
    const float *beta_dev;         /* train: the entropy coefficient (device float) */
    float critic, clip_eps;
    void *x0;                      /* train outputs (see above) */
    void *g[3];
    void *h[3];
    float *mean[3], *rstd[3];
    float *masked;                 /* train: out; KL: in */
    float *dz;
    void *dz_bf16;
    float *partials;
    void *keep;                    /* train, optional out: the blocks' dropout keep bits, uint64 [2][m][4]
                                    * (block, row, lane group g: bit 4 n + e = feature 16 n + 4 g + e),
                                    * g2048_ppo_backward's `keep` (8-byte aligned; NULL: not stored) */
    const int64_t *idx_offset;     /* optional device scalar: row r of the minibatch is
                                    * batch.idx[*idx_offset + r] (a whole epoch's permutation in one
                                    * buffer; g2048_ppo_forward_kl_stats advances it) */
} g2048_mlp_pass_args;

/* The head weights [wa (4 rows); wv] (fp32) as the passes' MFMA operand: an exact three-term bf16
 * split laid out in fragment order, g2048_head_split_bytes(h) bytes (16-byte aligned).  Run after
 * every change of the head weights (the optimizer step) and before the passes that read them;
 * wv NULL = zero value rows (the KL pass reads only the action rows). */
size_t g2048_head_split_bytes(int32_t hidden);
int g2048_head_split(g2048_stream_t stream, const float *wa, const float *wv, int32_t hidden, void *frag);
int g2048_mlp_pass_supported(int32_t hidden, int32_t num_layers);
size_t g2048_mlp_pass_partials(int64_t m, int32_t train);
int g2048_ppo_forward_loss(g2048_stream_t stream, const g2048_mlp_pass_args *args, float *dba, float *dbv, float *sums,
                           g2048_colsum_job *defer);
int g2048_ppo_forward_kl(g2048_stream_t stream, const g2048_mlp_pass_args *args, float *out, g2048_colsum_job *defer);
/* The KL re-forward with the minibatch statistics folded in: the pass's last block reduces the KL
 * partial rows and applies g2048_ppo_stats (same arithmetic) -- one launch instead of two.  sync: a
 * 4-byte device word, zero before the first call (each call leaves it zero). */
typedef struct g2048_ppo_stats_args {
    const float *sums;             /* the train pass's loss sums [3] */
    const float *grad_norm;        /* the pre-clip gradient norm (device scalar) */
    const float *beta_dev;
    const int64_t *rows;           /* nullable: the padded ragged minibatch's device row count */
    float *stats;                  /* [9] accumulated (g2048_ppo_stats) */
    uint64_t *counter;             /* nullable: += 1 (the next minibatch's dropout counter) */
    uint32_t *sync;
    float critic;
    int32_t pad_;
    int64_t m;
    int64_t *idx_offset;           /* nullable: += idx_step once the pass is done (the next minibatch) */
    int64_t idx_step;
} g2048_ppo_stats_args;
int g2048_ppo_forward_kl_stats(g2048_stream_t stream, const g2048_mlp_pass_args *args, const g2048_ppo_stats_args *st);

/* The MLP's backward after the train pass, in one launch (replaces the per-layer chain of three
 * g2048_ln_act_bwd and two g2048_linear_dgrad): per row tile the top block's LayerNorm / ReLU /
 * Dropout backward from the heads' share dz W_heads, its input gradient P2 = dG2 W2 (bf16), block
 * 1 from dz W_heads + P2, P1 = dG1 W1, the stem from dz W_heads + P1 + P2 -- P and dy stay in
 * registers.  Writes dG of the three layers (the weight gradients' operands, bitwise the chain's)
 * and the LayerNorm affine gradients (dgamma[l], dbeta[l]; summed in another order than
 * g2048_ln_act_bwd) through per-block partial rows [3][nb][2 h] (g2048_mlp_back_partials floats):
 * immediately, or as three deferred column-sum jobs defer[0..2]. */
typedef struct g2048_mlp_back_args {
    int64_t m;
    int32_t hidden, pad_;
    const void *w_block[2];        /* bf16 [h][h] (blocks 1, 2), 8-byte aligned */
    const float *ln_gamma[3], *ln_beta[3];
    const float *wa, *wv;          /* fp32 heads [4][h], [h] (wv NULL: decoupled critic) */
    const float *dz;               /* fp32 [m][8]: the train pass's head output gradient */
    const void *g[3];              /* bf16 [m][h] pre-norm G of the train pass */
    const float *mean[3], *rstd[3];
    g2048_dropout drop[2];         /* blocks 1, 2: the train pass's draws */
    void *dg[3];                   /* out: bf16 [m][h] */
    void *p_out[2];                /* optional out: bf16 [m][h] P1, P2 (tests) */
    float *partials;
    const void *keep;              /* optional: the train pass's keep bits (g2048_mlp_pass_args.keep) for
                                    * the same drop[] -- read instead of re-drawing the Philox masks */
} g2048_mlp_back_args;
size_t g2048_mlp_back_partials(int64_t m, int32_t hidden);
int g2048_ppo_backward(g2048_stream_t stream, const g2048_mlp_back_args *args, float *const *dgamma,
                       float *const *dbeta, g2048_colsum_job *defer);

/* Accumulates one minibatch into the update statistics (train.py:603-642): stats[0..7] +=
 * {loss, policy_loss, entropy_loss, value_loss, grad_norm, entropy, kl_total, kl_average} from the
 * head_loss sums, the KL {sum, max}, the pre-clip gradient norm and beta; stats[8] = max(stats[8],
 * KL max).  counter (optional) is incremented (the next minibatch's dropout counter).  kl is either
 * the final {sum, max} (kl_rows = 0) or the [kl_rows][2] partial rows of a deferred
 * g2048_ppo_head_kl (its job's part / nb), reduced here in a fixed order.  The means are over m rows,
 * or over *rows (device count, nullable) for a padded ragged minibatch. */
int g2048_ppo_stats(g2048_stream_t stream, const float *sums, const float *kl, int32_t kl_rows, const float *grad_norm,
                    const float *beta_dev, float critic, int64_t m, const int64_t *rows, float *stats,
                    uint64_t *counter);

/* The four weight gradients of the GameMLP minibatch backward in ONE launch (mlp_wgrad.hip):
 *   out_head [16][h] = dz_bf16^T H2   (dz as two bf16 terms: hi in rows 0-4, lo in rows 8-12)
 *   out_w[0] [h][48] = dg[0]^T x[0]    (the stem: x[0] = the bf16 observations [m][48])
 *   out_w[l] [h][h]  = dg[l]^T x[l]    (block l = 1, 2: x[l] = the block's input H_{l-1})
 * Every operand bf16 row-major with m rows, 16-byte aligned; h in {196, 192, 128, 64, 32}.  The CUs
 * split the products' rows in proportion to their bytes; each block writes an fp32 partial that
 * g2048_colsum_batch sums in a fixed order: `defer` (4 jobs: head, stem, block 1, block 2) receives
 * those jobs instead of summing at once.  Replaces g2048_wgrad (head, stem) + g2048_wgrad_pair. */
typedef struct g2048_mlp_wgrad_args {
    int64_t m;
    int32_t hidden, pad_;
    const void *dz_bf16;           /* [m][16] */
    const void *h2;                /* [m][h]  block 2's output */
    const void *dg[3];             /* [m][h]  the train step's dG of the stem, block 1, block 2 */
    const void *x[3];              /* the layers' inputs: x0 [m][48], H0 [m][h], H1 [m][h] */
    float *partials;               /* g2048_mlp_wgrad_partials(m, hidden) floats */
} g2048_mlp_wgrad_args;
size_t g2048_mlp_wgrad_partials(int64_t m, int32_t hidden);
int g2048_mlp_wgrad(g2048_stream_t stream, const g2048_mlp_wgrad_args *args, float *out_head, float *const *out_w,
                    g2048_colsum_job *defer);

/* Scratch floats of g2048_wgrad for (m, n1, n2); 0 when the shape is unsupported. */
size_t g2048_wgrad_partials(int64_t m, int32_t n1, int32_t n2);

/* Weight gradient of a Linear layer: out[n1][n2] = sum_{r<m} a[r][n1] b[r][n2] (out = dG^T X with
 * a = dG bf16 [m,n1], b = X bf16 [m,n2]), fp32 accumulate on bf16 MFMA, fp32 out (overwritten).
 * n1, n2 % 4 == 0 and <= 224. */
int g2048_wgrad(g2048_stream_t stream, const uint16_t *a, const uint16_t *b, int64_t m, int32_t n1, int32_t n2,
                float *partials, float *out, g2048_colsum_job *defer);

/* Two weight gradients of the same shape in ONE launch (out0 = a0^T b0, out1 = a1^T b1; the fused
 * backward's two block layers): twice the rows per block of g2048_wgrad, so half its partial rows
 * for the same CU count; partials* each g2048_wgrad_pair_partials floats; defer: two jobs. */
size_t g2048_wgrad_pair_partials(int64_t m, int32_t n1, int32_t n2);
int g2048_wgrad_pair(g2048_stream_t stream, const uint16_t *a0, const uint16_t *b0, const uint16_t *a1,
                     const uint16_t *b1, int64_t m, int32_t n1, int32_t n2, float *partials0, float *partials1,
                     float *out0, float *out1, g2048_colsum_job *defer);

/* Input gradient of a Linear layer: out = dg w  (dg bf16 [m, n] = dL/d(output), w bf16 [n, k] = the
 * weight [out, in], out bf16 [m, k] = dL/d(input), fp32 accumulate on bf16 MFMA, one rounding)
 * -- the `dG W` GEMM of the backward pass (replaces the library GEMM).  Square layers with
 * n = k in {64, 128, 196} (where it beats the library); dg / out 8-byte aligned. */
int g2048_linear_dgrad_supported(int32_t n, int32_t k);
int g2048_linear_dgrad(g2048_stream_t stream, const uint16_t *dg, const uint16_t *w, uint16_t *out, int64_t m,
                       int32_t n, int32_t k);

/* ---- optimizer step (train.py:553-568, :1587-1612) ------------------------------------------ */

/* clip_grad_norm_ of the flat gradient bucket, without touching it: norm_out = ||grad||,
 * coef_out = min(max_norm / (norm + 1e-6), 1) (device scalars read by the optimizer kernels).
 * grad 16-byte aligned; partials: 64 floats of scratch. */
int g2048_grad_clip(g2048_stream_t stream, const float *grad, int64_t n, float max_norm, float *norm_out,
                    float *coef_out, float *partials);

/* One Muon-optimised weight matrix (torch.optim.Muon, adjust_lr_fn="match_rms_adamw"). */
typedef struct g2048_muon_matrix {
    float *param;          /* [rows, cols] fp32, updated in place */
    const float *grad;     /* [rows, cols] fp32 (multiplied by *clip_coef_dev when given) */
    float *momentum;       /* [rows, cols] fp32 momentum buffer */
    uint16_t *param_bf16;  /* optional: bf16 copy of the updated weight */
    void *head_frag;       /* optional: a head matrix ([wa] or [wv], cols = h): the updated weight's
                            * three-term bf16 split written into rows frag_row .. frag_row + rows - 1
                            * of g2048_head_split's fragment image (its other bytes untouched) */
    int32_t rows, cols;
    int32_t lr_index;      /* this matrix's learning rate is lr_dev[lr_index] */
    int32_t frag_row;      /* the first head row of this matrix in head_frag (wa: 0, wv: 4) */
} g2048_muon_matrix;

typedef struct g2048_muon_cfg {
    float momentum, weight_decay, ns_a, ns_b, ns_c, ns_eps;
    int32_t ns_steps, nesterov;
    /* parts > 1 with a workspace: every 196 x 196 / 192 x 192 matrix runs on `parts` blocks (CUs, 7 <=
     * parts <= 13) that split the row blocks of the Newton-Schulz products and exchange X once per
     * iteration through the workspace (g2048_muon_workspace_bytes(), device memory, ZERO-FILLED ONCE
     * by the caller: each launch leaves its counters zero again).  parts <= 1 or workspace NULL: one
     * block per matrix.  The parts poll each other, so the grid must be resident at once: a device
     * with fewer CUs than the split grid needs runs every matrix on one block instead.  A poll that
     * gives up (~0.2 s: a part never became resident) leaves that launch's results garbage and adds
     * one to the workspace's sticky timeout count (g2048_muon_error_offset()), which only the caller
     * clears: read it and fail (FusedMuonAdamW.check_errors, with the train step's metrics). */
    int32_t parts;
    int32_t npartials;             /* the clip's sum-of-squares partials: 0 = g2048_grad_sumsq's 64, else
                                    * this many (g2048_colsum_batch_sq's, <= G2048_COLSUM_SQ_MAX) */
    void *workspace;
} g2048_muon_cfg;

size_t g2048_muon_workspace_bytes(void);

/* Byte offset in the Muon workspace of the uint32 count of timed-out hand-off waits (sticky across
 * launches; zero = every multi-CU Newton-Schulz so far was valid). */
size_t g2048_muon_error_offset(void);

/* Test hook: fill every CU's LDS with `word` (two 1024-thread blocks of the whole LDS per CU), so a
 * following kernel that reads LDS it did not write sees that pattern (a NaN bit pattern makes such a
 * read visible in its results).  Used by tests/test_gpu_ppo_fused.py; no part of the update. */
int g2048_lds_poison(g2048_stream_t stream, uint32_t word);

/* 1 if a [rows, cols] matrix fits the one-block-per-matrix Newton-Schulz kernel (min dim <= 224,
 * max dim <= 256, both LDS images <= ~159 KB: h <= 196 for square weights; rows of a length that
 * is not a multiple of 4 -- GameURM's [64, 3] stem -- take a per-element momentum / update pass). */
int g2048_muon_supported(int32_t rows, int32_t cols);

/* Muon step of up to 16 matrices (GameMLP: 5, GameURM: 11), all concurrently: momentum (nesterov), Newton-Schulz
 * orthogonalisation in bf16 (ns_steps iterations of X <- a X + (b G + c G^2) X, G = X X^T, on the
 * wide orientation), decoupled weight decay, update scaled by 0.2 sqrt(max(rows, cols)). */
int g2048_muon_step(g2048_stream_t stream, const g2048_muon_matrix *mats, int32_t count, const float *lr_dev,
                    const float *clip_coef_dev, const g2048_muon_cfg *cfg);

/* The clip folded into the Muon launch (one launch fewer per optimizer step): g2048_grad_sumsq
 * writes the 64 partial sums of squares of the flat gradient; g2048_muon_step_clip then computes
 * ||g|| and the clip coefficient from them in every block exactly like g2048_grad_clip, block 0
 * publishes them to norm_out / coef_out (device scalars read by g2048_adamw_step after it). */
int g2048_grad_sumsq(g2048_stream_t stream, const float *grad, int64_t n, float *partials);
int g2048_muon_step_clip(g2048_stream_t stream, const g2048_muon_matrix *mats, int32_t count, const float *lr_dev,
                         const float *partials, float max_norm, float *norm_out, float *coef_out,
                         const g2048_muon_cfg *cfg);

/* One flat group of 1-D parameters for AdamW (torch.optim.AdamW, decoupled weight decay). */
typedef struct g2048_adamw_group {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    int64_t n;
    int32_t lr_index;
    int32_t pad_;
} g2048_adamw_group;

/* AdamW step of up to 4 groups; *step_dev is the (already incremented) step count. */
int g2048_adamw_step(g2048_stream_t stream, const g2048_adamw_group *groups, int32_t count, const float *lr_dev,
                     const float *step_dev, const float *clip_coef_dev, float beta1, float beta2, float eps,
                     float weight_decay);

/* The whole clipped optimizer step in two launches: g2048_grad_sumsq_tick = g2048_grad_sumsq plus
 * *step_dev += 1 (the AdamW step count, train.py's optimizer.step bookkeeping); then
 * g2048_muon_adamw_step_clip = g2048_muon_step_clip whose launch also carries the AdamW update of
 * the 1-D groups (extra blocks deriving the clip coefficient from the same partials; *step_dev is
 * the incremented count).  Replaces g2048_muon_step_clip + a step increment + g2048_adamw_step. */
int g2048_grad_sumsq_tick(g2048_stream_t stream, const float *grad, int64_t n, float *partials, float *step_dev);
int g2048_muon_adamw_step_clip(g2048_stream_t stream, const g2048_muon_matrix *mats, int32_t count,
                               const g2048_adamw_group *groups, int32_t ngroups, const float *lr_dev,
                               const float *step_dev, const float *partials, float max_norm, float *norm_out,
                               float *coef_out, const g2048_muon_cfg *cfg, float beta1, float beta2, float eps,
                               float adam_weight_decay);

/* Test hook: the dropout keep mask (uint8 [m,h], 1 = kept) g2048_ln_act_fwd applies. */
int g2048_dropout_mask(g2048_stream_t stream, int64_t m, int32_t h, const g2048_dropout *drop, uint8_t *mask);

#ifdef __cplusplus
}
#endif

#endif /* G2048_PPO_H */
