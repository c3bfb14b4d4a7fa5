/*
 * g2048.h -- C ABI of libg2048.so, the MI355X (gfx950) implementation of RobotSail/2048-PPO's
 * data-parallel hot path: the vectorised 2048 board step and the per-env reward / return-to-go scan.
 *
 * The reference is pure Python and has no FFI of its own; each entry point below replaces the
 * reference function named in its comment, batched over N independent envs.  The Python seam a
 * maintainer would bind these through (ctypes) is 2048-ppo_amd/g2048/_lib.py; the drop-in module
 * the reference itself imports for this path is `batched_rollout.play_games_batched`
 * (train.py:30, :1676-1679, :2034).  See INTEGRATION.md.
 *
 * Conventions (all entry points):
 *   - Every pointer argument is a DEVICE pointer owned by the caller, except `const g2048_rng*`
 *     / `const g2048_reward_cfg*`, which are host structs read during the call.
 *   - Work is enqueued on `stream` (a hipStream_t; NULL = the legacy default stream) and is
 *     asynchronous.  No allocation, no host synchronisation: every call is hipGraph-capturable.
 *   - Return 0 on success, G2048_EINVAL for a bad argument (nothing enqueued), or the positive
 *     hipError_t of a failed launch.
 *   - No global mutable state: calls on different streams are independent.
 *
 * Data layout:
 *   board    int8[16] per env, row-major exponents (0 = empty, k = tile 2^k), 16-B aligned rows of
 *            the [N,16] array -- one 16-B load per lane.  game.py's Grid[i][j] == board[4*i+j].
 *   action   uint8 per env: 0 UP, 1 DOWN, 2 LEFT, 3 RIGHT (GameMLP.directions, game.py:1087-1092).
 *   flags    uint8 per env: bits 0-3 legal-action mask of the board written back (bit a = action a
 *            is legal), bit 4 the requested action was illegal (no-op, game.py:959-978), bit 5 the
 *            env was auto-reset, bit 6 env inactive (episodic mode, already finished), bit 7 done.
 *   pot      int8[4] per env: {monotonicity_before, monotonicity_after, emptiness_before,
 *            emptiness_after} as game.step reports them (game.py:985-1000); zero on an illegal
 *            action like game.py:972-976.
 *   Trajectory buffers of the reward scan are time-major [T][N].
 */
#ifndef G2048_H
#define G2048_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t *g2048_stream_t; /* == hipStream_t */

#define G2048_OK 0
#define G2048_EINVAL (-1)

#define G2048_UP 0
#define G2048_DOWN 1
#define G2048_LEFT 2
#define G2048_RIGHT 3

#define G2048_FLAG_LEGAL_MASK 0x0Fu
#define G2048_FLAG_INVALID 0x10u
#define G2048_FLAG_RESET 0x20u
#define G2048_FLAG_INACTIVE 0x40u
#define G2048_FLAG_DONE 0x80u

/* Spawn / action randomness. */
#define G2048_RNG_PHILOX 0  /* Philox4x32-10, stateless: key = seed, counter = {step, env, stream} */
#define G2048_RNG_MT19937 1 /* per-env CPython random.Random stream: bit-exact with game.py spawns */
#define G2048_RNG_INJECT 2  /* spawn draws supplied by the caller: inject[i] = {k-th empty, exponent} */

typedef struct g2048_rng {
    int32_t mode;               /* G2048_RNG_* */
    uint32_t env_base;          /* global id of env 0 of this call (shard / rank offset) */
    uint64_t seed;              /* Philox key */
    uint64_t counter;           /* Philox step counter (added to *counter_dev when that is set) */
    const uint64_t *counter_dev; /* optional device counter base, so graph replays advance */
    uint32_t *mt_state;         /* MT19937: device words [625][N] (word-major), see g2048_mt_seed */
    const int32_t *inject;      /* INJECT: device [N][2] */
} g2048_rng;

/* Options of g2048_env_step. */
#define G2048_OPT_AUTO_RESET 0x1u /* a finished env is reset in the same launch (fixed-horizon mode) */
#define G2048_OPT_SKIP_DONE 0x2u  /* an env whose board has no legal move is left untouched and
                                     flagged inactive (episodic mode: one game per env) */

/* Words of MT19937 state per env (624 state words + the index). */
size_t g2048_mt_state_words(void);

/* random.seed(seed[i]) for every env: CPython init_by_array seeding, seeds < 2**64.
   Replaces the `random.seed(seed)` of train.py:227-228 per env. */
int g2048_mt_seed(g2048_stream_t stream, uint32_t *mt_state, const uint64_t *seeds, int64_t n);

/* Game2048.reset (game.py:942-950): zero board + two spawns.  `where` (nullable) restricts the
   reset to envs with where[i] != 0.  Writes the legal mask of the new board into flags. */
int g2048_env_reset(g2048_stream_t stream, int8_t *boards, uint8_t *flags, const uint8_t *where,
                    int64_t n, const g2048_rng *rng);

/* Game2048.step (game.py:952-1030) for N envs, one 16-B board per lane:
   legality of the action, potentials before, slide/merge (simulate_move game.py:122-160), points
   (game.py:237), max tile created, potentials after (pre-spawn), spawn (_add_tile game.py:923-940),
   done = no legal move (game.py:1006), next legal mask.  boards_in may equal boards_out.
   actions_in == NULL draws a uniform random legal action (Philox stream 1) -- the synthetic
   benchmark policy; actions_out (nullable) records the action taken.  max_tile / pot nullable. */
int g2048_env_step(g2048_stream_t stream, const int8_t *boards_in, int8_t *boards_out,
                   const uint8_t *actions_in, uint8_t *actions_out, int32_t *points, int8_t *max_tile,
                   int8_t *pot, uint8_t *flags, int64_t n, const g2048_rng *rng, uint32_t options);

/* Synthetic random-action rollout (the BASELINE.md throughput workload): `steps` consecutive
   Game2048.step calls per env in ONE launch, board held in registers, uniform random legal actions
   (Philox stream 1), auto-reset on done.  Step t uses Philox counter rng->counter + t (+ *counter_dev):
   words x/y/z give the action and the spawn; a game that ends at step t restarts from the 4th words
   of the draws of steps t and t+1 (oracle or_reset_words).  1 <= N < 2^28 (0 is a no-op).
   Time-major trajectory records (all required): traj_boards [steps][N][16] = the board the action
   was taken on, traj_actions/traj_flags [steps][N] uint8, traj_points [steps][N] int32,
   traj_pot [steps][N][4] int8.  boards [N,16] is read at the start and written at the end.
   Replaces the per-env `play` / random-agent loop of train.py:2184-2297 batched over N envs. */
int g2048_env_rollout_random(g2048_stream_t stream, int8_t *boards, int64_t n, int64_t steps,
                             int8_t *traj_boards, uint8_t *traj_actions, int32_t *traj_points,
                             int8_t *traj_pot, uint8_t *traj_flags, const g2048_rng *rng);

/* g2048_env_rollout_random that also advances the Philox counter base: *rng->counter_dev += steps
   once the whole launch has read it (the last workgroup to finish adds; `ticket` is a ZERO-FILLED
   uint32 device word, left zero again by every launch).  rng->counter_dev is required (8-byte
   aligned, writable).  A graph of K such launches replays K consecutive chunks with no counter-bump
   kernel between them (bench.py's rollout leg). */
int g2048_env_rollout_random_adv(g2048_stream_t stream, int8_t *boards, int64_t n, int64_t steps, int8_t *traj_boards,
                                 uint8_t *traj_actions, int32_t *traj_points, int8_t *traj_pot, uint8_t *traj_flags,
                                 const g2048_rng *rng, uint32_t *ticket);

/* Game2048.preview_move_rewards (game.py:167-184): points4[i] = merge points of UP, DOWN, LEFT,
   RIGHT on board i, 0 for an illegal direction.  points4 is int32 [N][4], 16-B aligned. */
int g2048_preview_points(g2048_stream_t stream, const int8_t *boards, int32_t *points4, int64_t n);

/* Legal-action mask per board (can_move_in_direction || can_merge_in_direction,
   game.py:260-330 / current_valid_directions game.py:295-299) into flags bits 0-3, done bit 7. */
int g2048_legal_mask(g2048_stream_t stream, const int8_t *boards, uint8_t *flags, int64_t n);

/* Game2048.to_model_format (game.py:92-101): [N,48] = (e, row/3, col/3) per cell.
   dtype 0 = float32, 1 = bfloat16 (round-to-nearest-even). */
#define G2048_DTYPE_F32 0
#define G2048_DTYPE_BF16 1
int g2048_obs_encode(g2048_stream_t stream, const int8_t *boards, void *obs, int32_t dtype, int64_t n);

/* The rollout's action choice (train.py:266-291, :326): mask illegal logits to -inf, softmax,
   sample (Philox stream 1 inverse CDF; torch.multinomial's stream is not reproducible), entropy
   -sum p log p over p > 0, and log_softmax of the masked logits (-inf where illegal).
   logits (float32, row stride `logits_stride` floats, NULL = uniform over legal actions).
   The legal mask is read from flags bits 0-3.  logp [N,4] and entropy [N] are nullable. */
int g2048_sample_actions(g2048_stream_t stream, const float *logits, int64_t logits_stride,
                         const uint8_t *flags, uint8_t *actions, float *logp, float *entropy, int64_t n,
                         const g2048_rng *rng);

/* ---- return-to-go / advantage (calculate_advantage, train.py:651-904) ------------------------ */

/* Moment state, 8 doubles on the device:
   [0] rtg_mu  [1] rtg_m2  [2] rtg_first_moment  [3] rtg_step (train_step + 1)
   [4] mu_corrected  [5] stddev (written by g2048_rtg_prepare)  [6] batch mean  [7] batch var
   Initial state of train.py:1550-1552: {0, 1, 0, 1, ...}. */
#define G2048_RTG_STATE_DOUBLES 8

typedef struct g2048_reward_cfg {
    double gamma;    /* --gamma */
    double w_points; /* --points */
    double w_mono;   /* --mono */
    double w_empt;   /* --emptiness */
    double beta;     /* --rtg-beta */
} g2048_reward_cfg;

/* bias-corrected mean / stddev from the PREVIOUS moments (train.py:746-754). */
int g2048_rtg_prepare(g2048_stream_t stream, double *state, const g2048_reward_cfg *cfg);

/* Per-env reverse scan over a [T][N] trajectory (train.py:699-772):
   r = w_p*points + w_m*(gamma*mono_a - mono_b) + w_e*(gamma*empt_a - empt_b), after-potentials
   zeroed on the done step (train.py:318,322); G_t = r_t + gamma*G_{t+1}, reset after done, 0
   beyond the horizon; G_norm = (G - mu_c)/(std + 1e-8); adv = G_norm - value.  Arithmetic in
   float64, outputs float32.  Steps flagged inactive are skipped (outputs 0, not counted).
   Writes the batch sums {sum(G-mu_c), sum((G-mu_c)^2), count} to partials[3] (float64), for an
   optional cross-rank all-reduce before g2048_rtg_finalize.  `workspace` must hold
   g2048_reward_rtg_workspace_bytes(n) bytes. */
size_t g2048_reward_rtg_workspace_bytes(int64_t n);
int g2048_reward_rtg(g2048_stream_t stream, const int32_t *points, const int8_t *pot,
                     const uint8_t *flags, const float *value, int64_t T, int64_t n,
                     const g2048_reward_cfg *cfg, const double *state, float *g_raw, float *g_norm,
                     float *adv, double *partials, void *workspace, size_t workspace_bytes);
/* g2048_reward_rtg plus the per-step reward itself (train.py:702-719, float64, bit-identical to the
 * reference's Python floats; 0 on inactive steps) into reward [T][n] when it is not NULL. */
int g2048_reward_rtg_ex(g2048_stream_t stream, const int32_t *points, const int8_t *pot,
                        const uint8_t *flags, const float *value, int64_t T, int64_t n,
                        const g2048_reward_cfg *cfg, const double *state, float *g_raw, float *g_norm,
                        float *adv, double *reward, double *partials, void *workspace,
                        size_t workspace_bytes);

/* The info-only heuristic deltas of Game2048.step (game.py:981-1002; smoothness :339-357, corner
 * :359-399, adjacency :401-442, monotonic chain :444-506, topological with the pre-move anchor
 * corner :610-668 / :802-921): for board i [n][16] and action i [n], deltas[5 i + k] = heuristic k
 * after the move (pre-spawn) minus before, k = {smoothness, corner, adjacency, chain, topological}
 * (all 0 for an illegal action, game.py:959-978), float64 bit-identical to the reference;
 * anchor[i] (optional) = the anchor corner as 4 row + col.  They never reach the reward
 * (train.py:702-719): the EpisodeData records, breakdown tables and viz export use them. */
int g2048_info_deltas(g2048_stream_t stream, const int8_t *boards, const uint8_t *actions, double *deltas,
                      int8_t *anchor, int64_t n);

/* Episode statistics of a fixed-horizon rollout (compute_batch_stats' scores and tiles,
 * train.py:1040-1120): per env, the running score / max tile exponent of its current game is
 * carried across calls in run_score [n] / run_max [n]; scores[t][e] / tiles[t][e] are the finished
 * game's final score and max tile where step t ends a game (FLAG_DONE, not INACTIVE), else -1.
 * points / max_tile / step_flags [T][n]; boards [T][n][16] (the board before each step). */
int g2048_episode_scan(g2048_stream_t stream, const int32_t *points, const int8_t *boards, const int8_t *max_tile,
                       const uint8_t *step_flags, int64_t T, int64_t n, int64_t *run_score, int32_t *run_max,
                       int64_t *scores, int32_t *tiles);

/* The rollout half of a train step's metrics (train.py:1700-1760's reward / advantage / return
 * summaries and compute_batch_stats' finished games, train.py:1040-1120) in two launches, no host
 * sync.  out[23] (float32) = {rows, reward mean, reward var, zero-reward %, adv mean, adv var,
 * adv L2, adv min, adv max, G_norm mean, G_norm std, G_norm min, G_norm max, G_raw std, value
 * std, mean G_raw of episode starts, finished-score mean, lower median (-1: none), max (-1: none),
 * % finished with max tile >= 512 / 1024 / 2048, finished count}; variances are population ones,
 * sums in float64.  The reward is the float32 metric r = w_p points + w_m (gamma pot1 (1-done) -
 * pot0) + w_e (gamma pot3 (1-done) - pot2) over pot [T][n][4] int8 (4-B aligned).
 * episodic = 0 (fixed horizon): every row counts; the finished games are episode_scan's (run_score
 * / run_max carried, boards [T][n][16] = the board before each step, max_tile [T][n]); episode
 * starts are the steps after a FLAG_RESET.  episodic = 1: rows flagged INACTIVE are skipped; each
 * env is one finished game (its active points, the max tile of boards[T], boards [T+1][n][16]);
 * starts are t = 0; max_tile / run_* unused.  workspace: g2048_rollout_stats_workspace_bytes(T, n)
 * bytes, 16-B aligned; its first 4 bytes (the finished-key counter) must be zero on entry, and
 * every call leaves them zero (zero-fill the workspace once when allocating it). */
size_t g2048_rollout_stats_workspace_bytes(int64_t T, int64_t n);
int g2048_rollout_stats(g2048_stream_t stream, const int32_t *points, const int8_t *pot, const uint8_t *step_flags,
                        const float *value, const float *g_raw, const float *g_norm, const float *adv,
                        const int8_t *boards, const int8_t *max_tile, int64_t T, int64_t n, int32_t episodic,
                        const g2048_reward_cfg *cfg, int64_t *run_score, int32_t *run_max, void *workspace,
                        size_t workspace_bytes, float *out);

/* The PPO update's per-epoch minibatch order (DataLoader(shuffle=True), train.py:470; replaces
 * torch.randperm, a 4 M-key radix sort): out[i] (int64, i < n < 2^31) = a keyed Feistel bijection of
 * [0, n) (4 rounds over [0, 4^k) >= n, cycle-walked), round keys Philox-drawn from (*key_dev if
 * key_dev is non-NULL -- a device int64, e.g. a draw of the caller's generator, so no host read --
 * else seed, counter).  One launch, no workspace. */
int g2048_permutation(g2048_stream_t stream, int64_t *out, int64_t n, const int64_t *key_dev, uint64_t seed,
                      uint64_t counter);

/* EMA moment update with the batch statistics (train.py:898-901); advances rtg_step. */
int g2048_rtg_finalize(g2048_stream_t stream, double *state, const double *partials,
                       const g2048_reward_cfg *cfg);

/* D4 up-sampling of training samples on the device (calculate_advantage's augmentation,
 * train.py:774-881; mirror_grid / rotate_grid game.py:509-590).  Replaces the host loop over
 * random.sample(...) with:  sample j < k -> source row perm(j) of a keyed 4-round Feistel
 * permutation of [0, n) (cycle-walked: k DISTINCT rows, like random.sample); per sample the Philox
 * draw (seed, counter, j, stream 3) = {x, y, z, w}: x < 2^31 -> a mirror copy (y < 2^31 horizontal =
 * flip columns, else vertical = flip rows); independently z < 2^31 -> a rotation copy by
 * 90 * (1 + floor(3 w / 2^32)) degrees clockwise.  Copies are appended after the n real rows of the
 * sample pool, sample by sample, mirror before rotation; each copy remaps the board, the action,
 * bits 0-3 of legal (the other flag bits are kept) and the 4 old log-probs (new[remap(d)] = old[d],
 * train.py:810-824), and copies adv / ret.  Pool arrays (capacity >= n + 2k rows): boards [.,16]
 * int8, actions / legal [.] uint8, logp [.,4] f32, adv / ret [.] f32.  *count (device int64) =
 * n + number of copies.  Needs n < 2^31, k <= n, workspace of g2048_augment_workspace_bytes(k). */
size_t g2048_augment_workspace_bytes(int64_t k);
int g2048_augment(g2048_stream_t stream, int8_t *boards, uint8_t *actions, uint8_t *legal, float *logp, float *adv,
                  float *ret, int64_t n, int64_t k, uint64_t seed, uint64_t counter, void *workspace,
                  size_t workspace_bytes, int64_t *count);

/* Library build identification (gfx target, version). */
const char *g2048_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* G2048_H */
