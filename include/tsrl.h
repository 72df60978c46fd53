/*
 * libtsrl -- C ABI of the MI355X (gfx950) on-policy hot path:
 * rollout storage (VectorReplayBuffer), GAE reverse scan, PPO clipped-surrogate loss.
 *
 * The reference (tianshou 0.5.1) is pure Python; its "operators" for this path are the
 * Python methods listed against each entry point below.  tianshou_amd (the host package
 * under tianshou-fork_amd/) binds these symbols with ctypes and keeps the reference's
 * class API on top.
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer owned by the caller (PyTorch allocates).  Kernels
 *     never allocate; scratch comes from a caller buffer sized by *_workspace_bytes().
 *   - `stream` is a hipStream_t passed as void*; every call is stream-ordered and
 *     asynchronous; no call synchronises the device or the host.
 *   - Return value: 0 on success, otherwise a hipError_t code; tsrl_last_error() returns
 *     a thread-local message.  Argument errors return hipErrorInvalidValue (1).
 *   - No global mutable state; calls are reentrant.
 */
#ifndef TSRL_H_
#define TSRL_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Library identification / errors. */
const char* tsrl_version(void);
const char* tsrl_last_error(void);

/* ---------------------------------------------------------------------------------
 * GAE reverse scan.
 * Replaces BasePolicy.compute_episodic_return (tianshou/policy/base.py:337-384) and the
 * numba kernel _gae_return (tianshou/policy/base.py:453-497), with the value handling of
 * A2CPolicy._compute_returns (tianshou/policy/modelfree/a2c.py:83-117).
 *
 *   v_next_masked = v_s_ * !terminated                 (value_mask, base.py:317-335)
 *   end_i   = terminated_i | truncated_i | end_extra_i | ((i+1) % row_len == 0)
 *   delta_i = rew_i + v_next_masked_i * gamma - v_s_i  (f32 product when value_scale==NULL,
 *             f64 with v = (double)v * (*value_scale) otherwise: the rew_norm path)
 *   adv_i   = delta_i + (1 - end_i) * gamma * lambda * adv_{i+1}   (f64, no FMA)
 *   ret_i   = adv_i + v_s_i ;  ret_i /= *value_scale in rew_norm mode (a2c.py:110-111)
 *
 * row_len > 0 declares that every row_len-th element closes an episode segment (the
 * VectorReplayBuffer sample(0) layout: each env's segment ends at its unfinished/last
 * index, manager.py:68-74); the scan then runs independent row ranges in one pass.
 * row_len == 0 runs the general 3-phase scan (needs workspace).
 * Any of adv_out/ret_out/adv64_out/ret64_out may be NULL.  ret_partials (nullable,
 * rew_norm only) receives per-workgroup (count, mean, M2) of the UNNORMALISED f64 returns
 * for tsrl_ret_rms_update (RunningMeanStd.update, tianshou/utils/statistics.py:93-114).
 * ------------------------------------------------------------------------------- */
int64_t tsrl_gae_workspace_bytes(int64_t n, int64_t row_len);
int64_t tsrl_gae_num_partials(int64_t n, int64_t row_len);
int tsrl_gae(const float* v_s, const float* v_s_next, const double* rew,
             const uint8_t* terminated, const uint8_t* truncated, const uint8_t* end_extra,
             int64_t n, int64_t row_len, const double* value_scale, double gamma,
             double gae_lambda, float* adv_out, float* ret_out, double* adv64_out,
             double* ret64_out, double* ret_partials, void* workspace,
             int64_t workspace_bytes, void* stream);

/* Same scan with f64 value inputs and f64 outputs only (the public
 * compute_episodic_return on NumPy f64 values, base.py:337-384). */
int tsrl_gae_f64v(const double* v_s, const double* v_s_next, const double* rew,
                  const uint8_t* terminated, const uint8_t* truncated, const uint8_t* end_extra,
                  int64_t n, int64_t row_len, double gamma, double gae_lambda,
                  double* adv64_out, double* ret64_out, void* workspace,
                  int64_t workspace_bytes, void* stream);

/* Diagnostic (bench.py's roofline): the next row-path (row_len > 0) tsrl_gae call of this host
 * thread launches its kernel with hipExtLaunchKernel, which records the kernel's own start /
 * stop timestamps into these two HIP events (hipEvent_t, created with timing); NULL, NULL
 * clears.  The 3-phase general path ignores them. */
int tsrl_gae_time_next(void* start_event, void* stop_event);

/* Merge (count, mean, M2) partials into a RunningMeanStd held on device as
 * double rms[3] = {mean, var, count}  (statistics.py:93-114, Chan parallel merge). */
int tsrl_ret_rms_update(const double* partials, int64_t nparts, double* rms, void* stream);

/* ---------------------------------------------------------------------------------
 * Device synthetic vector env (oracle/synth_env.py restates it).
 * Stands behind BaseVectorEnv.step/reset (tianshou/env/venvs.py:260-381).
 * Rows r < k act on env ids[r] (ids NULL -> env r).  step() writes raw obs rows,
 * rew (f64), terminated/truncated (u8), and per-block column partial sums
 * (sum, sumsq as f64, layout [nblk][dim][2]) for the VectorEnvNormObs update;
 * reset() does the same for rows with mask[r] != 0 only (mask NULL -> all rows).
 * ------------------------------------------------------------------------------- */
int64_t tsrl_env_num_partials(int64_t k);
int tsrl_synth_box_step(const int64_t* ids, int64_t k, int64_t dim, uint64_t seed,
                        int64_t ep_len, int64_t* ep_j, int64_t* ep_t, float* obs_out,
                        double* rew_out, uint8_t* term_out, uint8_t* trunc_out,
                        double* col_partials, void* stream);
/* Step every env (ids = identity) and reset the finished ones in the same launch: step rows
 * -> obs_out with partials_step over all k rows; finished rows (done_out) -> reset_out with
 * partials_reset over those rows only and blk_done[nblk] = finished rows per partial block
 * (partials / blk_done all NULL when no obs normalisation is attached). */
int tsrl_synth_box_step_reset(int64_t k, int64_t dim, uint64_t seed, int64_t ep_len,
                              int64_t* ep_j, int64_t* ep_t, float* obs_out, float* reset_out,
                              double* rew_out, uint8_t* term_out, uint8_t* trunc_out,
                              uint8_t* done_out, double* partials_step,
                              double* partials_reset, double* blk_done, void* stream);
/* The action-coupled env (SyntheticVectorEnv(act_coef=c), synth.h coupled_val): the step rows
 * read act[k, act_dim] (the remapped actions): obs = f32(box + f32(c * act[r][d mod act_dim]));
 * reset rows are unchanged.  act NULL = the plain calls above. */
int tsrl_synth_box_step_act(const int64_t* ids, int64_t k, int64_t dim, uint64_t seed,
                            int64_t ep_len, int64_t* ep_j, int64_t* ep_t, float* obs_out,
                            double* rew_out, uint8_t* term_out, uint8_t* trunc_out,
                            double* col_partials, const float* act, int64_t act_dim,
                            float act_coef, void* stream);
int tsrl_synth_box_step_reset_act(int64_t k, int64_t dim, uint64_t seed, int64_t ep_len,
                                  int64_t* ep_j, int64_t* ep_t, float* obs_out,
                                  float* reset_out, double* rew_out, uint8_t* term_out,
                                  uint8_t* trunc_out, uint8_t* done_out, double* partials_step,
                                  double* partials_reset, double* blk_done, const float* act,
                                  int64_t act_dim, float act_coef, void* stream);
int tsrl_synth_box_reset(const int64_t* ids, const uint8_t* mask, int64_t k, int64_t dim,
                         uint64_t seed, int64_t ep_len, int64_t* ep_j, int64_t* ep_t,
                         float* obs_out, double* col_partials, void* stream);
/* u8 observations of obs_bytes per row; frame_stack S > 1 emulates gymnasium's FrameStack:
 * the row is S frames of obs_bytes/S, frame q = the frame of episode time
 * max(t - (S-1-q), episode start) (a reset repeats its first frame S times). */
int tsrl_synth_u8_step(const int64_t* ids, int64_t k, int64_t obs_bytes, int64_t frame_stack,
                       uint64_t seed, int64_t ep_len, int64_t* ep_j, int64_t* ep_t,
                       uint8_t* obs_out, double* rew_out, uint8_t* term_out,
                       uint8_t* trunc_out, void* stream);
int tsrl_synth_u8_reset(const int64_t* ids, const uint8_t* mask, int64_t k,
                        int64_t obs_bytes, int64_t frame_stack, uint64_t seed, int64_t ep_len,
                        int64_t* ep_j, int64_t* ep_t, uint8_t* obs_out, void* stream);

/* CartPole-v1 (BASELINE config 1; gymnasium classic_control cartpole.py + TimeLimit(500),
 * restated -- gymnasium parity unpinned): state f64 [N, 4] (x, x_dot, theta, theta_dot),
 * ep_t / ep_j per env.  step: rows r < k act on env ids[r] (NULL -> r) with Discrete(2)
 * actions act[r] (int64); writes obs f32 [k, 4], rew f64 (1, or 0 after termination),
 * terminated (x / theta thresholds) and truncated (ep_t >= max_steps).  reset: rows with
 * mask[r] (NULL -> all) start episode ep_j+1 from U(-0.05, 0.05)^4 of a counter hash
 * (oracle/cartpole.py).  Stands behind the Collector's env.step/reset for CartPoleVectorEnv
 * (tianshou/env/venvs.py:300-381 over gym envs in the reference). */
int tsrl_cartpole_step(const int64_t* ids, int64_t k, const int64_t* act, int64_t max_steps,
                       double* state, int64_t* ep_t, float* obs_out, double* rew_out,
                       uint8_t* term_out, uint8_t* trunc_out, void* stream);
int tsrl_cartpole_reset(const int64_t* ids, const uint8_t* mask, int64_t k, uint64_t seed,
                        double* state, int64_t* ep_j, int64_t* ep_t, float* obs_out,
                        void* stream);

/* ---------------------------------------------------------------------------------
 * Observation RunningMeanStd (VectorEnvNormObs, tianshou/env/venv_wrappers.py:65-112;
 * RunningMeanStd, tianshou/utils/statistics.py:69-114).
 * rms_merge folds column partials of a batch of `count` rows (count = number of mask
 * bytes set, or k when mask == NULL; zero rows -> no update) into mean/var (f32 [dim])
 * and *count (f64 scalar on device).  A non-NULL batch_count (device f64) overrides the
 * mask/k row count (data-parallel: partials and count summed over ranks).  `ticket` is a zero-initialised device word owned by
 * the statistics object (the last workgroup publishes the count and re-arms it; no host
 * state, so the call can be captured in a HIP graph).  rms_norm_rows writes
 * clip((x - mean) / sqrt(var + eps), +-clip) for rows with mask[r] (all when NULL).
 * ------------------------------------------------------------------------------- */
int tsrl_rms_merge(const double* col_partials, int64_t nblk, int64_t dim,
                   const uint8_t* mask, int64_t k, const double* batch_count, float* mean,
                   float* var, double* count, unsigned int* ticket, void* stream);
/* Two consecutive updates (step batch of k rows from partials_step, then the reset rows from
 * partials_reset counted by blk_done) in one launch; snap_mean / snap_var receive the state
 * after the first update (the statistics that normalise the step observations). */
int tsrl_rms_merge2(const double* partials_step, const double* partials_reset,
                    const double* blk_done, int64_t nblk, int64_t dim, int64_t k, float* mean,
                    float* var, double* count, float* snap_mean, float* snap_var,
                    unsigned int* ticket, const double* k_dev, void* stream);
/* Data parallel: fold this rank's merge2 inputs into out[4*dim+2] f64 = [step (sum, sumsq)
 * x dim | reset (sum, sumsq) x dim | reset-row count | step-row count k]; after an
 * all-reduce over the ranks, tsrl_rms_merge2(out, out + 2*dim, out + 4*dim, nblk = 1, dim,
 * k_dev = out + 4*dim + 1) applies the reference's single global VectorEnvNormObs update
 * (venv_wrappers.py:93-99).  k_dev (nullable) in merge2 overrides k. */
int tsrl_rms_sum_partials2(const double* partials_step, const double* partials_reset,
                           const double* blk_done, int64_t nblk, int64_t dim, int64_t k,
                           double* out, void* stream);
int tsrl_rms_norm_rows(const float* x, const uint8_t* mask, int64_t k, int64_t dim,
                       const float* mean, const float* var, float eps, float clip,
                       float* out, void* stream);
/* Exact (opt-in) form of RunningMeanStd.update: the reference's f32 arithmetic bit for bit --
 * np.mean / np.var over axis 0 (sequential row-order f32 column sums) and the f32 update with
 * the counts as NEP-50 f32 scalars (statistics.py:93-114).  Updates mean / var / *count with
 * the rows of x taken by mask (all when NULL); snap_mean / snap_var (nullable, both or none)
 * receive the state after it; then, when x2 is non-NULL, a second update with x2's rows taken
 * by mask2 (the reset rows of the same vector step).  `ticket`: a zero-initialised device word
 * of the statistics object (re-armed by the call).  One thread per column, latency-bound. */
int tsrl_rms_exact_update(const float* x, const uint8_t* mask, int64_t k, const float* x2,
                          const uint8_t* mask2, int64_t k2, int64_t dim, float* mean, float* var,
                          double* count, float* snap_mean, float* snap_var,
                          unsigned int* ticket, void* stream);

/* ---------------------------------------------------------------------------------
 * VectorReplayBuffer add for one vector step (ReplayBufferManager.add,
 * tianshou/data/buffer/manager.py:104-161 + ReplayBuffer._add_index, base.py:195-214).
 * Row r (env b = ids ? ids[r] : r) goes to storage row ptr[r] (or offset[b] + uniform_rel
 * when ptr is NULL: every env at the same ring position); every pointer except the
 * episode-statistics ones may be NULL (that key is then not written).
 *   obs_dst[ptr]      <- obs_src[r]                       (row_bytes_obs bytes)
 *   obs_next_dst[ptr] <- norm(obs_next_src[r]) or copy    (norm when mean != NULL)
 *   cur_obs[r]        <- the same obs_next value          (Collector's data.obs = obs_next)
 *   act_dst[ptr]      <- act_src[r]
 *   rew/flags/env_id scalars; episode stats per env b:
 *   ep_rew[b] += rew ; ep_len[b] += 1 ; on done record (ep_rew, ep_len, ep_idx+offset) in
 *   out_ep_* (per row, nullable) and stat_*[ptr] (per storage row, nullable), then reset
 *   and set ep_idx[b] = next_rel[r].
 * Auto-reset (nullable): rows with reset_mask[r] set take cur_obs[r] <- norm(reset_src[r])
 *   with reset_mean / reset_var (collector.py:342-361, the obs of the new episode).
 * rel_next (nullable, with rel_dev): receives (*rel_dev + 1) % ring_size -- the cursor of the
 *   next step in the other slot of a ping-pong pair (graph-captured steps alternate the two
 *   slots), replacing a separate tsrl_ring_advance launch.
 * ------------------------------------------------------------------------------- */
typedef struct tsrl_add_args {
    const int64_t* ids;      /* [k] env ids or NULL (identity) */
    const int64_t* ptr;      /* [k] global storage rows, or NULL: offset[b] + uniform_rel */
    const int64_t* next_rel; /* [k] sub-buffer index after the add (for ep_idx reset),
                                or NULL: uniform_next */
    const int64_t* offset;   /* [num_envs] sub-buffer offsets */
    int64_t k;
    int64_t uniform_rel;     /* every env at the same sub-buffer index (n_step collect) */
    int64_t uniform_next;
    const int64_t* rel_dev;  /* non-NULL: the uniform index is read from device memory (a
                                HIP-graph-replayable step; advance it with
                                tsrl_ring_advance), next = (rel + 1) % ring_size */
    int64_t ring_size;
    /* row payloads */
    const void* obs_src; void* obs_dst; int64_t obs_row_bytes;
    const float* obs_next_src; float* obs_next_dst; float* cur_obs; int64_t obs_dim;
    const float* norm_mean; const float* norm_var; float norm_eps; float norm_clip;
    const void* obs_next_src_raw; void* obs_next_dst_raw; /* non-f32 obs_next (copy) */
    const void* act_src; void* act_dst; int64_t act_row_bytes;
    /* scalars */
    const double* rew; const uint8_t* term; const uint8_t* trunc;
    double* rew_dst; uint8_t* term_dst; uint8_t* trunc_dst; uint8_t* done_dst;
    int64_t* env_id_dst;
    /* episode statistics (device state, per env) */
    double* ep_rew; int64_t* ep_len; int64_t* ep_idx;
    double* out_ep_rew; int64_t* out_ep_len; int64_t* out_ep_idx; /* per row, nullable */
    double* stat_rew; int64_t* stat_len; int64_t* stat_idx;       /* per storage row */
    /* auto-reset rows and fused ring advance (nullable) */
    const float* reset_src; const uint8_t* reset_mask;
    const float* reset_mean; const float* reset_var;
    int64_t* rel_next;
    /* source row pitches in bytes (0: the destination row size).  save_only_last_obs
     * (manager.py:127-132) stores the last frame of each [stack, ...] observation: the
     * source then points at frame stack-1 of row 0 and the pitch is the whole row. */
    int64_t obs_src_pitch;
    int64_t obs_next_src_pitch;
    /* destination row pitch of obs_dst / obs_next_dst / obs_next_dst_raw in bytes (0: the row
     * size): the storage of wide f32 observations is padded to a 128-byte multiple
     * (VectorReplayBuffer, e.g. 376 -> 384 floats) so the learn kernels' row gathers start on
     * a cache line; the pad columns stay zero. */
    int64_t obs_dst_pitch;
} tsrl_add_args;
int tsrl_buffer_add(const tsrl_add_args* a, void* stream);

/* ---------------------------------------------------------------------------------
 * One vector step of Collector.collect (collector.py:258-361) in ONE launch, for a
 * SyntheticVectorEnv with Box observations under VectorEnvNormObs (venv_wrappers.py:77-99)
 * and the Gaussian MuJoCo actor (utils/models.py:34-97, pg.py:133-171).  Replaces the
 * launch sequence tsrl_gauss_policy_act_rng -> tsrl_synth_box_step_reset -> tsrl_rms_merge2
 * -> tsrl_buffer_add of one step, rotated by one: the launch of step i first runs the buffer
 * add of step i-1 (`add`; add.k == 0: none), then the actor on the new live obs, the env
 * step + auto-reset, and both obs_rms updates (folded by the last workgroups to finish, no
 * grid barrier).  The caller issues the add of the LAST step as tsrl_buffer_add(&add).
 * The live obs of a step go to the buffer's obs rows from this launch (obs_dst ...), so the
 * adds copy no obs (add.obs_src = NULL) and write the new live obs to HBM only in that
 * closing tsrl_buffer_add.
 *   w1p: the actor's first-layer weight packed by tsrl_collect_pack_w1 (once per update);
 *   workspace: tsrl_collect_workspace_bytes(k, dim) bytes, ZEROED once before first use
 *     (its tickets re-arm themselves);
 *   no_moments (exact obs_rms): nonzero = the launch computes no obs_rms moments; the
 *     caller applies tsrl_rms_exact_update to raw / reset_raw between launches and the
 *     pending add normalises with mean / var / snap_*.  0: the step's integer moments are
 *     merged by the next launch of the chain (rms_step) or by tsrl_collect_rms_finalize;
 *     data parallel: the caller all-reduces the step's totals slot
 *     (tsrl_collect_totals_offset) in between.
 * ------------------------------------------------------------------------------- */
typedef struct tsrl_collect_args {
    tsrl_add_args add;       /* pending add of the previous step (add.k == 0: none) */
    int64_t k;               /* envs (rows) */
    int64_t dim;             /* observation columns (multiple of 4, <= 512) */
    float* cur;              /* [k, dim] live normalised observations (read when add.k == 0;
                                the fused add keeps them on chip) */
    /* this step's stored obs rows: obs_dst[(obs_offset[r] + ring position) * dim] = live obs
     * row r, the position read from *obs_rel_dev or obs_uniform_rel; the pending add (and the
     * closing tsrl_buffer_add) therefore run with obs_src = NULL */
    float* obs_dst; const int64_t* obs_offset; const int64_t* obs_rel_dev;
    int64_t obs_uniform_rel;
    /* actor */
    const float* w1p; const float* b1; const float* w2; const float* b2;
    const float* w3; const float* b3; const float* log_std; int64_t act_dim;
    uint64_t act_seed; const int64_t* rng_ctr; int64_t* rng_next; int sample;
    int bound_method; const float* low; const float* high;
    float* act; float* act_remap;   /* [k, act_dim] */
    /* synthetic env (tsrl_synth_box_step_reset's operands) */
    uint64_t env_seed; int64_t ep_len; int64_t* ep_j; int64_t* ep_t;
    float* raw; float* reset_raw; double* rew; uint8_t* term; uint8_t* trunc; uint8_t* done;
    /* obs RunningMeanStd */
    void* workspace;
    float* mean; float* var; float* snap_mean; float* snap_var; double* count;
    int64_t no_moments;      /* exact obs_rms: no moments (see above); 0: the deferred merge */
    int64_t rms_step;        /* index of this launch in its chain of deferred steps (0: the
                                first after tsrl_collect_rms_finalize or a fresh workspace) */
    int64_t obs_pitch;       /* obs_dst row pitch in floats (0: dim) */
    float act_coef;          /* 0: the quantised synthetic env (action-independent; int64
                                totals); c != 0: the action-coupled env (synth.h coupled_val:
                                env phase after the actor, f64 totals; the act_dim action
                                columns feed obs column d mod act_dim) */
    /* Pipelined exact obs_rms (xpipe != 0; exact_obs_rms with the action-independent env,
     * no_moments = 0): the env rows of step i + d are computed d launches ahead ("spec" env,
     * counters spec_j / spec_t) into spec_raw / spec_reset_raw / spec_done, so that their f32
     * batch statistics (tsrl_rms_exact_stats, on a second graph branch) are ready when
     * launch i + d + 1 merges them.  Launch i merges `xstats` (step i - 1's batch statistics,
     * when rms_step > 0) into the state slot in its prologue with the reference's f32
     * update_from_moments; its own env phase writes flags / counters only.  spec_raw NULL:
     * no spec step in this launch. */
    int64_t xpipe;
    const void* xstats;
    int64_t* spec_j; int64_t* spec_t;
    float* spec_raw; float* spec_reset_raw; uint8_t* spec_done;
} tsrl_collect_args;
int64_t tsrl_collect_pack_floats(int64_t dim);
int tsrl_collect_pack_w1(const float* W, int64_t dim, float* packed, void* stream);
int64_t tsrl_collect_workspace_bytes(int64_t k, int64_t dim);
int tsrl_collect_box_step(const tsrl_collect_args* a, void* stream);
/* After the last deferred step of a chain (rms_step = that step's index): its integer
 * obs_rms moments merged into mean / var / count, snap_mean / snap_var = the statistics after
 * its step rows (what the closing tsrl_buffer_add normalises obs_next with).  Replaces the
 * obs_rms update of VectorEnvNormObs.step (env/venv_wrappers.py:93-99) for that step. */
int tsrl_collect_rms_finalize(const tsrl_collect_args* a, void* stream);
/* Byte offset in the workspace of the int64 [4 * dim + 2] totals slot that step `step` of a
 * chain accumulates ([4*dim] reset rows, [4*dim + 1] step rows; data parallel: all-reduce it
 * with SUM before the next launch, world * k <= 2^17 keeps the sums exact). */
int64_t tsrl_collect_totals_offset(int64_t step);
/* Pipelined exact obs_rms (see tsrl_collect_args.xpipe).
 * tsrl_collect_spec_step: the spec env step alone (a pipeline's first d steps): with `init`
 *   the spec counters start from the env's (ep_j / ep_t), then one step of them writes the
 *   rows of that step to spec_raw / spec_reset_raw / spec_done.
 * tsrl_collect_xpipe_finalize: after the chain's last launch (rms_step = its index), its
 *   step's batch statistics `xstats` merged into the state that launch published -> mean /
 *   var / count, snap_mean / snap_var = after its step rows (the closing tsrl_buffer_add's
 *   obs_next statistics).
 * tsrl_rms_exact_stats: the batch moments of one RunningMeanStd.update pair in the
 *   reference's f32 arithmetic (statistics.py:93-101: np.mean / np.var over axis 0, sequential
 *   f32 column sums in row order) -- rows x [k, dim] (all), then the rows of reset_x [k, dim]
 *   whose done flag is set, in row order -- into `stats` (tsrl_rms_exact_stats_bytes(dim)):
 *   float bm1[dim], bv1[dim], bm2[dim], bv2[dim], then int64 n1, nd at byte offset
 *   16 * dim rounded up to 8.  Merging them with update_from_moments reproduces
 *   tsrl_rms_exact_update bit for bit.  dim % 4 == 0, x / reset_x 16-byte aligned. */
int tsrl_collect_spec_step(const tsrl_collect_args* a, int init, void* stream);
int tsrl_collect_xpipe_finalize(const tsrl_collect_args* a, void* stream);
int64_t tsrl_rms_exact_stats_bytes(int64_t dim);
int tsrl_rms_exact_stats(const float* x, int64_t k, const float* reset_x, const uint8_t* done,
                         int64_t dim, void* stats, void* stream);
/* The same for nsteps <= 4 steps in one launch (host arrays of the per-step pointers): the
 * pipelined collect computes two steps' statistics per launch, one graph edge fewer per
 * two steps. */
int tsrl_rms_exact_stats_n(int nsteps, const float* const* x, const float* const* reset_x,
                           const uint8_t* const* done, int64_t k, int64_t dim,
                           void* const* stats, void* stream);
/* The largest nsteps tsrl_rms_exact_stats_n accepts (the Collector clamps its exact_group). */
int tsrl_rms_exact_stats_max_steps(void);
/* *rel_dev = (*rel_dev + 1) % ring_size (device-side ring cursor for graph-captured steps). */
int tsrl_ring_advance(int64_t* rel_dev, int64_t ring_size, void* stream);

/* ---------------------------------------------------------------------------------
 * Episode-aware index stepping and frame stacking of a VectorReplayBuffer whose `num`
 * sub-buffers of `size` rows each hold lengths[b] rows and last wrote last_index[b]
 * (global row), with per-row done flags (ReplayBufferManager, manager.py:24-297).
 * tsrl_ring_step_index: out[r] = prev^steps(idx[r]) for steps > 0 (manager.py:259-277,
 *   _prev_index), next^(-steps)(idx[r]) for steps < 0 (manager.py:280-297, _next_index),
 *   idx[r] mod (size*num) for steps == 0.
 * tsrl_stack_gather: ReplayBuffer.get(idx, key, stack_num) (buffer/base.py:317-358):
 *   dst[r][s] = src[prev^(stack_num-1-s)(idx[r])] for rows of frame_bytes bytes (the
 *   save_only_last_obs frame store of the Atari setup, examples/atari/atari_ppo.py:183-189,
 *   or whole stored rows); chain_out [k][stack_num] (nullable) receives the row indices so
 *   that other keys (info, policy) can be stacked alike; dst may be NULL (chain only).
 * tsrl_stack_gather_pitched: the same with source rows src_pitch bytes apart (a padded
 *   storage: wide f32 observation rows kept 128-byte aligned, see tsrl_gather_rows_pitched);
 *   the output frames are packed (frame_bytes apart).
 * ------------------------------------------------------------------------------- */
int tsrl_ring_step_index(const int64_t* idx, int64_t k, const uint8_t* done,
                         const int64_t* last_index, const int64_t* lengths, int64_t size,
                         int64_t num, int steps, int64_t* out, void* stream);
int tsrl_stack_gather(const void* src, int64_t frame_bytes, const int64_t* idx, int64_t k,
                      int64_t stack_num, const uint8_t* done, const int64_t* last_index,
                      const int64_t* lengths, int64_t size, int64_t num, void* dst,
                      int64_t* chain_out, void* stream);
int tsrl_stack_gather_pitched(const void* src, int64_t src_pitch, int64_t frame_bytes,
                              const int64_t* idx, int64_t k, int64_t stack_num,
                              const uint8_t* done, const int64_t* last_index,
                              const int64_t* lengths, int64_t size, int64_t num, void* dst,
                              int64_t* chain_out, void* stream);

/* Frame-stack input of the Atari trunk: dst[r][p][ch] = lut[src[r][ch][p]] for n rows of c
 * planes of hw bytes -- the uint8 [n, c, h, w] observations as the channels_last (NHWC) f32
 * tensor the conv trunk reads, scaled through a 256-entry table the caller computes exactly as
 * scale_obs does (obs / 255, examples/atari/atari_network.py:18-30 + :84), in one HBM pass. */
int tsrl_frames_to_f32_nhwc(const uint8_t* src, int64_t n, int64_t c, int64_t hw,
                            const float* lut, float* dst, void* stream);

/* First convolution + ReLU of the Nature-DQN trunk straight from uint8 frame stacks:
 * out = relu(conv(frames, w) / scale + bias), frames [*][4][84][84] u8 (contiguous, 4-byte
 * aligned); output sample s reads frame stack rows[s] (rows: n int64 indices, nullable =
 * identity, so a minibatch is read in place from the whole batch -- round 6), w
 * [32][4][8][8] f32 addressed through its element strides (sw0..sw3, so a
 * channels_last weight needs no copy), bias [32] (nullable), out [n][20][20][32] f32 (NHWC,
 * 16-byte aligned).  Replaces scale_obs + Conv2d(4, 32, 8, 4) + ReLU of
 * examples/atari/atari_network.py:18-30,53-90 in DQN.forward (:84): bytes are exact bf16
 * operands, weights split exactly into 3 bf16 planes (f32 GEMM error). */
int tsrl_dqn_conv1_fwd(const uint8_t* frames, int64_t n, const int64_t* rows, const float* w,
                       int64_t sw0,
                       int64_t sw1, int64_t sw2, int64_t sw3, const float* bias, float scale,
                       int relu, float* out, void* stream);

/* Data gradient of the trunk's second convolution (Conv2d(32, 64, 4, stride 2), :53-90) with
 * the ReLU mask of its input fused: dx = (z1 > 0) * conv_transpose(gy, w), gy [n][9][9][64]
 * f32 NHWC, w [64][32][4][4] f32 through its element strides, z1 [n][20][20][32] f32 NHWC
 * (the first layer's ReLU output; NULL = no mask), dx [n][20][20][32] f32 NHWC.  Replaces
 * MIOpen's backward-data + ReLU backward of loss.backward() (ppo.py:146) for the trunk;
 * bf16x6 products (f32 GEMM error). */
int tsrl_dqn_conv2_dgrad(const float* gy, int64_t n, const float* w, int64_t sw0, int64_t sw1,
                         int64_t sw2, int64_t sw3, const float* z1, float* dx, void* stream);

/* Weight and bias gradient of the first convolution straight from the uint8 frames:
 * gw[co][ci][kh][kw] = sum_p gy[p][co] * frames[p's tap (ci, kh, kw)] / scale (gw contiguous
 * [32][4][8][8] f32), gb[co] = sum_p gy[p][co] (nullable), gy [n][20][20][32] f32 NHWC (the
 * gradient w.r.t. conv1's pre-ReLU output, 16-byte aligned), frames [n][4][84][84] u8
 * (4-byte aligned).  Replaces the MIOpen weight gradient of Conv2d(4, 32, 8, 4) over
 * scale_obs(frames) (examples/atari/atari_network.py:18-30,53-90) in loss.backward()
 * (ppo.py:146) and the u8 -> f32 frame conversion it needs: bytes exact in bf16, gy split
 * into 3 bf16 planes (f32 GEMM error), per-workgroup partials folded in fixed order (f64).
 * workspace: tsrl_dqn_conv1_wgrad_workspace_bytes(n) bytes.  rows: as tsrl_dqn_conv1_fwd
 * (gradient row s belongs to frame stack rows[s]; nullable). */
/* y = max(y + bias, 0) in place over rows x C f32 (NHWC activations of a convolution run
 * without bias; C % 4 == 0, 16-byte aligned; bias nullable): the bias add + ReLU of the
 * trunk's Conv2d + ReLU pairs (examples/atari/atari_network.py:53-90) in one pass. */
int tsrl_bias_relu_rows(float* y, const float* bias, int64_t rows, int64_t C, void* stream);

/* ReLU backward of the trunk's Conv2d + ReLU pairs fused with the bias gradient:
 * gy = (z > 0) * gz over rows x C f32 NHWC rows (gy may alias gz; 16-byte aligned;
 * C % 4 == 0, C / 4 a power of two, C <= 1024) and, when gb is not NULL, gb[c] = sum_r gy[r][c]
 * (per-workgroup f32 partials folded in f64 in fixed order; ws of
 * tsrl_relu_bwd_rows_workspace_bytes(rows, C) bytes).  Replaces threshold_backward + the bias
 * reduction of convolution_backward in loss.backward() (ppo.py:146) for
 * examples/atari/atari_network.py:53-90. */
int64_t tsrl_relu_bwd_rows_workspace_bytes(int64_t rows, int64_t C);
int tsrl_relu_bwd_rows(const float* gz, const float* z, float* gy, int64_t rows, int64_t C,
                       float* gb, void* ws, int64_t ws_bytes, void* stream);

int64_t tsrl_dqn_conv1_wgrad_workspace_bytes(int64_t n);
int tsrl_dqn_conv1_wgrad(const uint8_t* frames, int64_t n, const int64_t* rows,
                         const float* gy, float scale,
                         float* gw, float* gb, void* workspace, int64_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * np.random.permutation(n) of the global legacy RandomState, bit-exact: the shuffle order
 * of Batch.split (tianshou/data/batch.py:896-912, one permutation per PPO repeat,
 * ppo.py:106-107).  NumPy's legacy permutation = arange(n) shuffled by
 * `for i in n-1..1: j = random_interval(i); swap(x[i], x[j])`.
 *
 * tsrl_np_shuffle_draws (HOST function, host pointers): the MT19937 stream and the masked
 *   rejection loop.  key[624]/pos are the ('MT19937', key, pos, ...) of
 *   np.random.get_state(); both are advanced in place exactly as NumPy advances them, so the
 *   caller writes them back with set_state.  draws[i] = j_i for 1 <= i < n, draws[0] = 0.
 *   n < 2^32.  No HIP call; safe from any host thread.
 * tsrl_shuffle_apply (device): out[0..n) = the permutation those draws produce (int64),
 *   resolved in parallel (one stable radix sort of (j, step) + a pointer chase); workspace
 *   from tsrl_shuffle_apply_workspace_bytes(n).
 * ------------------------------------------------------------------------------- */
int tsrl_np_shuffle_draws(uint32_t* key, int32_t* pos, int64_t n, uint32_t* draws);
/* The same draws and final state computed by host threads (csrc/np_perm_mt.cpp): MT19937 jump
 * ahead (x^J mod the generator's minimal polynomial) so each thread generates its own stretch of
 * the stream, and the masked rejection resolved chunk-parallel (every word classified for a window
 * of possible starting i, only the uncertain words walked in order, then the draws written per
 * chunk from the exact starts).  For the global permutation of a data-parallel update
 * (batch.py:896-912 over world x n rows).  n < 2^21 runs tsrl_np_shuffle_draws; nthreads <= 0:
 * hardware concurrency (at most 32).  The first call builds the jump table (~1 s, cached). */
int tsrl_np_shuffle_draws_mt(uint32_t* key, int32_t* pos, int64_t n, uint32_t* draws,
                             int nthreads);
int64_t tsrl_shuffle_apply_workspace_bytes(int64_t n);
int tsrl_shuffle_apply(const uint32_t* draws, int64_t n, int64_t* out, void* workspace,
                       int64_t workspace_bytes, void* stream);

/* Row gather: dst[i] = src[idx[i]] for rows of row_bytes bytes (Batch.__getitem__ /
 * ReplayBuffer.__getitem__ fancy indexing, tianshou/data/batch.py:446-460,
 * buffer/base.py:360-389). */
int tsrl_gather_rows(const void* src, int64_t row_bytes, const int64_t* idx, int64_t k,
                     void* dst, void* stream);
/* The same from a source whose rows are src_pitch bytes apart (a padded buffer storage). */
int tsrl_gather_rows_pitched(const void* src, int64_t src_pitch, int64_t row_bytes,
                             const int64_t* idx, int64_t k, void* dst, void* stream);

/* out[c] = sum_r x[r][c] for a row-major f32 [rows, cols] matrix: the bias gradients
 * (db = sum over the minibatch of dY) and the reduction of the split-K partial products of
 * the weight gradients (dW = dY^T X).  Tall inputs use a caller workspace for per-chunk
 * partial rows (size from tsrl_sum_rows_workspace_bytes). */
int64_t tsrl_sum_rows_workspace_bytes(int64_t rows, int64_t cols);
int tsrl_sum_rows_f32(const float* x, int64_t rows, int64_t cols, float* out, void* workspace,
                      int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * PPO clipped surrogate + value + entropy loss, Gaussian Independent(Normal(mu, exp(s)),1)
 * with state-independent log-std s (PPOPolicy.learn, tianshou/policy/modelfree/ppo.py:
 * 106-151; ActorProb, utils/net/continuous.py:218-235; fixed_std_normal,
 * utils/models.py:96-97).  Minibatch rows come from the full-batch arrays through idx
 * (idx NULL -> identity).  Gradients of the MEAN loss over `b_global` rows are written
 * per row (grad_mu [b,A], grad_value [b]); per-block partial sums (layout
 * [nblk][4 + A]: clip_sum, vf_sum, count, unused, dlogstd[A]) feed tsrl_reduce_partials
 * and tsrl_ppo_gauss_finalize.
 * ------------------------------------------------------------------------------- */
typedef struct tsrl_ppo_params {
    double eps_clip;        /* Python floats, rounded to f32 where torch would */
    double dual_clip;       /* <= 0 : None */
    double vf_coef;
    double ent_coef;
    double adv_eps;         /* 1e-8 (PGPolicy._eps) */
    double b_global;        /* rows in the (global) minibatch */
    int32_t value_clip;
    int32_t norm_adv;
} tsrl_ppo_params;

int64_t tsrl_ppo_num_partials(int64_t b);
int tsrl_adv_moments(const float* adv, const int64_t* idx, int64_t b, double* partials,
                     void* stream);
/* Advantage moments (sum adv, sum adv^2) of every minibatch of an epoch in one pass:
 * segment g = rows [bounds[g], bounds[g+1]) of idx (device int64 [nseg+1]); out [nseg, 2]
 * f64; partials [nseg, tsrl_adv_moments_seg_parts(max_seg), 2] f64 scratch, max_seg = the
 * longest segment.  Under data parallelism one all-reduce of out serves the whole epoch. */
int64_t tsrl_adv_moments_seg_parts(int64_t max_seg);
int tsrl_adv_moments_seg(const float* adv, const int64_t* idx, const int64_t* bounds,
                         int64_t nseg, int64_t max_seg, double* partials, double* out,
                         void* stream);
int tsrl_reduce_partials(const double* partials, int64_t nblk, int64_t width, double* out,
                         void* stream);
int tsrl_ppo_gauss_fwd_bwd(const float* mu, const float* log_std, const float* value,
                           const float* act, const float* logp_old, const float* adv,
                           const float* ret, const float* v_s, const int64_t* idx,
                           int64_t b, int64_t act_dim, const double* adv_sums,
                           tsrl_ppo_params p, float* grad_mu, float* grad_value,
                           double* partials, void* stream);
int tsrl_ppo_gauss_finalize(const double* sums, int64_t act_dim, const float* log_std,
                            tsrl_ppo_params p, float* losses, float* grad_log_std,
                            void* stream);
/* log N(act | mu, exp(log_std)) summed over the action dim (Independent(...,1).log_prob),
 * used for logp_old in PPOPolicy.process_fn (ppo.py:95-96). */
int tsrl_gauss_logp(const float* mu, const float* log_std, const float* act, int64_t b,
                    int64_t act_dim, float* out, void* stream);

/* ---------------------------------------------------------------------------------
 * The same PPO minibatch loss for Categorical policies (discrete actions):
 * mode 0 = Categorical(logits=x) (examples/atari/atari_ppo.py:136-137), mode 1 =
 * Categorical(probs=x) (test/discrete/test_ppo.py:95 with the softmax Actor,
 * utils/net/discrete.py:69-70).  x [b, num_actions] is the dist_fn input of the minibatch
 * rows (minibatch order); act (i64 action indices), logp_old, adv, ret, v_s are read through
 * idx.  Writes d(mean loss)/dx [b, num_actions] and d/d(value) [b]; partials [nblk][4] =
 * (clip_sum, vf_sum, count, entropy_sum) for tsrl_reduce_partials, then
 * tsrl_ppo_cat_finalize -> losses [4] = (loss, clip, vf, ent).  tsrl_cat_logp is
 * dist.log_prob(act) for logp_old (ppo.py:95-96).
 * ------------------------------------------------------------------------------- */
int tsrl_ppo_cat_fwd_bwd(const float* x, const float* value, const int64_t* act,
                         const float* logp_old, const float* adv, const float* ret,
                         const float* v_s, const int64_t* idx, int64_t b, int64_t num_actions,
                         int mode, const double* adv_sums, tsrl_ppo_params p, float* grad_x,
                         float* grad_value, double* partials, void* stream);
int tsrl_ppo_cat_finalize(const double* sums, tsrl_ppo_params p, float* losses, void* stream);
int tsrl_cat_logp(const float* x, const int64_t* act, int64_t b, int64_t num_actions, int mode,
                  float* out, void* stream);

/* Categorical(logits).sample() of the Collector's policy step (pg.py:133-171): out[r] =
 * argmax_a(logits[r][a] - log(-log(u[r][a]))) (Gumbel-max; first index on ties), logits and
 * u [n][num_actions] f32 (u uniform in [0, 1), drawn by the caller), out [n] int64. */
int tsrl_cat_gumbel_argmax(const float* logits, const float* u, int64_t n, int64_t num_actions,
                           int64_t* out, void* stream);

/* ---------------------------------------------------------------------------------
 * Fused actor/critic MLP of the PPO minibatch for the MuJoCo network shape
 * (tianshou/utils/models.py:34-97: Net(D, (64, 64), Tanh) trunks, ActorProb mu head
 * Linear(64, A) unbounded, Critic head Linear(64, 1)); replaces the per-layer nn.Linear /
 * nn.Tanh forward and autograd backward of ppo.py:121-146 (utils/net/common.py:56-150,
 * continuous.py:87-235).
 *
 * tsrl_mlp_l1_fwd: H1 = act(X[idx] W^T + b) for the stacked first layers (Wa, ba: actor
 *   [64, D]; Wc, bc: critic [64, D]) -> 128 features per row.  frag_out = 1 writes the MFMA
 *   fragment layout consumed by tsrl_ppo_tail (tsrl_mlp_frag_floats(n) floats); 0 writes
 *   row-major [n, 128].  D and ldx multiples of 4, 16-byte aligned X / W / out.
 * tsrl_ppo_tail: layers 2-3 of both nets, the PPO loss of tsrl_ppo_gauss_fwd_bwd and the
 *   backward to dZ1 [n, 128] (row-major), writing the layer-2/3 parameter gradients of the
 *   mean loss and the loss sums [4 + A] (layout of tsrl_ppo_gauss_finalize's input).
 * tsrl_mlp_dw: first-layer gradients dW = dZ1^T X[idx], db = column sums of dZ1.  Row
 *   indices idx[] and the pitch ldx must be < 2^32 (the row offsets are 32 x 32-bit
 *   products; ldx is checked).
 * ------------------------------------------------------------------------------- */
typedef struct tsrl_tail_weights {
    const float *w2a, *b2a;   /* actor layer 2 [64,64], [64] */
    const float *w2c, *b2c;   /* critic layer 2 */
    const float *w3a, *b3a;   /* actor mu head [A,64], [A] */
    const float *w3c, *b3c;   /* critic head [1,64], [1] */
    const float *log_std;     /* [A] (sigma_param) */
} tsrl_tail_weights;

typedef struct tsrl_tail_grads {
    float *w2a, *b2a, *w2c, *b2c, *w3a, *b3a, *w3c, *b3c;
} tsrl_tail_grads;

int tsrl_mlp_l1_fwd(const float* X, int64_t ldx, const int64_t* idx, int64_t n, int64_t D,
                    const float* Wa, const float* ba, const float* Wc, const float* bc,
                    int act_tanh, float* out, int frag_out, void* stream);
int64_t tsrl_mlp_frag_floats(int64_t n);
/* The same first layer on the bf16 matrix cores with an exact three-way bf16 split of every
 * f32 operand and the six products of order <= 2 accumulated in f32 ("bf16x6": f32-level
 * error, 2.7x the f32-input MFMA rate; csrc/mlp_x6.hip).  wsplit holds the split stacked
 * weight (tsrl_mlp_split_bytes(D) bytes, 16-byte aligned), refreshed by tsrl_mlp_split_w after
 * every parameter update.  Output layouts as tsrl_mlp_l1_fwd. */
int64_t tsrl_mlp_split_bytes(int64_t D);
int tsrl_mlp_split_w(const float* Wa, const float* Wc, int64_t D, void* wsplit, void* stream);
int tsrl_mlp_l1_fwd_x6(const float* X, int64_t ldx, const int64_t* idx, int64_t n, int64_t D,
                       const void* wsplit, const float* ba, const float* bc, int act_tanh,
                       float* out, int frag_out, void* stream);
int64_t tsrl_ppo_tail_workspace_bytes(int64_t n);
int tsrl_ppo_tail(const float* h1frag, int64_t n, const int64_t* idx,
                  const tsrl_tail_weights* w, int64_t act_dim, const float* act,
                  const float* logp_old, const float* adv, const float* ret, const float* v_s,
                  const double* adv_sums, tsrl_ppo_params p, float* dz1,
                  const tsrl_tail_grads* grads, double* sums, void* workspace,
                  int64_t ws_bytes, void* stream);
/* tsrl_ppo_tail_fin: tsrl_ppo_tail followed, inside its reduction launch, by the loss
 * finalisation of tsrl_ppo_gauss_finalize on the reduced sums (losses[4] = loss, clip, vf,
 * entropy; grad_log_std[act_dim]): the single-process minibatch (no all-reduce of the sums
 * between the two), one launch fewer per minibatch. */
int tsrl_ppo_tail_fin(const float* h1frag, int64_t n, const int64_t* idx,
                      const tsrl_tail_weights* w, int64_t act_dim, const float* act,
                      const float* logp_old, const float* adv, const float* ret, const float* v_s,
                      const double* adv_sums, tsrl_ppo_params p, float* dz1,
                      const tsrl_tail_grads* grads, double* sums, void* workspace,
                      int64_t ws_bytes, const float* log_std, float* losses,
                      float* grad_log_std, void* stream);
/* tsrl_ppo_tail_stage: the same work in two stages so the caller can run the reduction on a
 * second stream beside tsrl_mlp_dw (both only read what the tail kernels wrote):
 * stages & 1 = the actor and critic tail kernels, stages & 2 = the reduction (with the loss
 * finalisation when log_std/losses/grad_log_std are given — all three or none), 3 = both;
 * stages & 4 / & 8 = the actor's / the critic's tail kernel alone (disjoint outputs: two
 * streams may run them concurrently, both before the reduction). */
int tsrl_ppo_tail_stage(const float* h1frag, int64_t n, const int64_t* idx,
                        const tsrl_tail_weights* w, int64_t act_dim, const float* act,
                        const float* logp_old, const float* adv, const float* ret,
                        const float* v_s, const double* adv_sums, tsrl_ppo_params p, float* dz1,
                        const tsrl_tail_grads* grads, double* sums, void* workspace,
                        int64_t ws_bytes, const float* log_std, float* losses,
                        float* grad_log_std, int stages, void* stream);
/* tsrl_ppo_eval: forward only (process_fn): value_out[n] = critic(obs) and, when logp_out is
 * given, logp_out[n] = log N(act | mu(obs), exp(log_std)) summed over the action dims, from
 * the fragment-layout layer-1 activations of tsrl_mlp_l1_fwd (critic only: the actor tiles
 * are not read). */
int tsrl_ppo_eval(const float* h1frag, int64_t n, const tsrl_tail_weights* w, int64_t act_dim,
                  const float* act, float* value_out, float* logp_out, void* stream);

/* tsrl_ppo_eval_fused: tsrl_mlp_l1_fwd_x6 (tanh, fragment layout) followed by tsrl_ppo_eval in
 * ONE launch: the layer-1 activations of each 32-row tile stay in registers and are evaluated
 * there (process_fn's values and log-probs, reference a2c.py:83-100 / ppo.py:95-96), with the
 * same products in the same order -- bit-identical outputs, without the 512 B per row of H1
 * written and read back.  X / ldx / idx / n / D / wsplit / ba / bc as tsrl_mlp_l1_fwd_x6; wt /
 * act_dim / act / value_out / logp_out as tsrl_ppo_eval; workspace: >=
 * tsrl_ppo_eval_fused_workspace_bytes() bytes of device memory, 16-byte aligned (rebuilt by
 * every call).  Enqueues two kernels on `stream`. */
int64_t tsrl_ppo_eval_fused_workspace_bytes(void);
int tsrl_ppo_eval_fused(const float* X, int64_t ldx, const int64_t* idx, int64_t n, int64_t D,
                        const void* wsplit, const float* ba, const float* bc,
                        const tsrl_tail_weights* wt, int64_t act_dim, const float* act,
                        float* value_out, float* logp_out, void* workspace, int64_t ws_bytes,
                        void* stream);
int64_t tsrl_mlp_dw_workspace_bytes(int64_t n, int64_t D);
int tsrl_mlp_dw(const float* dz1, const float* X, int64_t ldx, const int64_t* idx, int64_t n,
                int64_t D, float* gWa, float* gba, float* gWc, float* gbc, void* workspace,
                int64_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Fused Gaussian policy step of the collector (collector.py:286-303 -> pg.py:133-171 ->
 * base.py:183-215) for the get_actor_critic actor (two Tanh layers of 64, unbounded mu
 * head, state-independent log-std): act = eps * exp(log_std) + mu(obs) (eps NULL: act =
 * mu, deterministic eval), act_remap = scale(bound(act)) with bound_method 0 none / 1 clip /
 * 2 tanh and scaling to [low, high] when low/high are given.  The first-layer weight [64, D]
 * is packed once (tsrl_policy_pack_l1, tsrl_policy_pack_floats(D) floats) after each
 * parameter update.
 * ------------------------------------------------------------------------------- */
int64_t tsrl_policy_pack_floats(int64_t D);
int tsrl_policy_pack_l1(const float* W, int64_t D, float* packed, void* stream);
int tsrl_gauss_policy_act(const float* obs, int64_t ldx, int64_t n, int64_t D,
                          const float* w1packed, const float* b1, const float* w2,
                          const float* b2, const float* w3, const float* b3,
                          const float* log_std, int64_t act_dim, const float* eps,
                          int bound_method, const float* low, const float* high, float* act,
                          float* act_remap, void* stream);
/* Same step drawing the noise in-kernel: standard normals from a splitmix64 counter hash of
 * (seed, *rng_ctr, row, dim) through Box-Muller; *rng_next = *rng_ctr + 1 (the other slot of
 * a ping-pong pair), so HIP-graph replays draw fresh noise each step. */
int tsrl_gauss_policy_act_rng(const float* obs, int64_t ldx, int64_t n, int64_t D,
                              const float* w1packed, const float* b1, const float* w2,
                              const float* b2, const float* w3, const float* b3,
                              const float* log_std, int64_t act_dim, uint64_t seed,
                              const int64_t* rng_ctr, int64_t* rng_next, int bound_method,
                              const float* low, const float* high, float* act,
                              float* act_remap, void* stream);

/* ---------------------------------------------------------------------------------
 * Off-policy neighbours.
 * tsrl_nstep_return: BasePolicy.compute_nstep_return + _nstep_return (policy/base.py:386-440,
 *   500-524) over a VectorReplayBuffer ring (done / last_index / lengths as for
 *   tsrl_ring_step_index): for every sampled row idx[b] the next() chain of n_step rows,
 *   episode ends = done or the unfinished last row, out[b][x] = target_q[b][x] *
 *   !terminated[chain[n_step-1]] * gamma^gammas + G_b in f64 (reference operation order),
 *   rounded to the target dtype (f64 != 0: double target_q/out, else float).
 *   1 <= n_step <= 64; target_q holds Q_target(s_{t+n}) at the chain's last row.
 * Sum tree of SegmentTree (data/utils/segtree.py:7-137): tree = f64[2*bound], bound a power of
 *   two, leaves at [bound, bound + size).
 * tsrl_segtree_set: _setitem (:98-104): tree[bound + idx[j]] = values[j * value_stride]
 *   (value_stride 0 broadcasts values[0]; duplicate indices: the last occurrence wins), then
 *   every ancestor = left + right.  win: int32 workspace of size entries, all -1 (restored).
 * tsrl_segtree_reduce: _reduce (:107-119) over leaves [start, end) -> *out (device f64).
 * tsrl_segtree_prefix_idx: _get_prefix_sum_idx (:122-137) for k query values (f64 or f32).
 * ------------------------------------------------------------------------------- */
int tsrl_nstep_return(const double* rew, const uint8_t* done, const uint8_t* terminated,
                      const int64_t* last_index, const int64_t* lengths, int64_t size,
                      int64_t num, const int64_t* idx, int64_t bsz, int64_t n_step,
                      double gamma, const void* target_q, int64_t X, int f64, void* out,
                      void* stream);
int tsrl_segtree_set(double* tree, int64_t bound, const int64_t* idx, const double* values,
                     int64_t value_stride, int64_t k, int* win, void* stream);
int tsrl_segtree_reduce(const double* tree, int64_t bound, int64_t start, int64_t end,
                        double* out, void* stream);
int tsrl_segtree_prefix_idx(const double* tree, int64_t bound, const void* values, int f64,
                            int64_t k, int64_t* out, void* stream);

/* torch.nn.utils.clip_grad_norm_(max_norm) + torch.optim.Adam.step() (ppo.py:143-151) over
 * flat f32 parameter / gradient / moment buffers of n elements: partials (f64,
 * tsrl_clip_adam_partials(n) entries) receive slice norms, norm_out[0] = gradient norm,
 * norm_out[1] = clip coefficient (max_norm <= 0: no clipping, partials / norm_out may be
 * NULL); step[0..nstep) (device f32 step counters, all equal) is
 * advanced by one.  ticket: three device uint32, zero-initialised; [0] and [1] re-arm
 * themselves, [2] is a sticky flag set to 1 when the in-kernel slice-norm hand-off timed
 * out (the step is then invalid for EVERY slice: the caller must check it and reject it).
 * lr_dev (nullable device f32): the learning rate read at run time instead of `lr`, so a
 * captured learn graph follows an lr_scheduler (BasePolicy.update, base.py:312-313).
 * scale_grads: leave the gradient scaled by the clip coefficient in place (what p.grad holds
 * after clip_grad_norm_); 0 skips that pass when the gradient is overwritten next anyway.
 * split (nullable): also write the updated first-layer weights of both nets (flat element
 * ranges [off_a, off_a + 64 d) and [off_c, off_c + 64 d), row-major [64][d]) as the bf16x6
 * planes of tsrl_mlp_split_w (row pitch kp), fusing the next minibatch's re-split. */
typedef struct {
    void* out;
    int64_t off_a, off_c, d, kp;
} tsrl_w1_split;
int64_t tsrl_clip_adam_partials(int64_t n);
int tsrl_clip_adam(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                   float* step, int64_t nstep, float lr, float beta1, float beta2, float eps,
                   float max_norm, double* partials, float* norm_out, unsigned int* ticket,
                   const float* lr_dev, const tsrl_w1_split* split, int scale_grads,
                   void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TSRL_H_ */
