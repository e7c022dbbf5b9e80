/*
 * prl_abi.h — C-ABI of libprl_hip.so, the MI355X (gfx950) hot path of the PPO rollout + update
 * engine that drops in under Raven4567/Parallel-Reinforcement-Learning's Python API.
 *
 * The reference has no FFI: its boundary is the duck-typed Python API of `AsyncTools.AsyncPPO`
 * and `PPO.PPO`.  Every entry point below replaces one piece of that Python code
 * and cites the reference lines (paths relative to the reference repository root).  The Python
 * packages `PPO/` and `AsyncTools/` in this repository bind these symbols with ctypes
 * (see INTEGRATION.md for the stub a maintainer of the reference would add).
 *
 * Conventions (all entry points):
 *   - every pointer is a caller-owned DEVICE pointer unless the comment says "host";
 *   - nothing allocates: scratch comes in through `workspace` (size from prl_workspace_bytes).
 *     The GAE / statistics / surrogate workspaces carry in-launch synchronisation state: they
 *     must be zero-initialised ONCE, dedicated to one op and one stream, and every launch
 *     leaves them re-armed (so each call is a single kernel launch, graph-capturable);
 *   - every call is asynchronous on `stream` (a hipStream_t passed as void*; NULL = null stream)
 *     and contains no host synchronisation, so callers may capture it into a hipGraph;
 *   - return 0 on success, a negative prl_status on failure; prl_last_error() then holds a
 *     thread-local message.  Python wrappers raise RuntimeError with that message.
 *   - not re-entrant per env batch; one host thread per GPU.
 */
#ifndef PRL_ABI_H
#define PRL_ABI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRL_ABI_VERSION 2

enum prl_status {
  PRL_OK = 0,
  PRL_ERR_ARG = -1,     /* bad argument (shape, alignment, null pointer) */
  PRL_ERR_HIP = -2,     /* a HIP runtime call failed */
  PRL_ERR_TIMEOUT = -3  /* an in-kernel bounded spin gave up (never expected) */
};

enum prl_env_kind {
  PRL_ENV_CARTPOLE = 0,        /* gymnasium CartPole-v1 + TimeLimit(500), discrete(2), obs 4  */
  PRL_ENV_PENDULUM = 1,        /* gymnasium Pendulum-v1 + TimeLimit(200), continuous(1), obs 3 */
  PRL_ENV_SYNTH_HUMANOID = 2   /* synthetic Humanoid-v5-shaped env: obs 348, act 17, cont.    */
};

enum prl_op {
  PRL_OP_GAE = 0,        /* n = transitions                 */
  PRL_OP_SURROGATE = 1,  /* n = minibatch size              */
  PRL_OP_SCAN = 2,       /* n = elements (scan/compaction)  */
  PRL_OP_STATS = 3,      /* n = elements (prl_adv_stats)    */
  PRL_OP_GN = 4          /* n = rows (prl_gn_silu_bwd)      */
};

/* ---- housekeeping ------------------------------------------------------------------------- */
int prl_abi_version(void);
const char* prl_last_error(void);
/* sha256 (hex) of the csrc sources + headers this library was built from (csrc/build.py stamps
 * it); prl_native refuses a library whose stamp differs from the sources next to it, so a stale
 * build cannot run silently.  No reference counterpart. */
const char* prl_source_id(void);
/* Bytes of device workspace an op needs for n elements (host call, no GPU work). */
int64_t prl_workspace_bytes(int op, int64_t n);
/* Host call: static geometry of an env kind (AsyncPPO.py:45-46 action_space/observation_space). */
int prl_env_dims(int kind, int* obs_dim, int* act_dim, int* phys_dim, int* max_episode_steps,
                 int* is_discrete);

/* ---- environments (replace EnvVectorizer + gymnasium envs) --------------------------------- */
/* Seed per-env PCG64 generators exactly as numpy's SeedSequence(seed_e) -> PCG64 does, i.e. as
 * gymnasium's `env.reset(seed=seed_e)` seeds `env.np_random` (gymnasium.utils.seeding.np_random).
 * rng[E][4] u64 = {state_hi, state_lo, inc_hi, inc_lo}.  Replaces the per-env RNG that each
 * deep-copied env carries (AsyncTools/AsyncPPO.py:39). */
int prl_pcg64_seed(const uint64_t* seeds, int64_t E, uint64_t* rng, void* stream);

/* EnvVectorizer.reset (AsyncTools/AsyncPPO.py:48-62): reset every env (or those with
 * reset_mask[e] != 0 when reset_mask is non-NULL), clear envs_active (terminal[e] = 0),
 * t_elapsed[e] = 0, write obs[e*obs_stride .. +D) f32.  phys[E][phys_dim] f64. */
int prl_env_reset(int kind, int64_t E, double* phys, uint64_t* rng, int32_t* t_elapsed,
                  uint8_t* terminal, const uint8_t* reset_mask, float* obs, int64_t obs_stride,
                  void* stream);

/* EnvVectorizer.step, compat form (AsyncTools/AsyncPPO.py:64-102): the i-th of the n active envs
 * (env index active_idx[i], ascending) takes actions[i] (discrete: int64[n]; continuous: f32[n][A])
 * and writes its results COMPACTED to row i: obs_out[n][D] f32, reward_out[n] f64,
 * terminated_out[n] u8, truncated_out[n] u8 (TimeLimit).  Does not touch `terminal`. */
int prl_env_step_compact(int kind, int64_t E, double* phys, int32_t* t_elapsed,
                         const int64_t* active_idx, int64_t n, const void* actions,
                         float* obs_out, double* reward_out, uint8_t* terminated_out,
                         uint8_t* truncated_out, void* stream);

/* One vector step of the device-resident AsyncPPO.worker (AsyncTools/AsyncPPO.py:120-141):
 * fuses PPO.get_action's sampling (PPO/PPO.py:85-91), EnvVectorizer.step (:64-102),
 * utils.buffer_append + VecMemory.push (utils.py:17-36, AsyncPPO.py:20-24),
 * utils.update_active_environments_list (utils.py:38-43) and the score counters (:137-138).
 * For every env e with terminal[e] == 0, with t = t_elapsed[e]:
 *   dist row e (stride dist_stride floats): discrete -> probs[A]; continuous -> mu[A], std[A];
 *   action sampled with Philox4x32-10 keyed by (sample_seed, e, t); continuous actions are
 *   tanh(sample) * action_scaling;
 *   traj_obs[t+1][e] = next obs, traj_act[t][e] = action (f32), traj_rew[t][e] = reward (f32),
 *   traj_done[t][e] = terminated|truncated, terminal[e] = that, t_elapsed[e] = ep_len[e] = t+1.
 * traj_obs row t must already hold the pre-step observation (reset writes row 0).
 * active_after[step] += number of envs still non-terminal after this step; reward_sum[0] += sum
 * of rewards (f64) — both must be zeroed by the caller before the rollout. */
int prl_rollout_step(int kind, int64_t E, int32_t step, double* phys, int32_t* t_elapsed,
                     uint8_t* terminal, const float* dist, int64_t dist_stride,
                     float action_scaling, uint64_t sample_seed, int32_t t_max, float* traj_obs,
                     float* traj_act, float* traj_rew, uint8_t* traj_done, int32_t* ep_len,
                     int32_t* active_after, double* reward_sum, void* stream);
/* prl_rollout_step with the step index on the device: step_dev = int64 {k, arrivals} (arrivals 0
 * between launches).  The count goes to active_after[k] (nothing when k is outside [0, t_max)),
 * and the launch's last block sets k = k + 1 and re-arms arrivals, so a captured vector step
 * replayed T times walks k = 0..T-1 with no separate increment.  AsyncPPO's captured vector step
 * (same reference lines). */
int prl_rollout_step_at(int kind, int64_t E, int64_t* step_dev, double* phys,
                        int32_t* t_elapsed, uint8_t* terminal, const float* dist,
                        int64_t dist_stride, float action_scaling, uint64_t sample_seed,
                        int32_t t_max, float* traj_obs, float* traj_act, float* traj_rew,
                        uint8_t* traj_done, int32_t* ep_len, int32_t* active_after,
                        double* reward_sum, void* stream);

/* A WHOLE device rollout of a wide-net policy in ONE persistent launch (AsyncPPO.worker's loop,
 * AsyncTools/AsyncPPO.py:117-146, with PPO.get_action's forward + sampling, PPO/PPO.py:81-96 /
 * ActorCritic.get_dist, PPO/ActorCritic.py:85-105, and the env step, AsyncPPO.py:64-102): every
 * env with terminal[e] == 0 is stepped until its episode ends — the action from the continuous
 * actor (params: policy_old's flat parameters, torch parameters() order) sampled exactly as
 * prl_rollout_step samples it, the trajectory rows, t_elapsed / ep_len / terminal and the counters
 * written as the per-step kernels write them (active_after[t] += envs still active after step t,
 * reward_sum[0] += rewards).  Each wave owns 16 envs and keeps the actor in LDS.  Supported:
 * prl_wide_rollout_supported() (the synthetic env with its D = 348 / A = 17 continuous net;
 * CartPole with the D = 4 / A = 2 discrete net, run by prl_cartpole_rollout below). */
int prl_wide_rollout_supported(int kind, int32_t D, int32_t A, int32_t discrete);
/* The whole CartPole rollout of the discrete actor (ActorCritic, D 4, A 2: policy_old's flat
 * parameters in torch parameters() order, the actor's 4,738 used) as ONE launch, one thread
 * per env: forward, Categorical sampling (the fused step kernel's Philox stream), the float64
 * step, trajectory push and mask, every non-terminal env to the end of its episode.  Replaces
 * AsyncPPO.worker's loop (AsyncTools/AsyncPPO.py:117-146) with PPO.get_action (PPO/PPO.py:81-96)
 * and EnvVectorizer.step (AsyncPPO.py:64-102).  probs_out: null, or [t_max][E][2] f32 receiving
 * the probabilities each step sampled from (tests).  prl_wide_rollout dispatches here for
 * PRL_ENV_CARTPOLE. */
int prl_cartpole_rollout(const float* params, int64_t E, double* phys, int32_t* t_elapsed,
                         uint8_t* terminal, uint64_t sample_seed, int32_t t_max, float* traj_obs,
                         float* traj_act, float* traj_rew, uint8_t* traj_done, int32_t* ep_len,
                         int32_t* active_after, double* reward_sum, float* probs_out,
                         void* stream);
int prl_wide_rollout(int kind, const float* params, int32_t D, int32_t A, int32_t discrete,
                     int64_t E, double* phys, int32_t* t_elapsed, uint8_t* terminal,
                     float action_scaling, uint64_t sample_seed, int32_t t_max, float* traj_obs,
                     float* traj_act, float* traj_rew, uint8_t* traj_done, int32_t* ep_len,
                     int32_t* active_after, double* reward_sum, void* stream);

/* ---- mask / compaction / flatten (replace AsyncTools/utils.py) ----------------------------- */
/* utils.indexes_of_active_environments + number_of_active_environments (utils.py:3-7):
 * idx_out[0..count) = ascending e with terminal[e] == 0; count_out[0] = count (int64). */
int prl_active_indices(const uint8_t* terminal, int64_t E, int64_t* idx_out, int64_t* count_out,
                       void* workspace, void* stream);
/* utils.update_active_environments_list (utils.py:38-43): terminal[active[i]] = dones[i] for the
 * n envs active before the call (ascending order), i.e. mask[where(~mask)] = dones. */
int prl_mask_update(uint8_t* terminal, int64_t E, const uint8_t* dones, int64_t n,
                    void* workspace, void* stream);
/* utils.inactive_states_dropout (utils.py:14-15): dst = src[~drop] (row_bytes per row, order
 * kept); count_out[0] = rows kept. */
int prl_compact_rows(const void* src, int64_t rows, int64_t row_bytes, const uint8_t* drop,
                     void* dst, int64_t* count_out, void* workspace, void* stream);
/* Exclusive scan of episode lengths: offsets[0..E] (offsets[E] = N), int64. */
int prl_exclusive_scan_i32(const int32_t* in, int64_t n, int64_t* offsets, void* workspace,
                           void* stream);
/* utils.buffer_to_target_buffer_transfer (utils.py:45-51): env-major concatenation of the
 * time-major trajectory buffers: row offsets[e] + t of S/A/R/Dn <- traj[t][e] for t < len_e.
 * traj_obs is [T+1][E][D], traj_act [T][E][Adim], traj_rew/traj_done [T][E]. */
int prl_flatten_env_major(int64_t E, int32_t t_max, int32_t D, int32_t Adim,
                          const int64_t* offsets, int64_t N, const float* traj_obs,
                          const float* traj_act, const float* traj_rew,
                          const uint8_t* traj_done, float* S, float* A, float* R, float* Dn,
                          void* stream);

/* ---- PPO.learn hot path -------------------------------------------------------------------- */
/* PPO.compute_gae (PPO/PPO.py:107-120) + `advantages = returns - V` (:198), float32, evaluated in
 * the reference's exact operation order (bit-exact for finite inputs).  next_value: device
 * scalar, NULL -> V[n-1] (PPO.py:188).  adv may be NULL.  sums_out[2] (f64) receives
 * {sum(adv), sum(adv^2)} when adv != NULL (for prl_adv_normalize / a cross-GPU all-reduce). */
int prl_gae(const float* r, const float* d, const float* V, const float* next_value, int64_t n,
            double gamma, double lam, float* ret, float* adv, double* sums_out,
            void* workspace, int64_t workspace_bytes, void* stream);
/* {sum, sum of squares} (f64) of x[n] (PPO.py:199 statistics). */
int prl_adv_stats(const float* x, int64_t n, double* sums_out, void* workspace,
                  int64_t workspace_bytes, void* stream);
/* PPO.py:199: out = (x - mean) / (std_unbiased + eps), mean/std from sums[2] over `count`
 * elements (count may exceed n when sums were all-reduced across GPUs). out may alias x. */
int prl_adv_normalize(const float* x, int64_t n, const double* sums, double count, float eps,
                      float* out, void* stream);

/* PPO.learn's surrogate (PPO/PPO.py:225-249):
 *   ratio = exp(clamp(logp - old_logp, -20, 20)); s1 = ratio*adv; s2 = clamp(ratio,1-clip,1+clip)*adv
 *   loss  = mean(-min(s1, s2)) + vf_coef * SmoothL1(V, ret) - ent_coef * entropy   (scalar)
 * and the gradient of `loss` w.r.t. logp and V (torch semantics: min tie splits 1/2-1/2, clamp
 * passes gradient at inclusive bounds) into dlogp/dV (NULL = skip).  entropy: device scalar. */
int prl_ppo_surrogate_fwd(const float* logp, const float* old_logp, const float* adv,
                          const float* V, const float* ret, const float* entropy, int64_t mb,
                          float clip, float vf_coef, float ent_coef, float* loss_out,
                          float* dlogp, float* dV, void* workspace, int64_t workspace_bytes,
                          void* stream);
/* Backward of the above for an upstream gradient grad_out (device scalar):
 * dlogp = grad_out * dlogp_unit, dV = grad_out * dV_unit. */
int prl_ppo_surrogate_bwd(const float* grad_out, const float* dlogp_unit, const float* dV_unit,
                          int64_t mb, float* dlogp, float* dV, void* stream);

/* RND.compute_intrinsic_reward (PPO/RND.py:71-94): out[i] = beta * || pred(x_i) - target(x_i) ||_2
 * with each net Linear(D,64)+b -> GroupNorm(8, 64, eps 1e-5) -> SiLU -> Linear(64,D)+b
 * (RND.py:25-38).  Weights in torch layout: W1[64][D], b1[64], g[64], beta_gn[64], W2[D][64], b2[D].
 * fp32 MFMA (v_mfma_f32_32x32x2_f32).  x[n][D] f32 row-major. */
int prl_rnd_forward(const float* x, int64_t n, int32_t D,
                    const float* t_w1, const float* t_b1, const float* t_gw, const float* t_gb,
                    const float* t_w2, const float* t_b2,
                    const float* p_w1, const float* p_b1, const float* p_gw, const float* p_gb,
                    const float* p_w2, const float* p_b2, float beta, float* out, void* stream);
/* RND.update_pred's gradient (PPO/RND.py:96-115: loss = MSELoss('mean')(pred(x), target(x)),
 * loss.backward()) for one minibatch x[n][D], fused: both forwards, dY = scale (pred - target)
 * (scale = 2 / (rows D) for the mean; a data-parallel rank passes 2 / (union rows D)), and the
 * predictor's whole backward, written to grad[129 D + 192] in the predictor's parameters() order
 * (W1[64][D], b1[64], gamma[64], beta[64], W2[D][64], b2[D]).  One launch per 128-row block into
 * partial[ceil(n / 128)][129 D + 192] (partial_floats >= prl_rnd_pred_grad_ws_floats(n, D)), then
 * a fold in a fixed order (f64: 16 segments of blocks, each in block order, then the segments in
 * order): deterministic.  D % 4 == 0; x, W1, W2, partial 16-B aligned. */
int prl_rnd_pred_grad(const float* x, int64_t n, int32_t D,
                      const float* t_w1, const float* t_b1, const float* t_gw, const float* t_gb,
                      const float* t_w2, const float* t_b2,
                      const float* p_w1, const float* p_b1, const float* p_gw, const float* p_gb,
                      const float* p_w2, const float* p_b2, float scale, float* partial,
                      int64_t partial_floats, float* grad, void* stream);
/* Floats of prl_rnd_pred_grad's partial buffer for n rows (0 for n <= 0). */
int64_t prl_rnd_pred_grad_ws_floats(int64_t n, int32_t D);

/* ---- actor-critic / RND hidden blocks ------------------------------------------------------ */
/* GroupNorm(groups=8, C=64, eps) + SiLU over x[N][64] (PPO/ActorCritic.py:19-60, PPO/RND.py:25-30):
 * out = silu(groupnorm(x) * w + b) (silu = 0: groupnorm only).  Replaces nn.GroupNorm + nn.SiLU on
 * device tensors (the PyTorch-ROCm GroupNorm backward in this image returns wrong dw/db for
 * N >= 512 rows).  x/out 16-B aligned. */
int prl_gn_silu_fwd(const float* x, int64_t N, int32_t C, int32_t groups, const float* w,
                    const float* b, float eps, int32_t silu, float* out, void* stream);
/* Backward of the above: dx[N][64], dw[64], db[64] (column sums over rows, deterministic). */
int prl_gn_silu_bwd(const float* x, const float* dout, int64_t N, int32_t C, int32_t groups,
                    const float* w, const float* b, float eps, int32_t silu, float* dx, float* dw,
                    float* db, void* workspace, int64_t workspace_bytes, void* stream);

/* ---- graph-captured optimizer step (PPO/PPO.py:219-255) ------------------------------------- */
/* Copy rows [cursor[0]*mb, cursor[0]*mb + mb) of `count` (<= 6) row-major float tensors (widths in
 * floats) into static minibatch buffers; rows past nrows are zero-filled.  srcs/dsts/widths are
 * HOST arrays of device pointers; cursor is a device int64 (the minibatch index j). */
int prl_gather_minibatch(const float* const* srcs, float* const* dsts, const int32_t* widths,
                         int32_t count, const int64_t* cursor, int64_t mb, int64_t nrows,
                         void* stream);
/* torch.distributions.Categorical(probs).log_prob(actions) and .entropy() per row
 * (ActorCritic.py:105,136-142): q = p/sum(p), logits = log(clamp(q, eps, 1-eps)).  entropy may be
 * NULL.  actions are float class indices (the reference stores them as float32). */
int prl_categorical_fwd(const float* probs, const float* actions, int64_t n, int32_t A,
                        float* logp, float* entropy, void* stream);
/* d log_prob / d probs for an upstream gradient dlogp[n]. */
int prl_categorical_bwd(const float* probs, const float* actions, const float* dlogp, int64_t n,
                        int32_t A, float* dprobs, void* stream);

/* ---- fused update engine (PPO/PPO.py:216-255 in ONE persistent launch) --------------------- */
/* Host call: parameter count, device workspace bytes and grid of the fused engine for the
 * reference's ActorCritic(is_continuous = !discrete, observ_dim = D, action_dim = A) at
 * mini_batch.  Returns PRL_ERR_ARG (all outputs 0) for shapes outside the engine (D > 64, A > 8,
 * LDS > 160 KiB): the caller then runs the per-step path. */
int prl_ppo_update_info(int32_t D, int32_t A, int32_t discrete, int64_t mini_batch,
                        int64_t* n_params, int64_t* workspace_bytes, int32_t* grid);
/* All k_epochs x ceil(N / mini_batch) optimizer steps of PPO.learn (PPO.py:216-255) in order:
 * per minibatch j (rows [j*mb, min((j+1)*mb, N)) of S/actions/old_logp/adv/ret, unshuffled):
 * ActorCritic.get_evaluate (ActorCritic.py:118-146), loss = mean(-min(surr1, surr2)) +
 * vf_coef * SmoothL1(V, ret) - ent_coef * H (PPO.py:225-245), its gradient,
 * clip_grad_norm_(max_norm) and AdamW(lr, (beta1, beta2), eps, weight_decay) — the betas as
 * doubles everywhere in this ABI (the reference forms 1 - beta and the bias corrections in
 * Python double precision; from a float32 0.999 they would be 1.3e-5 off).  params /
 * exp_avg / exp_avg_sq: the flat parameter vector and moments in torch parameters() order
 * (updated in place); adam_step: device f32 step count (read, then advanced by the step count);
 * loss_out: device f32, the last step's loss.  Workspace: prl_ppo_update_info's size (its status
 * word, see prl_ppo_update_status_ptr, is 0 after a good launch).  Cooperative launch. */
int prl_ppo_update(float* params, float* exp_avg, float* exp_avg_sq, float* adam_step, int32_t D,
                   int32_t A, int32_t discrete, const float* S, const float* actions,
                   const float* old_logp, const float* adv, const float* ret, int64_t N,
                   int32_t mini_batch, int32_t k_epochs, float clip, float vf_coef,
                   float ent_coef, float lr, double beta1, double beta2, float eps,
                   float weight_decay, float max_norm, float* loss_out, void* workspace,
                   int64_t workspace_bytes, void* stream);
/* ActorCritic.get_evaluate (ActorCritic.py:118-146) over N rows, as PPO.learn evaluates
 * policy_old (PPO.py:127-154): logp[N], V[N] and optionally entropy[N] (NULL = skip), with the
 * fused update's forward arithmetic (so learn()'s first minibatch has ratio == 1 exactly).
 * params: flat, torch parameters() order.  No workspace, no inter-workgroup communication. */
int prl_ppo_evaluate(const float* params, int32_t D, int32_t A, int32_t discrete, const float* S,
                     const float* actions, int64_t N, float* logp, float* V, float* entropy,
                     void* stream);
/* ---- stepped engine (world_size > 1: one launch pair per optimizer step, gradient all-reduced
 * by the caller between them; PPO.py:216-255 with the union of the ranks' j-th slices as the
 * global minibatch j).  Parameters and moments live in an "image" layout (padded, Lp floats) in
 * HBM for the whole loop. */
/* Host call: floats of one image (Lp) + 4 (the gradient vector's loss-partials quad). */
int64_t prl_ppo_image_floats(int32_t D, int32_t A, int32_t discrete);
/* flat torch vectors (parameters() order) <-> images; to_image != 0: flat -> image. */
int prl_ppo_image(int32_t D, int32_t A, int32_t discrete, float* params, float* exp_avg,
                  float* exp_avg_sq, float* img_params, float* img_m, float* img_v,
                  int32_t to_image, void* stream);
/* Gradient of this rank's rows [j*mb, min((j+1)*mb, N)) of the union minibatch j, scaled by
 * inv_count = 1 / (rows of the union), summed over the rank's rows into grad_out[Lp + 4] (last
 * quad: loss partials).  All-reduce grad_out (SUM) over the ranks before prl_ppo_adam_step. */
int prl_ppo_grad_step(const float* img_params, int32_t D, int32_t A, int32_t discrete,
                      const float* S, const float* actions, const float* old_logp,
                      const float* adv, const float* ret, int64_t N, int32_t mini_batch,
                      int64_t minibatch_index, float inv_count, float clip, float vf_coef,
                      float* grad_out, void* workspace, int64_t workspace_bytes, void* stream);
/* clip_grad_norm_(max_norm) + AdamW step number `step` (1-based) on the images from the
 * all-reduced gradient; loss_out (device f32, may be NULL) = that step's loss. */
int prl_ppo_adam_step(float* img_params, float* img_m, float* img_v, int32_t D, int32_t A,
                      int32_t discrete, const float* grad, int64_t step, float lr, double beta1,
                      double beta2, float eps, float weight_decay, float max_norm, float inv_count,
                      float vf_coef, float ent_coef, float* loss_out, void* stream);
/* One launch per optimizer step (what the data-parallel loops use): the PREVIOUS step's
 * clip_grad_norm_(max_norm) + AdamW (step number step_prev, its all-reduced gradient grad_prev,
 * state in_* -> out_*, loss_out = its loss with inv_count_prev) folded in front of this step's
 * prl_ppo_grad_step (minibatch j from the updated parameters) -> grad_out.  Bit-identical to
 * prl_ppo_adam_step followed by prl_ppo_grad_step.  in_* != out_* and grad_prev != grad_out (the
 * caller double-buffers: the launch's workgroups read `in` while each writes its slice of `out`).
 * grad_prev == NULL: no AdamW, parameters from in_p (the first step).  Replaces the per-step
 * optimizer.step() + next forward/backward of PPO.py:247-250 / :225-245. */
int prl_ppo_grad_fold_step(const float* in_p, const float* in_m, const float* in_v, float* out_p,
                           float* out_m, float* out_v, const float* grad_prev, int64_t step_prev,
                           float inv_count_prev, int32_t D, int32_t A, int32_t discrete,
                           const float* S, const float* actions, const float* old_logp,
                           const float* adv, const float* ret, int64_t N, int32_t mini_batch,
                           int64_t minibatch_index, float inv_count, float clip, float vf_coef,
                           float ent_coef, float lr, double beta1, double beta2, float eps,
                           float weight_decay, float max_norm, float* loss_out, float* grad_out,
                           void* workspace, int64_t workspace_bytes, void* stream);
/* ---- wide-net optimizer step (shapes outside the persistent engine: D <= 352, <= 48 outputs) -- */
/* Host call: parameter count, partial-gradient scratch floats and grid of prl_ppo_wide_grad for
 * ActorCritic(is_continuous = !discrete, D, A) at mini_batch; PRL_ERR_ARG (outputs 0) for shapes
 * outside it.  Replaces, for those shapes, the per-step forward + loss + backward of
 * PPO/PPO.py:219-249 (get_evaluate, the surrogate, loss.mean().backward()). */
int prl_ppo_wide_info(int32_t D, int32_t A, int32_t discrete, int64_t mini_batch,
                      int64_t* n_params, int64_t* part_floats, int32_t* grid);
/* One optimizer step's gradient: minibatch j = *cursor (device int64; rows [j*mb, min((j+1)*mb, N))
 * of S [N][D], actions [N][discrete ? 1 : A], old_logp, adv, ret), loss = mean(-min(surr1,
 * surr2)) + vf_coef * SmoothL1(V, ret) - ent_coef * H (PPO.py:225-245; H detached) times
 * scales[j] (device f32, null = 1), its gradient w.r.t. params (flat f32, torch parameters()
 * order) into grad [n_params], the loss into loss_out[0] (nullable).  part: prl_ppo_wide_info's
 * part_floats of scratch.  Two launches on `stream`, no host synchronisation (graph-capturable);
 * deterministic (fixed summation order). */
int prl_ppo_wide_grad(const float* params, int32_t D, int32_t A, int32_t discrete, const float* S,
                      const float* actions, const float* old_logp, const float* adv,
                      const float* ret, int64_t N, int64_t mini_batch, const int64_t* cursor,
                      const float* scales, float clip, float vf_coef, float ent_coef, float* grad,
                      float* loss_out, float* part, int64_t part_floats, void* stream);
/* ActorCritic.dist_params (PPO/ActorCritic.py: the rollout's sampling input; AsyncPPO.py:120-141
 * calls the policy on every vector step) for the wide nets: out = [N][A] softmax probabilities
 * (discrete) or [N][2A] = [mu | softplus(clamp(log_std, -2, 2))] (continuous), from the wide
 * kernel's forward; params flat in torch parameters() order.  One launch, graph-capturable. */
int prl_ppo_wide_dist(const float* params, int32_t D, int32_t A, int32_t discrete, const float* S,
                      int64_t N, float* out, void* stream);
/* prl_ppo_wide_dist on rows [k*rows, (k+1)*rows) of S ([N][D]), k = step_dev[0] read on the
 * device: the rollout's captured vector step samples from traj_obs[k] in place (reference
 * AsyncPPO.worker's get_action on the current observations, AsyncTools/AsyncPPO.py:120-141,
 * PPO/PPO.py:81-96).  out is [rows][A] or [rows][2A]. */
int prl_ppo_wide_dist_at(const float* params, int32_t D, int32_t A, int32_t discrete,
                         const float* S, int64_t N, int64_t rows, const int64_t* step_dev,
                         float* out, void* stream);
/* policy_old.get_evaluate over all N rows for the wide nets (PPO/PPO.py:127-154,
 * ActorCritic.py:118-146): log_prob into logp_out [N] and the state value into V_out [N], with
 * exactly prl_ppo_wide_grad's forward and row arithmetic, so the first minibatch of learn() sees
 * ratio == 1 exactly, as in the reference (one get_evaluate for both).  One launch. */
int prl_ppo_wide_evaluate(const float* params, int32_t D, int32_t A, int32_t discrete,
                          const float* S, const float* actions, int64_t N, float* logp_out,
                          float* V_out, void* stream);
/* prl_ppo_wide_grad with workgroup 0's s_memrealtime ticks (100 MHz) per tile stage added into
 * prof[8] (stage, trunk, heads, outputs, loss, heads bwd, dW1 + dF, dW0); diagnostics. */
int prl_ppo_wide_grad_prof(const float* params, int32_t D, int32_t A, int32_t discrete,
                           const float* S, const float* actions, const float* old_logp,
                           const float* adv, const float* ret, int64_t N, int64_t mini_batch,
                           const int64_t* cursor, const float* scales, float clip, float vf_coef,
                           float ent_coef, float* grad, float* loss_out, float* part,
                           int64_t part_floats, unsigned long long* prof, void* stream);
/* Column sums out[c] = sum_r x[r][c] of a row-major f32 matrix (cols >= 1): the bias
 * gradient of a Linear over a large batch (nn.Linear backward, reached from PPO.py:249 /
 * RND.py:112).  Two deterministic passes; `partial` holds prl_colsum_partial_floats(rows, cols)
 * floats of scratch. */
int64_t prl_colsum_partial_floats(int64_t rows, int32_t cols);
int prl_colsum_f32(const float* x, int64_t rows, int32_t cols, float* out, float* partial,
                   int64_t partial_floats, void* stream);
/* nn.utils.clip_grad_norm_(params, max_norm) followed by AdamW.step() (PPO/PPO.py:248-250; torch
 * defaults, capturable: the update uses step[0] + 1, and step[0] f32 on the device is advanced)
 * over FLAT f32 vectors of P entries in parameters() order: params, exp_avg, exp_avg_sq and grad
 * (left clipped, as torch leaves p.grad).  The norm is summed in float64 in a fixed order
 * (deterministic) and stored to total_norm[0] (f32, what clip_grad_norm_ returns); total_norm[1]
 * is a u32 arrival counter that must be zero before the first call (every call leaves it zero):
 * the last workgroup to finish clips grad and advances the step.  One launch up to 262,144
 * parameters (two above: update; clip of grad + step count), graph-capturable; the wide step's
 * optimizer tail (PPO/update.py) and the RND predictor's AdamW.  16-B aligned buffers. */
int prl_flat_adamw(float* params, float* exp_avg, float* exp_avg_sq, float* step, float* grad,
                   int64_t P, float lr, double beta1, double beta2, float eps, float weight_decay,
                   float max_norm, float* total_norm, void* stream);
/* Host call: device address of the u32 status words inside an engine workspace ([0] last
 * launch, [1] sticky timeout flag). */
int prl_ppo_update_status_ptr(void* workspace, uint32_t** status);
/* The engine's timing words in `workspace` (u64[32]: workgroup 0's s_memrealtime ticks per phase
 * and per tile stage, summed over the launch's steps; [7] = steps; [30], [31] = wall ticks and
 * shader clocks of the launch).  Instrumentation of this build, no reference counterpart. */
int prl_ppo_update_profile_ptr(void* workspace, uint64_t** prof);

/* ---- data-parallel update loop (world > 1): PPO.py:216-255 per rank, one optimizer step =
 * one prl_ppo_grad_fold_step launch (previous AdamW + this gradient) -> all-reduce of the
 * gradient image (the last step's AdamW: one prl_ppo_adam_step), enqueued from C
 * (no Python per step).  RCCL is resolved at run time from `lib_path` (the librccl torch
 * loaded); the communicator is the engine's own, built from a unique id the caller broadcasts
 * over torch.distributed.  No reference counterpart (the reference is single-process). */
int prl_dp_rccl_open(const char* lib_path);
int prl_dp_unique_id(uint8_t* id_out, int64_t id_bytes);
int prl_dp_comm_init(const uint8_t* id, int64_t id_bytes, int32_t nranks, int32_t rank,
                     void** comm);
int prl_dp_comm_destroy(void* comm);
/* counts[j] = rows of union minibatch j over all ranks (host array, nb entries); step0 = AdamW
 * steps taken so far.  Semantics = nb x k_epochs calls of prl_ppo_grad_step(j, 1 / counts[j])
 * + all-reduce + prl_ppo_adam_step(step0 + 1 + ...), bit for bit. */
int prl_ppo_update_dp(float* img_params, float* img_m, float* img_v, int32_t D, int32_t A,
                      int32_t discrete, const float* S, const float* actions,
                      const float* old_logp, const float* adv, const float* ret, int64_t N,
                      int32_t mini_batch, int32_t k_epochs, int64_t nb, const int64_t* counts,
                      int64_t step0, float clip, float vf_coef, float ent_coef, float lr,
                      double beta1, double beta2, float eps, float weight_decay, float max_norm,
                      float* grad, float* loss_out, void* workspace, int64_t workspace_bytes,
                      void* comm, void* stream);

/* ---- data-parallel persistent update (world > 1, opt-in PRL_DP_PERSISTENT=1): PPO.py:216-255
 * per rank as ONE launch of the persistent engine (prl_ppo_update) per rank, the cross-rank sum
 * done inside it: after each step's in-GPU slice reduction, workgroup g publishes its rank's
 * slice in its own slice buffer, raises a per-step flag, waits for workgroup g of every rank and
 * sums their slices in rank order (float32) over IPC-mapped peer memory — no RCCL call, no
 * host work per step.  nb_union = minibatches of the union (max over ranks); inv_count = device
 * [nb_union], float(1 / rows of union minibatch j); xbufs = host array of `world` slice-buffer
 * pointers (this rank's own, and the others' opened with prl_dp_ipc_open), each
 * prl_dp_xbuf_bytes long, allocated by prl_dp_xbuf_alloc (zeroed once).  seq0 = the exchange
 * sequence number of this launch's first step: 0 for the first launch on a buffer set, then
 * advanced by nb_union x k_epochs per launch, the same on every rank (the flags only grow, so
 * one buffer set serves every later launch).  All ranks' launches must be resident together.
 * fine_grained != 0 when ANY rank's slice buffer is fine-grained memory (prl_dp_xbuf_alloc's
 * fallback): each workgroup then orders its slice stores before its flag with a system-scope
 * release fence and its slice loads after the poll with a system-scope acquire fence (the
 * uncached form relies on write-through system-scope stores and cache-missing loads instead).
 * fine_grained is a bit field: bit 0 the above; bit 1 the push form of the exchange (the
 * head-split kernel's); bit 2 forces the 8-wave kernel (no head split) — the ranks' kernel
 * choice must be the same everywhere, so the caller votes with prl_ppo_update_dp_split and sets
 * bit 2 unless every rank would run the split form.
 * No reference counterpart (the reference is single-process). */
int prl_ppo_update_dpx(float* params, float* exp_avg, float* exp_avg_sq, float* adam_step,
                       int32_t D, int32_t A, int32_t discrete, const float* S,
                       const float* actions, const float* old_logp, const float* adv,
                       const float* ret, int64_t N, int32_t mini_batch, int32_t k_epochs,
                       int32_t nb_union, const float* inv_count, float clip, float vf_coef,
                       float ent_coef, float lr, double beta1, double beta2, float eps,
                       float weight_decay, float max_norm, float* loss_out, int32_t world,
                       int32_t rank, void* const* xbufs, int64_t seq0, int32_t fine_grained,
                       void* workspace, int64_t workspace_bytes, void* stream);
int64_t prl_dp_xbuf_bytes(int32_t D, int32_t A, int32_t discrete, int32_t mini_batch);
/* polls of prl_ppo_update_dpx's cross-rank wait before it gives up (the launch then ends with a
 * nonzero status word and the caller restores its snapshot, PPO/engine.py); 0 restores the
 * default (2^24 polls, each a system-scope load: seconds, which also absorbs launch skew between
 * the ranks).  Per process; returns the previous value.  Tests lower it to exercise the failure
 * path.  No reference counterpart. */
uint32_t prl_dp_set_spin_limit(uint32_t polls);
/* Form of prl_ppo_update's persistent kernel: 0 = the latency form (gradient image in LDS,
 * AdamW moments in registers), 1 = the throughput form whenever a launch has >= 2 steps
 * (gradient in registers, moments streamed from the workspace), 2 = auto (default: the
 * throughput form when a workgroup takes >= 2 16-row tiles per step).  Both give the same bits.
 * Per process (initial value from PRL_UPD_TP); returns the previous mode.  No reference
 * counterpart (performance knob / tests). */
int32_t prl_ppo_update_set_tp(int32_t mode);
/* Replicas per tile group of the latency form (single GPU): every 16-row tile of a step runs on
 * `replicas` workgroups at once, each publishing 1/replicas of the tile's partial gradient; the
 * grid grows to tiles x replicas, capped at one workgroup per CU.  Same bits at every value.
 * Per process (initial value from PRL_UPD_REPL); returns the previous value.  No reference
 * counterpart (performance knob / tests). */
int32_t prl_ppo_update_set_repl(int32_t replicas);
/* The head-split latency form (csrc/prl_ppo_split.h: the actor and the critic head of a 16-row
 * tile on two workgroups) for the two-head CartPole shape: 1 = on (default, PRL_UPD_SPLIT), 0 =
 * the 8-wave kernel.  Per process; returns the previous value.  No reference counterpart
 * (performance knob / tests). */
int32_t prl_ppo_update_set_split(int32_t mode);
/* 1 when a prl_ppo_update_dpx launch of this shape and mini_batch would run the head-split kernel
 * in this process (the split mode above, the shape, and 2 x tile groups <= the CUs), else 0: the
 * data-parallel caller's vote (every rank must launch the same kernel form).  No reference
 * counterpart. */
int32_t prl_ppo_update_dp_split(int32_t D, int32_t A, int32_t discrete, int32_t mini_batch);
/* Host-only check (no GPU): 1 when the head-split kernel's wave-block AdamW lists
 * (csrc/prl_ppo_split.h spl_wb_quad: wave b of role h updates, and publishes, the parameter quads
 * its own next forward reads before the tile's first barrier) cover every quad role h owns
 * exactly once for this shape, else 0.  The launch refuses a shape that fails it.  No reference
 * counterpart (tests). */
int32_t prl_ppo_update_wb_check(int32_t D, int32_t A, int32_t discrete);
/* Test utility: fill every CU's LDS with `value` (LDS is not cleared between launches; a kernel
 * that reads LDS it did not write in its own launch sees the previous launch's contents).  No
 * reference counterpart. */
int prl_debug_fill_lds(float value, void* stream);
/* What the last prl_ppo_update / prl_ppo_update_dpx call in this process launched:
 * out[0] = 1 for the throughput form, 0 for the latency form; out[1] = waves per workgroup;
 * out[2] = workgroups; out[3] = 16-row tiles per workgroup and step (ceil of rows / 16 / G);
 * out[4] = 1 for a compile-time-layout (CartPole / Pendulum) kernel, 0 for the runtime layout;
 * out[5] = workgroups per tile group (the latency form's replicated tiles, PRL_UPD_REPL; out[2]
 * counts them all; the split form: its two head roles); out[6] = 1 for the head-split latency
 * form, 2 for its slice-owner variant (AdamW by the slice owners, PRL_UPD_SPL_OWN); out[7] = the
 * split form's phase-B helper workgroups (launched beside out[2]; PRL_UPD_SPL_HELP).  All -1
 * before the first launch.  No reference counterpart (tests assert which kernel ran).
 * (ABI 2: out has 8 entries; ABI 1 had 7.) */
void prl_ppo_update_last_plan(int32_t out[8]);
/* A zeroed slice buffer of its own (shareable by IPC handle).  *kind in: 0 = uncached, falling
 * back to fine-grained memory, 1 = uncached only, 2 = fine-grained only; out: 1 = uncached,
 * 2 = fine-grained (what the buffer is; prl_ppo_update_dpx's fine_grained follows it). */
int prl_dp_xbuf_alloc(int64_t bytes, int32_t* kind, void** out);
int prl_dp_xbuf_free(void* p);
int prl_dp_ipc_handle(void* p, uint8_t* out, int64_t out_bytes);   /* out: 64 bytes */
int prl_dp_ipc_open(const uint8_t* handle, int64_t bytes, void** out);
int prl_dp_ipc_close(void* p);

#ifdef __cplusplus
}
#endif

#endif /* PRL_ABI_H */
