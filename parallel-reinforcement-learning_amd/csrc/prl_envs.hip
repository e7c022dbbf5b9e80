// prl_envs.hip — batched gymnasium classic-control envs + the fused device-resident rollout step.
//
// Replaces, for the hot path of AsyncTools.AsyncPPO.worker (AsyncTools/AsyncPPO.py:117-146):
//   EnvVectorizer.reset/step (AsyncPPO.py:48-102) over deep-copied gymnasium envs,
//   PPO.get_action's sampling (PPO/PPO.py:85-91),
//   utils.buffer_append + VecMemory.push (utils.py:17-36, AsyncPPO.py:20-24),
//   utils.update_active_environments_list (utils.py:38-43) and the score counters (:137-138).
//
// The physics restates gymnasium==1.1.1 (requirements.txt:4; third-party, absent from the
// reference tree) CartPoleEnv / PendulumEnv + TimeLimit: float64 state, the exact operation
// order of the numpy scalar code, compiled with -ffp-contract=off.  Trig is prl_sin/prl_cos
// (fdlibm) on both this side and the CPU oracle.
//
// HBM layout (per env batch, E envs): phys f64[E][P] (AoS: one 16/32-B row per env, coalesced
// 16-B loads), t_elapsed i32[E], terminal u8[E] (reference envs_active: True = terminal),
// trajectory buffers time-major [t][E][..] so that one vector step writes contiguous rows and the
// policy's input for step t is the contiguous slice traj_obs[t].
#include "prl_common.h"
#include "prl_envs.h"

#include <math.h>

namespace prl {

// ---------------------------------------------------------------------------------------------
__global__ void pcg64_seed_kernel(const uint64_t* seeds, int64_t E, uint64_t* rng) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const pcg64 g = pcg64_from_seed(seeds[e]);
  rng[4 * e + 0] = g.shi; rng[4 * e + 1] = g.slo; rng[4 * e + 2] = g.ihi; rng[4 * e + 3] = g.ilo;
}

__device__ inline pcg64 load_pcg(const uint64_t* rng, int64_t e) {
  return pcg64{rng[4 * e], rng[4 * e + 1], rng[4 * e + 2], rng[4 * e + 3]};
}
__device__ inline void store_pcg(uint64_t* rng, int64_t e, const pcg64& g) {
  rng[4 * e] = g.shi; rng[4 * e + 1] = g.slo; rng[4 * e + 2] = g.ihi; rng[4 * e + 3] = g.ilo;
}

template <class Env>
__global__ void reset_kernel(int64_t E, double* phys, uint64_t* rng, int32_t* t_elapsed,
                             uint8_t* terminal, const uint8_t* reset_mask, float* obs,
                             int64_t obs_stride) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  if (reset_mask && !reset_mask[e]) return;
  pcg64 g = load_pcg(rng, e);
  double s[Env::P];
  Env::reset(s, g);
  store_pcg(rng, e, g);
  for (int i = 0; i < Env::P; ++i) phys[e * Env::P + i] = s[i];
  float o[Env::D];
  Env::obs(s, o);
  for (int i = 0; i < Env::D; ++i) obs[e * obs_stride + i] = o[i];
  t_elapsed[e] = 0;
  terminal[e] = 0;
}

// synthetic env reset: one wave per env (obs rows are 1392 B: lanes stride over j, coalesced)
__global__ void synth_reset_kernel(int64_t E, double* phys, uint64_t* rng, int32_t* t_elapsed,
                                   uint8_t* terminal, const uint8_t* reset_mask, float* obs,
                                   int64_t obs_stride) {
  const int64_t e = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= E) return;
  if (reset_mask && !reset_mask[e]) return;
  pcg64 g = load_pcg(rng, e);
  const uint64_t key = pcg64_next64(g);
  for (int j = lane; j < Synth::D; j += 64) obs[e * obs_stride + j] = Synth::obs_at(key, 0u, (uint32_t)j);
  if (lane == 0) {
    store_pcg(rng, e, g);
    phys[2 * e] = (double)Synth::episode_len(key);
    phys[2 * e + 1] = __builtin_bit_cast(double, key);
    t_elapsed[e] = 0;
    terminal[e] = 0;
  }
}

// EnvVectorizer.step compat form: row i <-> env active_idx[i].
template <class Env, bool DISCRETE>
__global__ void step_compact_kernel(int64_t E, double* phys, int32_t* t_elapsed,
                                    const int64_t* active_idx, int64_t n, const void* actions,
                                    float* obs_out, double* reward_out, uint8_t* terminated_out,
                                    uint8_t* truncated_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t e = active_idx[i];
  if (e < 0 || e >= E) return;
  double s[Env::P];
  for (int k = 0; k < Env::P; ++k) s[k] = phys[e * Env::P + k];
  double reward;
  bool term;
  if constexpr (DISCRETE) {
    const int64_t a = reinterpret_cast<const int64_t*>(actions)[i];
    term = Env::step(s, (int)a, reward);
  } else {
    const float a = reinterpret_cast<const float*>(actions)[i * Env::A];
    term = Env::step(s, a, reward);
  }
  for (int k = 0; k < Env::P; ++k) phys[e * Env::P + k] = s[k];
  const int32_t t = t_elapsed[e] + 1;
  t_elapsed[e] = t;
  float o[Env::D];
  Env::obs(s, o);
  for (int k = 0; k < Env::D; ++k) obs_out[i * Env::D + k] = o[k];
  reward_out[i] = reward;
  terminated_out[i] = term ? 1 : 0;
  truncated_out[i] = (t >= Env::TMAX) ? 1 : 0;
}

__global__ void synth_step_compact_kernel(int64_t E, double* phys, int32_t* t_elapsed,
                                          const int64_t* active_idx, int64_t n,
                                          const float* actions, float* obs_out,
                                          double* reward_out, uint8_t* terminated_out,
                                          uint8_t* truncated_out) {
  const int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const int64_t e = active_idx[i];
  if (e < 0 || e >= E) return;
  const uint32_t L = (uint32_t)phys[2 * e];
  const uint64_t key = __builtin_bit_cast(uint64_t, phys[2 * e + 1]);
  const int32_t t = t_elapsed[e] + 1;
  for (int j = lane; j < Synth::D; j += 64) obs_out[i * Synth::D + j] = Synth::obs_at(key, (uint32_t)t, (uint32_t)j);
  if (lane == 0) {
    float acc = 0.f;
    for (int j = 0; j < Synth::A; ++j) {
      const float a = actions[i * Synth::A + j];
      acc += a * a;
    }
    reward_out[i] = (double)(1.0f - 0.01f * acc);
    terminated_out[i] = ((uint32_t)t >= L) ? 1 : 0;
    truncated_out[i] = (t >= Synth::TMAX) ? 1 : 0;
    t_elapsed[e] = t;
  }
}

// ---------------------------------------------------------------------------------------------
// End of a rollout step block (thread 0): add the block's still-active count to the step's slot.
// Eager form (step_dev null): active_after_step is the slot.  Captured form (prl_rollout_step_at):
// step_dev = {k, arrivals}; the count goes to active_after[k] (skipped outside [0, t_max): a
// stale k never writes past the store), and the last block to arrive advances k and re-arms the
// arrival counter, so the captured vector step needs no separate increment node.
__device__ __forceinline__ void rollout_count_and_advance(int ct, int32_t* active_after_step,
                                                          int64_t* step_dev, int32_t t_max) {
  if (!step_dev) {
    if (ct) atomicAdd(active_after_step, ct);
    return;
  }
  const int64_t k = step_dev[0];
  if (ct && k >= 0 && k < t_max) atomicAdd(active_after_step + k, ct);
  __threadfence();   // this block's read of k (and its count) before its arrival
  const unsigned long long prev =
      atomicAdd(reinterpret_cast<unsigned long long*>(step_dev + 1), 1ull);
  if (prev == (unsigned long long)gridDim.x - 1) {   // every other block has read k
    step_dev[1] = 0;
    step_dev[0] = k + 1;
  }
}

// ---------------------------------------------------------------------------------------------
// The fused rollout step (thread per env) for the classic-control envs.
template <class Env, bool DISCRETE>
__global__ __launch_bounds__(256) void rollout_step_kernel(
    int64_t E, double* __restrict__ phys, int32_t* __restrict__ t_elapsed,
    uint8_t* __restrict__ terminal, const float* __restrict__ dist, int64_t dist_stride,
    float action_scaling, uint64_t seed, int32_t t_max, float* __restrict__ traj_obs,
    float* __restrict__ traj_act, float* __restrict__ traj_rew, uint8_t* __restrict__ traj_done,
    int32_t* __restrict__ ep_len, int32_t* __restrict__ active_after_step,
    double* __restrict__ reward_sum, int64_t* step_dev) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int still_active = 0;
  double rew = 0.0;
  if (e < E && !terminal[e]) {
    const int32_t t = t_elapsed[e];
    double s[Env::P];
    if constexpr (Env::P == 4) {
      const double4 v = reinterpret_cast<const double4*>(phys)[e];
      s[0] = v.x; s[1] = v.y; s[2] = v.z; s[3] = v.w;
    } else {
      const double2 v = reinterpret_cast<const double2*>(phys)[e];
      s[0] = v.x; s[1] = v.y;
    }
    const float* drow = dist + e * dist_stride;
    float act;
    bool term;
    if constexpr (DISCRETE) {
      float p[2] = {drow[0], drow[1]};
      const int a = sample_categorical(p, 2, seed, (uint32_t)e, (uint32_t)t);
      act = (float)a;
      term = Env::step(s, a, rew);
    } else {
      const float mu = drow[0], sd = drow[Env::A];
      const float z = sample_normal(seed, (uint32_t)e, (uint32_t)t, 0u);
      act = tanhf(mu + sd * z) * action_scaling;
      term = Env::step(s, act, rew);
    }
    const int32_t t1 = t + 1;
    const bool done = term || (t1 >= Env::TMAX) || (t1 >= t_max);
    if constexpr (Env::P == 4) {
      reinterpret_cast<double4*>(phys)[e] = double4{s[0], s[1], s[2], s[3]};
    } else {
      reinterpret_cast<double2*>(phys)[e] = double2{s[0], s[1]};
    }
    float o[Env::D];
    Env::obs(s, o);
    float* orow = traj_obs + ((int64_t)t1 * E + e) * Env::D;
    if constexpr (Env::D == 4) {
      *reinterpret_cast<float4*>(orow) = float4{o[0], o[1], o[2], o[3]};
    } else {
      for (int k = 0; k < Env::D; ++k) orow[k] = o[k];
    }
    const int64_t slot = (int64_t)t * E + e;
    traj_act[slot] = act;
    traj_rew[slot] = (float)rew;
    traj_done[slot] = done ? 1 : 0;
    t_elapsed[e] = t1;
    ep_len[e] = t1;
    terminal[e] = done ? 1 : 0;
    still_active = done ? 0 : 1;
  }
  // block reduction of the counters -> one atomic per block
  __shared__ int s_cnt[4];
  __shared__ double s_rew[4];
  int c = wave_sum(still_active);
  double r = wave_sum(rew);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { s_cnt[wid] = c; s_rew[wid] = r; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int ct = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    const double rt = s_rew[0] + s_rew[1] + s_rew[2] + s_rew[3];
    if (rt != 0.0) atomicAdd(reward_sum, rt);
    rollout_count_and_advance(ct, active_after_step, step_dev, t_max);
  }
}

// Synthetic env rollout step: one wave per env; lanes 0..16 sample the 17 action dims, all
// lanes write the 348-float next observation.
__global__ __launch_bounds__(256) void synth_rollout_step_kernel(
    int64_t E, double* __restrict__ phys, int32_t* __restrict__ t_elapsed,
    uint8_t* __restrict__ terminal, const float* __restrict__ dist, int64_t dist_stride,
    float action_scaling, uint64_t seed, int32_t t_max, float* __restrict__ traj_obs,
    float* __restrict__ traj_act, float* __restrict__ traj_rew, uint8_t* __restrict__ traj_done,
    int32_t* __restrict__ ep_len, int32_t* __restrict__ active_after_step,
    double* __restrict__ reward_sum, int64_t* step_dev) {
  const int64_t e = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __shared__ float s_a2[4][64];
  __shared__ int s_cnt[4];
  __shared__ double s_rew[4];
  int still_active = 0;
  double rew = 0.0;
  const bool live = (e < E) && !terminal[e];
  if (live) {
    const int32_t t = t_elapsed[e];
    const int32_t t1 = t + 1;
    const uint64_t key = __builtin_bit_cast(uint64_t, phys[2 * e + 1]);
    const uint32_t L = (uint32_t)phys[2 * e];
    float a = 0.f;
    if (lane < Synth::A) {
      const float* drow = dist + e * dist_stride;
      const float z = sample_normal(seed, (uint32_t)e, (uint32_t)t, (uint32_t)lane);
      a = tanhf(drow[lane] + drow[Synth::A + lane] * z) * action_scaling;
      traj_act[((int64_t)t * E + e) * Synth::A + lane] = a;
    }
    s_a2[wid][lane] = a * a;
    float* orow = traj_obs + ((int64_t)t1 * E + e) * Synth::D;
    for (int j = lane; j < Synth::D; j += 64) orow[j] = Synth::obs_at(key, (uint32_t)t1, (uint32_t)j);
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      float acc = 0.f;
      for (int j = 0; j < Synth::A; ++j) acc += s_a2[wid][j];
      const float r = 1.0f - 0.01f * acc;
      const bool done = ((uint32_t)t1 >= L) || (t1 >= Synth::TMAX) || (t1 >= t_max);
      const int64_t slot = (int64_t)t * E + e;
      traj_rew[slot] = r;
      traj_done[slot] = done ? 1 : 0;
      t_elapsed[e] = t1;
      ep_len[e] = t1;
      terminal[e] = done ? 1 : 0;
      still_active = done ? 0 : 1;
      rew = (double)r;
    }
  }
  if (lane == 0) { s_cnt[wid] = still_active; s_rew[wid] = rew; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int ct = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    const double rt = s_rew[0] + s_rew[1] + s_rew[2] + s_rew[3];
    if (rt != 0.0) atomicAdd(reward_sum, rt);
    rollout_count_and_advance(ct, active_after_step, step_dev, t_max);
  }
}

}  // namespace prl

// ============================================================================= C-ABI ========
using namespace prl;

extern "C" int prl_env_dims(int kind, int* obs_dim, int* act_dim, int* phys_dim,
                            int* max_episode_steps, int* is_discrete) {
  int D, A, P, T, disc;
  switch (kind) {
    case PRL_ENV_CARTPOLE: D = CartPole::D; A = 2; P = CartPole::P; T = CartPole::TMAX; disc = 1; break;
    case PRL_ENV_PENDULUM: D = Pendulum::D; A = 1; P = Pendulum::P; T = Pendulum::TMAX; disc = 0; break;
    case PRL_ENV_SYNTH_HUMANOID: D = Synth::D; A = Synth::A; P = Synth::P; T = Synth::TMAX; disc = 0; break;
    default: return set_error(PRL_ERR_ARG, "prl_env_dims: unknown env kind %d", kind);
  }
  if (obs_dim) *obs_dim = D;
  if (act_dim) *act_dim = A;
  if (phys_dim) *phys_dim = P;
  if (max_episode_steps) *max_episode_steps = T;
  if (is_discrete) *is_discrete = disc;
  return PRL_OK;
}

extern "C" int prl_pcg64_seed(const uint64_t* seeds, int64_t E, uint64_t* rng, void* stream) {
  PRL_REQUIRE(E >= 0, "prl_pcg64_seed: E < 0");
  if (E == 0) return PRL_OK;
  PRL_REQUIRE(seeds && rng, "prl_pcg64_seed: null pointer");
  hipLaunchKernelGGL(pcg64_seed_kernel, dim3((unsigned)cdiv(E, 256)), dim3(256), 0,
                     as_stream(stream), seeds, E, rng);
  PRL_LAUNCH_CHECK("pcg64_seed");
  return PRL_OK;
}

extern "C" int prl_env_reset(int kind, int64_t E, double* phys, uint64_t* rng, int32_t* t_elapsed,
                             uint8_t* terminal, const uint8_t* reset_mask, float* obs,
                             int64_t obs_stride, void* stream) {
  PRL_REQUIRE(E >= 0, "prl_env_reset: E < 0");
  if (E == 0) return PRL_OK;
  PRL_REQUIRE(phys && rng && t_elapsed && terminal && obs, "prl_env_reset: null pointer");
  hipStream_t s = as_stream(stream);
  switch (kind) {
    case PRL_ENV_CARTPOLE:
      PRL_REQUIRE(obs_stride >= CartPole::D, "prl_env_reset: obs_stride < obs dim");
      hipLaunchKernelGGL(reset_kernel<CartPole>, dim3((unsigned)cdiv(E, 256)), dim3(256), 0, s, E,
                         phys, rng, t_elapsed, terminal, reset_mask, obs, obs_stride);
      break;
    case PRL_ENV_PENDULUM:
      PRL_REQUIRE(obs_stride >= Pendulum::D, "prl_env_reset: obs_stride < obs dim");
      hipLaunchKernelGGL(reset_kernel<Pendulum>, dim3((unsigned)cdiv(E, 256)), dim3(256), 0, s, E,
                         phys, rng, t_elapsed, terminal, reset_mask, obs, obs_stride);
      break;
    case PRL_ENV_SYNTH_HUMANOID:
      PRL_REQUIRE(obs_stride >= Synth::D, "prl_env_reset: obs_stride < obs dim");
      hipLaunchKernelGGL(synth_reset_kernel, dim3((unsigned)cdiv(E, 4)), dim3(256), 0, s, E, phys,
                         rng, t_elapsed, terminal, reset_mask, obs, obs_stride);
      break;
    default: return set_error(PRL_ERR_ARG, "prl_env_reset: unknown env kind %d", kind);
  }
  PRL_LAUNCH_CHECK("env_reset");
  return PRL_OK;
}

extern "C" int prl_env_step_compact(int kind, int64_t E, double* phys, int32_t* t_elapsed,
                                    const int64_t* active_idx, int64_t n, const void* actions,
                                    float* obs_out, double* reward_out, uint8_t* terminated_out,
                                    uint8_t* truncated_out, void* stream) {
  PRL_REQUIRE(E >= 0 && n >= 0 && n <= E, "prl_env_step_compact: bad sizes E=%lld n=%lld",
              (long long)E, (long long)n);
  if (n == 0) return PRL_OK;
  PRL_REQUIRE(phys && t_elapsed && active_idx && actions && obs_out && reward_out &&
                  terminated_out && truncated_out,
              "prl_env_step_compact: null pointer");
  hipStream_t s = as_stream(stream);
  switch (kind) {
    case PRL_ENV_CARTPOLE:
      hipLaunchKernelGGL((step_compact_kernel<CartPole, true>), dim3((unsigned)cdiv(n, 256)),
                         dim3(256), 0, s, E, phys, t_elapsed, active_idx, n, actions, obs_out,
                         reward_out, terminated_out, truncated_out);
      break;
    case PRL_ENV_PENDULUM:
      hipLaunchKernelGGL((step_compact_kernel<Pendulum, false>), dim3((unsigned)cdiv(n, 256)),
                         dim3(256), 0, s, E, phys, t_elapsed, active_idx, n, actions, obs_out,
                         reward_out, terminated_out, truncated_out);
      break;
    case PRL_ENV_SYNTH_HUMANOID:
      hipLaunchKernelGGL(synth_step_compact_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0, s,
                         E, phys, t_elapsed, active_idx, n, (const float*)actions, obs_out,
                         reward_out, terminated_out, truncated_out);
      break;
    default: return set_error(PRL_ERR_ARG, "prl_env_step_compact: unknown env kind %d", kind);
  }
  PRL_LAUNCH_CHECK("env_step_compact");
  return PRL_OK;
}

static int rollout_step_launch(int kind, int64_t E, int32_t step, int64_t* step_dev,
                               double* phys, int32_t* t_elapsed, uint8_t* terminal,
                               const float* dist, int64_t dist_stride, float action_scaling,
                               uint64_t sample_seed, int32_t t_max, float* traj_obs,
                               float* traj_act, float* traj_rew, uint8_t* traj_done,
                               int32_t* ep_len, int32_t* active_after, double* reward_sum,
                               void* stream) {
  PRL_REQUIRE(E >= 0 && step >= 0 && t_max > 0, "prl_rollout_step: bad sizes");
  if (E == 0) return PRL_OK;
  PRL_REQUIRE(phys && t_elapsed && terminal && dist && traj_obs && traj_act && traj_rew &&
                  traj_done && ep_len && active_after && reward_sum,
              "prl_rollout_step: null pointer");
  PRL_REQUIRE(aligned16(phys) && aligned16(traj_obs), "prl_rollout_step: phys/traj_obs must be 16-B aligned");
  hipStream_t s = as_stream(stream);
  int32_t* aa = active_after + step;
  switch (kind) {
    case PRL_ENV_CARTPOLE:
      PRL_REQUIRE(dist_stride >= 2, "prl_rollout_step: dist_stride < 2 for CartPole probs");
      hipLaunchKernelGGL((rollout_step_kernel<CartPole, true>), dim3((unsigned)cdiv(E, 256)),
                         dim3(256), 0, s, E, phys, t_elapsed, terminal, dist, dist_stride,
                         action_scaling, sample_seed, t_max, traj_obs, traj_act, traj_rew,
                         traj_done, ep_len, aa, reward_sum, step_dev);
      break;
    case PRL_ENV_PENDULUM:
      PRL_REQUIRE(dist_stride >= 2, "prl_rollout_step: dist_stride < 2 for Pendulum mu/std");
      hipLaunchKernelGGL((rollout_step_kernel<Pendulum, false>), dim3((unsigned)cdiv(E, 256)),
                         dim3(256), 0, s, E, phys, t_elapsed, terminal, dist, dist_stride,
                         action_scaling, sample_seed, t_max, traj_obs, traj_act, traj_rew,
                         traj_done, ep_len, aa, reward_sum, step_dev);
      break;
    case PRL_ENV_SYNTH_HUMANOID:
      PRL_REQUIRE(dist_stride >= 2 * Synth::A, "prl_rollout_step: dist_stride < 34 for synth mu/std");
      hipLaunchKernelGGL(synth_rollout_step_kernel, dim3((unsigned)cdiv(E, 4)), dim3(256), 0, s, E,
                         phys, t_elapsed, terminal, dist, dist_stride, action_scaling, sample_seed,
                         t_max, traj_obs, traj_act, traj_rew, traj_done, ep_len, aa, reward_sum,
                         step_dev);
      break;
    default: return set_error(PRL_ERR_ARG, "prl_rollout_step: unknown env kind %d", kind);
  }
  PRL_LAUNCH_CHECK("rollout_step");
  return PRL_OK;
}

extern "C" int prl_rollout_step(int kind, int64_t E, int32_t step, double* phys, int32_t* t_elapsed,
                                uint8_t* terminal, const float* dist, int64_t dist_stride,
                                float action_scaling, uint64_t sample_seed, int32_t t_max,
                                float* traj_obs, float* traj_act, float* traj_rew,
                                uint8_t* traj_done, int32_t* ep_len, int32_t* active_after,
                                double* reward_sum, void* stream) {
  return rollout_step_launch(kind, E, step, nullptr, phys, t_elapsed, terminal, dist, dist_stride,
                             action_scaling, sample_seed, t_max, traj_obs, traj_act, traj_rew,
                             traj_done, ep_len, active_after, reward_sum, stream);
}

// The graphed vector step: the count goes to active_after[step_dev[0]] (step index read on the
// device) and the kernel advances step_dev[0] itself, so the captured graph needs no per-step
// scalar, zero fill, index copy or increment.
extern "C" int prl_rollout_step_at(int kind, int64_t E, int64_t* step_dev, double* phys,
                                   int32_t* t_elapsed, uint8_t* terminal, const float* dist,
                                   int64_t dist_stride, float action_scaling,
                                   uint64_t sample_seed, int32_t t_max, float* traj_obs,
                                   float* traj_act, float* traj_rew, uint8_t* traj_done,
                                   int32_t* ep_len, int32_t* active_after, double* reward_sum,
                                   void* stream) {
  PRL_REQUIRE(step_dev != nullptr, "prl_rollout_step_at: null step index");
  return rollout_step_launch(kind, E, 0, step_dev, phys, t_elapsed, terminal, dist, dist_stride,
                             action_scaling, sample_seed, t_max, traj_obs, traj_act, traj_rew,
                             traj_done, ep_len, active_after, reward_sum, stream);
}
