// prl_envs.h — the per-env device code shared by the rollout kernels: the restated gymnasium
// classic-control envs (CartPole-v1, Pendulum-v1 + TimeLimit), the synthetic Humanoid-shaped env
// and the in-kernel action sampling (Philox4x32-10).  Used by prl_envs.hip (reset / step / the
// fused per-vector-step rollout kernel) and prl_wide_rollout.hip (the persistent wide-net rollout).
#pragma once
#include "prl_common.h"

#include <math.h>

namespace prl {

// ---------------------------------------------------------------------------------------------
// gymnasium CartPole-v1 (classic_control/cartpole.py) + TimeLimit(max_episode_steps=500)
struct CartPole {
  static constexpr int D = 4, A = 1, P = 4, TMAX = 500;
  static constexpr double gravity = 9.8, masscart = 1.0, masspole = 0.1;
  static constexpr double total_mass = masspole + masscart;
  static constexpr double length = 0.5;
  static constexpr double polemass_length = masspole * length;
  static constexpr double force_mag = 10.0, tau = 0.02;
  static constexpr double theta_threshold = 12 * 2 * 3.141592653589793 / 360;
  static constexpr double x_threshold = 2.4;

  // reset(): state = np_random.uniform(low=-0.05, high=0.05, size=(4,))
  __device__ static void reset(double* s, pcg64& g) {
    for (int i = 0; i < 4; ++i) s[i] = pcg64_uniform(g, -0.05, 0.05);
  }
  // step(action): Euler integration; returns terminated.  reward is 1.0 on every step an env
  // takes (gymnasium returns 1.0 also on the step that terminates; terminated envs are never
  // stepped again by EnvVectorizer).
  __device__ static bool step(double* s, int action, double& reward) {
    double x = s[0], x_dot = s[1], theta = s[2], theta_dot = s[3];
    const double force = (action == 1) ? force_mag : -force_mag;
    const double costheta = prl_cos(theta);
    const double sintheta = prl_sin(theta);
    const double temp = (force + polemass_length * (theta_dot * theta_dot) * sintheta) / total_mass;
    const double thetaacc = (gravity * sintheta - costheta * temp) /
                            (length * (4.0 / 3.0 - masspole * (costheta * costheta) / total_mass));
    const double xacc = temp - polemass_length * thetaacc * costheta / total_mass;
    x = x + tau * x_dot;
    x_dot = x_dot + tau * xacc;
    theta = theta + tau * theta_dot;
    theta_dot = theta_dot + tau * thetaacc;
    s[0] = x; s[1] = x_dot; s[2] = theta; s[3] = theta_dot;
    reward = 1.0;
    return x < -x_threshold || x > x_threshold || theta < -theta_threshold ||
           theta > theta_threshold;
  }
  __device__ static void obs(const double* s, float* o) {
    for (int i = 0; i < 4; ++i) o[i] = (float)s[i];
  }
};

// gymnasium Pendulum-v1 (classic_control/pendulum.py, g=10.0) + TimeLimit(200)
struct Pendulum {
  static constexpr int D = 3, A = 1, P = 2, TMAX = 200;
  static constexpr double max_speed = 8, max_torque = 2.0, dt = 0.05, g = 10.0, m = 1.0, l = 1.0;
  static constexpr double pi = 3.141592653589793;

  // reset(): high = [pi, 1.0]; state = np_random.uniform(low=-high, high=high)
  __device__ static void reset(double* s, pcg64& gen) {
    s[0] = pcg64_uniform(gen, -pi, pi);
    s[1] = pcg64_uniform(gen, -1.0, 1.0);
  }
  // numpy float64 remainder: fmod, then fix the sign to the divisor's (npy_divmod).
  __device__ static double py_mod(double a, double b) {
    double mod = fmod(a, b);
    if (mod != 0.0) {
      if ((b < 0) != (mod < 0)) mod += b;
    } else {
      mod = copysign(0.0, b);
    }
    return mod;
  }
  __device__ static double angle_normalize(double x) { return py_mod(x + pi, 2 * pi) - pi; }
  // u arrives as float32 (PPO.get_action returns float32, PPO/PPO.py:90-96); under NumPy 2
  // (NEP 50) `3.0 * u`, `u**2` and `0.001 * u**2` stay float32, everything else is float64.
  __device__ static bool step(double* s, float u_in, double& reward) {
    const double th = s[0], thdot = s[1];
    const float u = fminf(fmaxf(u_in, -2.0f), 2.0f);  // np.clip(u, -2, 2)[0] (NaN kept below)
    const float uc = (u_in != u_in) ? u_in : u;
    const float u2 = uc * uc;
    const float ucost = 0.001f * u2;
    const double an = angle_normalize(th);
    const double costs = an * an + 0.1 * (thdot * thdot) + (double)ucost;
    const float u3 = 3.0f * uc;
    double newthdot = thdot + (15.0 * prl_sin(th) + (double)u3) * dt;
    newthdot = newthdot < -max_speed ? -max_speed : (newthdot > max_speed ? max_speed : newthdot);
    const double newth = th + newthdot * dt;
    s[0] = newth;
    s[1] = newthdot;
    reward = -costs;
    return false;
  }
  __device__ static void obs(const double* s, float* o) {
    o[0] = (float)prl_cos(s[0]);
    o[1] = (float)prl_sin(s[0]);
    o[2] = (float)s[1];
  }
};

// Synthetic Humanoid-v5-shaped env (no reference counterpart; BASELINE.json config 5):
// obs 348 f32, action 17 f32.  Per episode a 64-bit key is drawn from the env's PCG64; episode
// length L = 1 + #failures before the first success of Bernoulli(13/256) trials read from
// Philox(key) bytes (mean 19.7), capped by TimeLimit(1000); obs_t[j] is a unit-variance
// triangular variate from Philox(key ^ t, j); reward = 1 - 0.01 * sum_j a_j^2 (f32, in j order).
struct Synth {
  static constexpr int D = 348, A = 17, P = 2, TMAX = 1000;
  __device__ static uint32_t episode_len(uint64_t key) {
    for (uint32_t blk = 0; blk < 64; ++blk) {
      const u32x4 r = philox4x32_10(u32x4{blk, 0x5eedu, 0u, 0u}, (uint32_t)key, (uint32_t)(key >> 32));
      const uint32_t w[4] = {r.x, r.y, r.z, r.w};
      for (int k = 0; k < 16; ++k) {
        const uint32_t byte = (w[k >> 2] >> ((k & 3) * 8)) & 0xffu;
        if (byte < 13u) {
          const uint32_t L = blk * 16u + (uint32_t)k + 1u;
          return L > (uint32_t)TMAX ? (uint32_t)TMAX : L;
        }
      }
    }
    return TMAX;
  }
  __device__ static float obs_at(uint64_t key, uint32_t t, uint32_t j) {
    const u32x4 r = philox4x32_10(u32x4{j >> 1, t, 0x0b5u, 0u}, (uint32_t)key ^ t,
                                  (uint32_t)(key >> 32));
    const uint32_t a = (j & 1) ? r.z : r.x, b = (j & 1) ? r.w : r.y;
    return ((u01(a) + u01(b)) - 1.0f) * 2.4494898f;
  }
};

// ---------------------------------------------------------------------------------------------
// Action sampling (PPO.get_action, PPO/PPO.py:85-91): Categorical(probs).sample() and
// tanh(MultivariateNormal(mu, diag(std^2)).sample()) * action_scaling, with Philox4x32-10 keyed
// by (seed, env, t).  Categorical normalises probs (probs / probs.sum) — done by scaling u.
__device__ inline int sample_categorical(const float* p, int A, uint64_t seed, uint32_t e,
                                         uint32_t t) {
  const u32x4 r = philox4x32_10(u32x4{e, t, 0xca7u, 0u}, (uint32_t)seed, (uint32_t)(seed >> 32));
  float total = 0.f;
  for (int k = 0; k < A; ++k) total += p[k];
  const float target = u01(r.x) * total;
  float c = 0.f;
  for (int k = 0; k < A - 1; ++k) {
    c += p[k];
    if (target < c) return k;
  }
  return A - 1;
}

// standard normal for action dim j (Box-Muller, f32)
__device__ inline float sample_normal(uint64_t seed, uint32_t e, uint32_t t, uint32_t j) {
  const u32x4 r = philox4x32_10(u32x4{e, t, 0x6a055u, j >> 1}, (uint32_t)seed,
                                (uint32_t)(seed >> 32));
  const float rad = sqrtf(-2.0f * logf(u01_open0(r.x)));
  const float ang = 6.2831853071795864f * u01(r.y);
  return (j & 1) ? rad * sinf(ang) : rad * cosf(ang);
}

}  // namespace prl
