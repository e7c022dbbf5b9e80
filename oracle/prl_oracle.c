/*
 * prl_oracle.c — CPU ORACLE (test infrastructure, NOT product code).
 *
 * A plain-C restatement of the reference's hot path, used only by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg, as the checker for libprl_hip.so.
 * Nothing in the product imports, links or executes this file.
 *
 * What it restates (reference paths relative to the reference repository root):
 *   - PPO.compute_gae (PPO/PPO.py:107-120): the sequential reverse loop in float32, NumPy-2 /
 *     NEP-50 promotion (Python float scalars are weak -> float32), gamma*lambda in float64.
 *   - gymnasium==1.1.1 CartPole-v1 / Pendulum-v1 step (third-party, pinned at requirements.txt:4,
 *     called at AsyncTools/AsyncPPO.py:76): float64 numpy-scalar order of operations.
 *     Trig is fdlibm's (__kernel_sin/__kernel_cos, __ieee754_rem_pio2 medium case); numpy uses
 *     glibc, which differs from fdlibm by 1 ulp on a small fraction of arguments — measured in
 *     tests/test_oracle.py.
 *   - EnvVectorizer's per-env sequential stepping over the active envs (AsyncPPO.py:64-102) and
 *     the one-episode-per-env worker (AsyncPPO.py:117-146) for the CPU baseline.
 *   - Philox4x32-10 action sampling and the synthetic Humanoid-shaped env (no reference
 *     counterpart; semantics defined in DESIGN.md).
 * Compile: gcc -O2 -fPIC -shared -ffp-contract=off -fno-fast-math (see oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* ------------------------------------------------------------------ fdlibm sin / cos */
static int32_t hiw(double x) { uint64_t u; memcpy(&u, &x, 8); return (int32_t)(u >> 32); }

static double ksin(double x, double y, int iy) {
  static const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                      S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                      S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x, v = z * x, r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

static double kcos(double x, double y) {
  static const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                      C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                      C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x, w = z * z;
  double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  double hz = 0.5 * z, ww = 1.0 - hz;
  return ww + (((1.0 - ww) - hz) + (z * r - x * y));
}

static int rempio2(double x, double* y) {
  static const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                      pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                      pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                      pio2_3t = 8.47842766036889956997e-32;
  int32_t ix = hiw(x) & 0x7fffffff;
  double fn = rint(x * invpio2), r, w, t;
  int n = (int)fn, j, i;
  r = x - fn * pio2_1;
  w = fn * pio2_1t;
  y[0] = r - w;
  j = ix >> 20;
  i = j - ((hiw(y[0]) >> 20) & 0x7ff);
  if (i > 16) {
    t = r; w = fn * pio2_2; r = t - w; w = fn * pio2_2t - ((t - r) - w); y[0] = r - w;
    i = j - ((hiw(y[0]) >> 20) & 0x7ff);
    if (i > 49) { t = r; w = fn * pio2_3; r = t - w; w = fn * pio2_3t - ((t - r) - w); y[0] = r - w; }
  }
  y[1] = (r - y[0]) - w;
  return n;
}

double or_sin(double x) {
  int32_t ix = hiw(x) & 0x7fffffff;
  double y[2];
  if (ix <= 0x3fe921fb) return ix < 0x3e400000 ? x : ksin(x, 0.0, 0);
  if (ix >= 0x7ff00000) return x - x;
  if (ix >= 0x41200000) x = fmod(x, 6.283185307179586);
  switch (rempio2(x, y) & 3) {
    case 0: return ksin(y[0], y[1], 1);
    case 1: return kcos(y[0], y[1]);
    case 2: return -ksin(y[0], y[1], 1);
    default: return -kcos(y[0], y[1]);
  }
}

double or_cos(double x) {
  int32_t ix = hiw(x) & 0x7fffffff;
  double y[2];
  if (ix <= 0x3fe921fb) return ix < 0x3e400000 ? 1.0 : kcos(x, 0.0);
  if (ix >= 0x7ff00000) return x - x;
  if (ix >= 0x41200000) x = fmod(x, 6.283185307179586);
  switch (rempio2(x, y) & 3) {
    case 0: return kcos(y[0], y[1]);
    case 1: return -ksin(y[0], y[1], 1);
    case 2: return -kcos(y[0], y[1]);
    default: return ksin(y[0], y[1], 1);
  }
}

void or_sin_cos_array(const double* x, int64_t n, double* s, double* c) {
  for (int64_t i = 0; i < n; ++i) { s[i] = or_sin(x[i]); c[i] = or_cos(x[i]); }
}

/* ------------------------------------------------------------------ Philox4x32-10 */
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
static float ou01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
static float ou01o(uint32_t x) { return (float)((x >> 8) + 1u) * (1.0f / 16777216.0f); }

void or_philox(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  philox(c, k0, k1);
  memcpy(out, c, 16);
}

/* Categorical(probs).sample() by inverse CDF on the normalised probs, Philox(seed; e, t). */
int or_sample_categorical(const float* p, int A, uint64_t seed, uint32_t e, uint32_t t) {
  uint32_t c[4] = {e, t, 0xca7u, 0u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float total = 0.f, acc = 0.f, target;
  for (int k = 0; k < A; ++k) total += p[k];
  target = ou01(c[0]) * total;
  for (int k = 0; k < A - 1; ++k) { acc += p[k]; if (target < acc) return k; }
  return A - 1;
}

float or_sample_normal(uint64_t seed, uint32_t e, uint32_t t, uint32_t j) {
  uint32_t c[4] = {e, t, 0x6a055u, j >> 1};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float rad = sqrtf(-2.0f * logf(ou01o(c[0])));
  float ang = 6.2831853071795864f * ou01(c[1]);
  return (j & 1) ? rad * sinf(ang) : rad * cosf(ang);
}

void or_sample_categorical_batch(const float* probs, int64_t E, int A, uint64_t seed,
                                 const int32_t* t, int32_t* out) {
  for (int64_t e = 0; e < E; ++e) out[e] = or_sample_categorical(probs + e * A, A, seed, (uint32_t)e, (uint32_t)t[e]);
}

/* ------------------------------------------------------------------ CartPole-v1 */
int or_cartpole_step1(double* s, int action) {
  const double gravity = 9.8, masscart = 1.0, masspole = 0.1, total_mass = masspole + masscart;
  const double length = 0.5, polemass_length = masspole * length, force_mag = 10.0, tau = 0.02;
  const double theta_threshold_radians = 12 * 2 * 3.141592653589793 / 360, x_threshold = 2.4;
  double x = s[0], x_dot = s[1], theta = s[2], theta_dot = s[3];
  double force = action == 1 ? force_mag : -force_mag;
  double costheta = or_cos(theta), sintheta = or_sin(theta);
  double temp = (force + polemass_length * (theta_dot * theta_dot) * sintheta) / total_mass;
  double thetaacc = (gravity * sintheta - costheta * temp) /
                    (length * (4.0 / 3.0 - masspole * (costheta * costheta) / total_mass));
  double xacc = temp - polemass_length * thetaacc * costheta / total_mass;
  x = x + tau * x_dot;
  x_dot = x_dot + tau * xacc;
  theta = theta + tau * theta_dot;
  theta_dot = theta_dot + tau * thetaacc;
  s[0] = x; s[1] = x_dot; s[2] = theta; s[3] = theta_dot;
  return x < -x_threshold || x > x_threshold || theta < -theta_threshold_radians ||
         theta > theta_threshold_radians;
}

/* batched: E envs with states s[E][4], actions a[E]; terminated out u8[E] */
void or_cartpole_step(double* s, const int64_t* a, int64_t E, uint8_t* term) {
  for (int64_t e = 0; e < E; ++e) term[e] = (uint8_t)or_cartpole_step1(s + 4 * e, (int)a[e]);
}

/* ------------------------------------------------------------------ Pendulum-v1 */
static double py_mod(double a, double b) {
  double mod = fmod(a, b);
  if (mod != 0.0) { if ((b < 0) != (mod < 0)) mod += b; }
  else mod = copysign(0.0, b);
  return mod;
}

double or_pendulum_step1(double* s, float u_in) {
  const double pi = 3.141592653589793, dt = 0.05;
  double th = s[0], thdot = s[1];
  float u = u_in != u_in ? u_in : (u_in < -2.0f ? -2.0f : (u_in > 2.0f ? 2.0f : u_in));
  double an = py_mod(th + pi, 2 * pi) - pi;
  float ucost = 0.001f * (u * u);
  double costs = an * an + 0.1 * (thdot * thdot) + (double)ucost;
  float u3 = 3.0f * u;
  double newthdot = thdot + (15.0 * or_sin(th) + (double)u3) * dt;
  if (newthdot < -8) newthdot = -8; else if (newthdot > 8) newthdot = 8;
  s[0] = th + newthdot * dt;
  s[1] = newthdot;
  return -costs;
}

void or_pendulum_step(double* s, const float* u, int64_t E, double* reward) {
  for (int64_t e = 0; e < E; ++e) reward[e] = or_pendulum_step1(s + 2 * e, u[e]);
}

/* ------------------------------------------------------------------ synthetic Humanoid env */
uint32_t or_synth_episode_len(uint64_t key) {
  for (uint32_t blk = 0; blk < 64; ++blk) {
    uint32_t c[4] = {blk, 0x5eedu, 0u, 0u};
    philox(c, (uint32_t)key, (uint32_t)(key >> 32));
    for (int k = 0; k < 16; ++k) {
      uint32_t byte = (c[k >> 2] >> ((k & 3) * 8)) & 0xffu;
      if (byte < 13u) { uint32_t L = blk * 16u + (uint32_t)k + 1u; return L > 1000u ? 1000u : L; }
    }
  }
  return 1000u;
}

void or_synth_obs(uint64_t key, uint32_t t, float* o) {
  for (uint32_t j = 0; j < 348; ++j) {
    uint32_t c[4] = {j >> 1, t, 0x0b5u, 0u};
    philox(c, (uint32_t)key ^ t, (uint32_t)(key >> 32));
    uint32_t a = (j & 1) ? c[2] : c[0], b = (j & 1) ? c[3] : c[1];
    o[j] = ((ou01(a) + ou01(b)) - 1.0f) * 2.4494898f;
  }
}

/* ------------------------------------------------------------------ GAE (PPO.py:107-120) */
void or_gae(const float* r, const float* d, const float* V, float next_value, int64_t n,
            double gamma, double lam, float* ret) {
  const float gf = (float)gamma;         /* weak Python float meets float32 */
  const float glf = (float)(gamma * lam); /* Python float product, then meets float32 */
  float gae = 0.0f, nv = next_value;
  for (int64_t t = n - 1; t >= 0; --t) {
    float omd = 1.0f - d[t];
    float a = gf * nv;
    a = a * omd;
    float s = r[t] + a;
    float delta = s - V[t];
    float c = glf * omd;
    gae = delta + c * gae;
    ret[t] = gae + V[t];
    nv = V[t];
  }
}

/* ------------------------------------------------------------------ CPU baseline rollout */
/* The reference worker's algorithm on one core: every vector step, for each still-active env in
 * ascending order, sample an action from the given fixed 2-way probabilities, step the env and
 * append the transition to that env's episode; stop when every env is terminal; then write the
 * env-major concatenation.  (Policy evaluation is excluded: the baseline times env work +
 * buffering, i.e. AsyncPPO.py:123-146.)  Returns N. */
int64_t or_cartpole_rollout(int64_t E, const double* s0, uint64_t seed, float p1, int32_t tmax,
                            double* s_work, uint8_t* term, int32_t* len, float* traj_obs,
                            float* flat_obs, float* flat_act, float* flat_rew, float* flat_done,
                            int32_t* traj_act) {
  memcpy(s_work, s0, sizeof(double) * 4 * E);
  memset(term, 0, E);
  memset(len, 0, sizeof(int32_t) * E);
  const float probs[2] = {1.0f - p1, p1};
  int64_t active = E;
  for (int32_t t = 0; t < tmax && active > 0; ++t) {
    for (int64_t e = 0; e < E; ++e) {
      if (term[e]) continue;
      double* s = s_work + 4 * e;
      float* o = traj_obs + ((int64_t)t * E + e) * 4;
      for (int k = 0; k < 4; ++k) o[k] = (float)s[k];
      int a = or_sample_categorical(probs, 2, seed, (uint32_t)e, (uint32_t)t);
      traj_act[(int64_t)t * E + e] = a;
      int done = or_cartpole_step1(s, a) || (t + 1 >= 500) || (t + 1 >= tmax);
      len[e] = t + 1;
      if (done) { term[e] = 1; --active; }
    }
  }
  int64_t off = 0;
  for (int64_t e = 0; e < E; ++e) {
    for (int32_t t = 0; t < len[e]; ++t, ++off) {
      memcpy(flat_obs + 4 * off, traj_obs + ((int64_t)t * E + e) * 4, 16);
      flat_act[off] = (float)traj_act[(int64_t)t * E + e];
      flat_rew[off] = 1.0f;
      flat_done[off] = (t == len[e] - 1) ? 1.0f : 0.0f;
    }
  }
  return off;
}
