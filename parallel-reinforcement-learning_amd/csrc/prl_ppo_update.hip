// prl_ppo_update.hip — the whole PPO.learn update loop (PPO/PPO.py:216-255) as ONE persistent
// kernel: k_epochs x ceil(N / mb) sequential, unshuffled minibatch steps of
//     forward (ActorCritic.get_evaluate, PPO/ActorCritic.py:118-146)
//  -> clipped surrogate + 0.5 SmoothL1 - 0.01 H (PPO.py:225-245)
//  -> backward -> clip_grad_norm_(2.0) -> AdamW (torch defaults, lr from PPO.__init__, PPO.py:51-54)
// for the reference's actor-critic: trunk Linear(D,64,no bias) -> GroupNorm(8,64) -> SiLU, heads
// Linear(64,64,no bias) -> GroupNorm(8,64) -> SiLU -> Linear(64,out) (ActorCritic.py:19-60);
// discrete: actor (softmax -> Categorical) + critic; continuous: mu, log_std
// (softplus(clamp(.,-2,2)), diagonal Gaussian) + critic.
//
// Why one kernel: at the reference's mini_batch_size = 512 a step is ~25 MFLOP spread over ~50
// tiny kernels; the graph-replayed PyTorch step costs ~180 us, almost all launch gaps.
//
// Decomposition (G workgroups of 256 threads, one per CU, co-resident: cooperative launch):
//   phase A  workgroup g takes rows [g*R, (g+1)*R) of the step's minibatch in chunks of RC = 8
//            rows; forward + backward run out of LDS with the CURRENT parameters in LDS (every
//            workgroup holds a full, bit-identical copy), accumulating this workgroup's partial
//            gradient (and the loss partials) in LDS, then publishes it write-through (sc1
//            16-B stores) to part[g] and bumps counter A;
//   phase B  when all G partials are in, workgroup g sums its 1/G slice of the gradient over the
//            G partials in workgroup order (deterministic), publishes the slice + its sum of
//            squares (sc1) and bumps counter B;
//   phase C  when all slices are in, EVERY workgroup reads the whole reduced gradient and the G
//            squared-norm pieces (sc1 loads, same order everywhere), forms the clip coefficient
//            and applies AdamW to its own copy of the parameters (LDS) and moments (a private
//            global slab) — identical inputs, identical code, so every copy stays bit-identical
//            and no parameter broadcast (third hand-off) is needed.
// Hand-offs follow the MI355X guide's Guideline 16 (first row of the sc1 table): payload stored
// sc1 and drained by every storing wave, one lane adds to the counter behind a workgroup
// barrier, one lane polls it relaxed (bounded, s_sleep), every load of the payload is sc1.
// The counters are zeroed by a memset node ahead of the launch and are monotonic within it.
//
// LDS layout of a parameter tensor [rows][cols]: row stride 68 for the 64-wide matrices (16-B
// aligned rows, conflict-free 16-B reads across 16 lanes), odd stride for the trunk weight
// (conflict-free 4-B reads); padding entries stay exactly 0 through AdamW (0 grad, 0 moments).
#include "prl_common.h"

#include <float.h>

#include <algorithm>

namespace prl {

constexpr int UPD_THREADS = 256;
constexpr int UPD_RC = 8;         // rows per chunk
constexpr int UPD_H = 64;         // hidden width
constexpr int UPD_HS = 68;        // LDS row stride of [*][64] arrays
constexpr int UPD_MAXH = 3;       // heads
constexpr int UPD_MAXD = 64;      // max observation dim on the fused path
constexpr int UPD_MAXA = 8;       // max action dim on the fused path
constexpr unsigned UPD_SPIN_LIMIT = 1u << 22;  // ~0.1-0.3 s of s_sleep polls: never expected

struct UpdTensor {
  int flat, lds, rows, cols, stride;
};

struct UpdNet {
  int D, A, nh, discrete;
  int out[UPD_MAXH];            // outputs of each head (A | A | 1)
  int ocol[UPD_MAXH];           // first column of each head in the O / dO rows
  int nout;                     // sum of out
  UpdTensor w0, g0, b0;
  UpdTensor w1[UPD_MAXH], g1[UPD_MAXH], b1[UPD_MAXH], w2[UPD_MAXH], b2[UPD_MAXH];
  int Lp;                       // LDS floats of the parameter image (multiple of 4)
  int P;                        // flat parameter count
};

struct UpdArgs {
  UpdNet net;
  const float* S;
  const float* act;
  const float* old_logp;
  const float* adv;
  const float* ret;
  int64_t N;
  int mb, nb, total_steps, G, R;
  float clip, vf_coef, ent_coef, lr, beta1, beta2, eps, wd, max_norm;
  float* params;
  float* exp_avg;
  float* exp_avg_sq;
  float* adam_step;
  float* loss_out;
  float* part;      // [G][Qtot * 4]
  float* red;       // [Qtot * 4]
  float* sq;        // [G]
  unsigned* ctr;    // [0] arrivals A, [1] arrivals B, [2] abort, [3] status (zeroed per launch),
                    // [4] sticky timeout flag (never zeroed by a launch)
  unsigned long long* prof;  // [8] workgroup 0's time per phase (100 MHz ticks, summed over steps)
};

// ---- sc1 (write-through / L1-bypassing) accessors -------------------------------------------
typedef unsigned v4u __attribute__((ext_vector_type(4)));

// The resource is built from a WAVE-UNIFORM base (a kernel argument); the per-lane part of the
// address goes in the byte offset.  (A per-lane base forces a 64-iteration waterfall loop.)
__device__ inline __amdgpu_buffer_rsrc_t upd_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ inline float4 ld4_sc1(__amdgpu_buffer_rsrc_t rs, size_t float_off) {
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(float_off * 4), 0, 16);
  return float4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                __uint_as_float(v.w)};
}
__device__ inline void st4_sc1(__amdgpu_buffer_rsrc_t rs, size_t float_off, float4 x) {
  v4u v;
  v.x = __float_as_uint(x.x);
  v.y = __float_as_uint(x.y);
  v.z = __float_as_uint(x.z);
  v.w = __float_as_uint(x.w);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, (unsigned)(float_off * 4), 0, 16);
}
__device__ inline float ld_sc1f(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}
__device__ inline void st_sc1f(float* p, float x) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(x), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned ld_sc1u(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one lane: wait until *c >= target (or abort); false on timeout / abort
__device__ inline bool upd_wait(unsigned* ctr, int which, unsigned target) {
  for (unsigned spins = 0;; ++spins) {
    if (ld_sc1u(ctr + which) >= target) return true;
    if (ld_sc1u(ctr + 2) != 0u) return false;
    if (spins > UPD_SPIN_LIMIT) {
      __hip_atomic_store(ctr + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_or(ctr + 4, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sticky
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ inline float upd_sigmoid(float y) { return 1.0f / (1.0f + expf(-y)); }

// flat index of LDS-image entry k (-1 = padding)
__device__ inline bool upd_in(const UpdTensor& t, int k, int& f) {
  if (k < t.lds || k >= t.lds + t.rows * t.stride) return false;
  const int r = (k - t.lds) / t.stride, c = (k - t.lds) % t.stride;
  f = c < t.cols ? t.flat + r * t.cols + c : -1;
  return true;
}
__device__ inline int upd_flat_of(const UpdNet& n, int k) {
  int f = -1;
  if (upd_in(n.w0, k, f) || upd_in(n.g0, k, f) || upd_in(n.b0, k, f)) return f;
  for (int h = 0; h < n.nh; ++h)
    if (upd_in(n.w1[h], k, f) || upd_in(n.g1[h], k, f) || upd_in(n.b1[h], k, f) ||
        upd_in(n.w2[h], k, f) || upd_in(n.b2[h], k, f))
      return f;
  return -1;
}

// ---- per-chunk activation buffers (floats, offsets into the dynamic LDS) ---------------------
constexpr int UPD_HEAD_FLOATS = 4 * UPD_RC * UPD_HS + UPD_RC * 8;
struct UpdAct {
  float* X;       // [RC][DX]
  float* Ar;      // [RC][AX] actions
  float* oldlp;   // [RC]
  float* adv;     // [RC]
  float* ret;     // [RC]
  float* lossp;   // [RC][4]
  float* T0;      // [RC][HS]  dH0
  float* XH0;     // [RC][HS]
  float* F;       // [RC][HS]
  float* DU0;     // [RC][HS]
  float* rstd0;   // [RC][8]
  float* heads;   // per head h at heads + h * UPD_HEAD_FLOATS:
                  //   ZB [RC][HS] (dZ), XH, Gh, DU [RC][HS], rstd [RC][8]
  __device__ float* ZB(int h) const { return heads + h * UPD_HEAD_FLOATS; }
  __device__ float* XH(int h) const { return heads + h * UPD_HEAD_FLOATS + UPD_RC * UPD_HS; }
  __device__ float* Gh(int h) const { return heads + h * UPD_HEAD_FLOATS + 2 * UPD_RC * UPD_HS; }
  __device__ float* DU(int h) const { return heads + h * UPD_HEAD_FLOATS + 3 * UPD_RC * UPD_HS; }
  __device__ float* rstd(int h) const { return heads + h * UPD_HEAD_FLOATS + 4 * UPD_RC * UPD_HS; }
  float* dFh;     // [MAXH][RC][HS] per-head parts of dF
  __device__ float* dF(int h) const { return dFh + h * UPD_RC * UPD_HS; }
  float* O;       // [RC][OX]
  float* dO;      // [RC][OX]
  int DX, AX, OX;
};

__host__ __device__ inline int upd_act_floats(int D, int A, int nout, int& DX, int& AX, int& OX) {
  DX = (D + 3) & ~3;
  AX = (A + 3) & ~3;
  OX = (nout + 3) & ~3;
  return UPD_RC * (DX + AX + 4 + 4 + 4 * UPD_HS + 8 + UPD_MAXH * (5 * UPD_HS + 8) + 2 * OX) + 16;
}

__device__ inline UpdAct upd_carve(float* base, const UpdNet& n) {
  UpdAct a;
  upd_act_floats(n.D, n.A, n.nout, a.DX, a.AX, a.OX);
  float* p = base;
  auto take = [&](int nf) { float* q = p; p += (nf + 3) & ~3; return q; };
  a.X = take(UPD_RC * a.DX);
  a.Ar = take(UPD_RC * a.AX);
  a.oldlp = take(UPD_RC);
  a.adv = take(UPD_RC);
  a.ret = take(UPD_RC);
  a.lossp = take(UPD_RC * 4);
  a.T0 = take(UPD_RC * UPD_HS);
  a.XH0 = take(UPD_RC * UPD_HS);
  a.F = take(UPD_RC * UPD_HS);
  a.DU0 = take(UPD_RC * UPD_HS);
  a.rstd0 = take(UPD_RC * 8);
  a.heads = take(UPD_MAXH * UPD_HEAD_FLOATS);
  a.dFh = take(UPD_MAXH * UPD_RC * UPD_HS);
  a.O = take(UPD_RC * a.OX);
  a.dO = take(UPD_RC * a.OX);
  return a;
}

// GroupNorm(8 groups of 8) + SiLU forward of one (row, group) held in registers: same
// arithmetic as gn_silu_fwd.  Writes xhat and the block output (16-B aligned LDS rows).
__device__ inline void upd_gn_fwd(const float (&v)[8], const float* gw, const float* gb,
                                  float* xh_out, float* y_out, float* rstd_out) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += v[k];
  const float mean = s * (1.0f / 8);
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) q += (v[k] - mean) * (v[k] - mean);
  const float rstd = 1.0f / sqrtf(q * (1.0f / 8) + 1e-5f);
  float xh[8], y[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    xh[k] = (v[k] - mean) * rstd;
    const float u = xh[k] * gw[k] + gb[k];
    y[k] = u / (1.0f + expf(-u));
  }
  *reinterpret_cast<float4*>(xh_out) = float4{xh[0], xh[1], xh[2], xh[3]};
  *reinterpret_cast<float4*>(xh_out + 4) = float4{xh[4], xh[5], xh[6], xh[7]};
  *reinterpret_cast<float4*>(y_out) = float4{y[0], y[1], y[2], y[3]};
  *reinterpret_cast<float4*>(y_out + 4) = float4{y[4], y[5], y[6], y[7]};
  *rstd_out = rstd;
}

// backward of the above: go = d(block output) in registers; writes dX and du = d(pre-SiLU)
__device__ inline void upd_gn_bwd(const float (&go)[8], const float* xh_in, const float* gw,
                                  const float* gb, float rstd, float* dx_out, float* du_out) {
  float xh[8];
  {
    const float4 c = *reinterpret_cast<const float4*>(xh_in);
    const float4 d = *reinterpret_cast<const float4*>(xh_in + 4);
    xh[0] = c.x; xh[1] = c.y; xh[2] = c.z; xh[3] = c.w; xh[4] = d.x; xh[5] = d.y; xh[6] = d.z; xh[7] = d.w;
  }
  float dy[8], dxh[8];
  float m1 = 0.f, m2 = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float u = xh[k] * gw[k] + gb[k];
    const float s = upd_sigmoid(u);
    dy[k] = go[k] * (s * (1.0f + u * (1.0f - s)));
    dxh[k] = dy[k] * gw[k];
    m1 += dxh[k];
    m2 += dxh[k] * xh[k];
  }
  m1 *= (1.0f / 8);
  m2 *= (1.0f / 8);
  float dx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) dx[k] = rstd * (dxh[k] - m1 - xh[k] * m2);
  *reinterpret_cast<float4*>(dx_out) = float4{dx[0], dx[1], dx[2], dx[3]};
  *reinterpret_cast<float4*>(dx_out + 4) = float4{dx[4], dx[5], dx[6], dx[7]};
  *reinterpret_cast<float4*>(du_out) = float4{dy[0], dy[1], dy[2], dy[3]};
  *reinterpret_cast<float4*>(du_out + 4) = float4{dy[4], dy[5], dy[6], dy[7]};
}

// log_prob and entropy of one row's action under the head outputs O (ActorCritic.get_evaluate,
// ActorCritic.py:118-146): discrete softmax -> Categorical(probs) (torch's normalise + clamped
// log); continuous diagonal Gaussian with std = softplus(clamp(log_std, -2, 2)).  Shared by the
// update and the evaluation kernel so old and new log-probs come from identical arithmetic.
struct UpdDist {
  float p[UPD_MAXA], q[UPD_MAXA];
  float S2, qa, logp, H;
  int ai;
};
// KD: 1 discrete / 0 continuous / -1 runtime;  KA: action dim (0 = runtime).  Specialised
// kernels keep the per-row code (executed by 8 lanes, but fetched every step) small.
template <int KD, int KA>
__device__ inline void upd_row_dist(const UpdNet& n, const float* O, const float* act, UpdDist& d) {
  const int A = KA > 0 ? KA : n.A;
  const bool discrete = KD >= 0 ? (KD != 0) : (n.discrete != 0);
  d.logp = 0.f;
  d.H = 0.f;
  d.S2 = 0.f;
  d.qa = 1.f;
  d.ai = 0;
  if (discrete) {
    float mx = O[0];
#pragma unroll
    for (int k = 1; k < UPD_MAXA; ++k)
      if (k < A) mx = fmaxf(mx, O[k]);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      d.p[k] = k < A ? expf(O[k] - mx) : 0.f;
      s += d.p[k];
    }
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      d.p[k] = k < A ? d.p[k] / s : 0.f;
      d.S2 += d.p[k];
    }
    d.ai = (int)act[0];
    const bool bad = d.ai < 0 || d.ai >= A;   // torch's gather would raise: poison instead
    float la = 0.f;
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      d.q[k] = d.p[k] / d.S2;
      if (k < A) {
        const float c = d.q[k] < FLT_EPSILON ? FLT_EPSILON
                                             : (d.q[k] > 1.0f - FLT_EPSILON ? 1.0f - FLT_EPSILON : d.q[k]);
        const float l = logf(c);
        d.H += l * d.q[k];
        if (k == d.ai) { la = l; d.qa = d.q[k]; }
      }
    }
    d.H = -d.H;
    d.logp = bad ? __builtin_nanf("") : la;
  } else {
    const float half_log_2pi = 0.91893853320467274f;  // log(sqrt(2 pi))
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      if (k < A) {
        const float mu = O[k];
        const float lsr = O[A + k];
        const float lsc = lsr < -2.0f ? -2.0f : (lsr > 2.0f ? 2.0f : lsr);
        const float sd = log1pf(expf(lsc));               // softplus, beta 1 (lsc <= 2 < 20)
        const float dd = act[k] - mu;
        const float lsd = logf(sd);
        d.logp += -(dd * dd) / (2.0f * (sd * sd)) - lsd - half_log_2pi;
        d.H += 0.5f + half_log_2pi + lsd;
      }
    }
  }
}

// Per-row loss (surrogate, prl_loss.hip semantics) and the gradient w.r.t. the head outputs.
// Loops run to the compile-time UPD_MAXA with `k < A` guards so everything stays in registers.
template <int KD, int KA>
__device__ inline void upd_row_loss(const UpdNet& n, const UpdAct& a, int r, float invB, float clip,
                                    float vf_coef) {
  const float* O = a.O + r * a.OX;
  float* dO = a.dO + r * a.OX;
  const int A = KA > 0 ? KA : n.A;
  const bool discrete = KD >= 0 ? (KD != 0) : (n.discrete != 0);
  const int vcol = discrete ? A : 2 * A;      // critic output column
  UpdDist dist;
  upd_row_dist<KD, KA>(n, O, a.Ar + r * a.AX, dist);
  const float logp = dist.logp, H = dist.H, S2 = dist.S2, qa = dist.qa;
  const int ai = dist.ai;
  const float* p = dist.p;
  const float V = O[vcol];
  // surrogate
  const float diff = logp - a.oldlp[r];
  const float cl = diff < -20.0f ? -20.0f : (diff > 20.0f ? 20.0f : diff);
  const float ratio = expf(cl);
  const float adv = a.adv[r];
  const float s1 = ratio * adv;
  const float lo = 1.0f - clip, hi = 1.0f + clip;
  const float rcl = ratio < lo ? lo : (ratio > hi ? hi : ratio);
  const float s2 = rcl * adv;
  const float m = (s1 != s1 || s2 != s2) ? __builtin_nanf("") : fminf(s1, s2);
  float w1, w2;
  if (s1 < s2) { w1 = 1.0f; w2 = 0.0f; }
  else if (s2 < s1) { w1 = 0.0f; w2 = 1.0f; }
  else { w1 = 0.5f; w2 = 0.5f; }
  const float in_clip = (ratio >= lo && ratio <= hi) ? 1.0f : 0.0f;
  const float in_20 = (diff >= -20.0f && diff <= 20.0f) ? 1.0f : 0.0f;
  const float dlogp = -invB * (w1 * adv + w2 * adv * in_clip) * ratio * in_20;
  const float x = V - a.ret[r];
  const float ax = fabsf(x);
  const float sl = ax < 1.0f ? 0.5f * ax * ax : ax - 0.5f;
  const float gx = ax < 1.0f ? x : (x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f));
  dO[vcol] = vf_coef * invB * gx;
  a.lossp[r * 4 + 0] = -m;
  a.lossp[r * 4 + 1] = sl;
  a.lossp[r * 4 + 2] = H;
  // d logp / d head outputs
  if (discrete) {
    const float mk = (qa >= FLT_EPSILON && qa <= 1.0f - FLT_EPSILON) ? 1.0f : 0.0f;
    const float gq = (logp != logp) ? logp : dlogp * mk;
    float dp[UPD_MAXA];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      dp[k] = k < A ? gq * (((k == ai) ? 1.0f / qa : 0.0f) - 1.0f) / S2 : 0.f;
      dot += p[k] * dp[k];
    }
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k)
      if (k < A) dO[k] = p[k] * (dp[k] - dot);
  } else {
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      if (k < A) {
        const float mu = O[k];
        const float lsr = O[A + k];
        const float lsc = lsr < -2.0f ? -2.0f : (lsr > 2.0f ? 2.0f : lsr);
        const float sd = log1pf(expf(lsc));
        const float d = a.Ar[r * a.AX + k] - mu;
        const float var = sd * sd;
        dO[k] = dlogp * (d / var);
        const float dsd = dlogp * ((d * d) / (var * sd) - 1.0f / sd);
        const float pass = (lsr >= -2.0f && lsr <= 2.0f) ? 1.0f : 0.0f;
        dO[A + k] = dsd * upd_sigmoid(lsc) * pass;
      }
    }
  }
}

// Cross-lane moves within 8-lane groups by DPP (no LDS round trip, unlike __shfl*, which lowers
// to ds_bpermute): quad_perm [1,0,3,2] = xor 1, [2,3,0,1] = xor 2, row_half_mirror (lane i <->
// 7 - i) carries the other quad's sum.  Every lane of a group ends with the same bits (IEEE add
// is commutative).
template <int CTRL>
__device__ inline float upd_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ inline float upd_xor1(float v) { return upd_dpp<0xB1>(v); }
__device__ inline float upd_xor2(float v) { return upd_dpp<0x4E>(v); }
// sum over the 8 consecutive lanes of a GroupNorm group (lanes = channels)
__device__ inline float upd_gsum8(float v) {
  v += upd_xor1(v);
  v += upd_xor2(v);
  v += upd_dpp<0x141>(v);
  return v;
}

// GroupNorm(8, 64) + SiLU forward of one element, lanes = channels o (group = 8 lanes)
__device__ inline void upd_gn_fwd_lane(float v, float gw, float gb, float* xh_out, float* y_out,
                                       float* rstd_out, bool write_rstd) {
  const float mean = upd_gsum8(v) * (1.0f / 8);
  const float dv = v - mean;
  const float rstd = 1.0f / sqrtf(upd_gsum8(dv * dv) * (1.0f / 8) + 1e-5f);
  const float xh = dv * rstd;
  const float u = xh * gw + gb;
  *xh_out = xh;
  *y_out = u / (1.0f + expf(-u));
  if (write_rstd) *rstd_out = rstd;
}

// backward of the above: go = d(block output); writes dX, returns du (= d pre-SiLU)
__device__ inline float upd_gn_bwd_lane(float go, float xh, float gw, float gb, float rstd,
                                        float* dx_out) {
  const float u = xh * gw + gb;
  const float sg = upd_sigmoid(u);
  const float dy = go * (sg * (1.0f + u * (1.0f - sg)));
  const float dxh = dy * gw;
  const float m1 = upd_gsum8(dxh) * (1.0f / 8);
  const float m2 = upd_gsum8(dxh * xh) * (1.0f / 8);
  *dx_out = rstd * (dxh - m1 - xh * m2);
  return dy;
}

__device__ inline int upd_head_of(const UpdNet& n, int j) {
  int h = 0;
  while (h + 1 < n.nh && j >= n.ocol[h + 1]) ++h;
  return h;
}

// Forward of rc <= RC rows (ActorCritic.get_evaluate's network part): S0 inputs, S1 trunk,
// S2 heads, then the head outputs O gathered to each row's leader lane (t == 32 r) — the only
// reader of O[r] in the caller's per-row epilogue, so no barrier follows.
__device__ inline void upd_forward(const UpdNet& n, const float* W, const UpdAct& a,
                                   const float* Sg, const float* actg, int64_t row0, int rc,
                                   unsigned long long* tm, bool timer, unsigned long long& tl) {
  const int t = threadIdx.x;
  const int D = n.D, A = n.A, nh = n.nh;
#define UPD_CMARK(i)                                                   \
  if (timer) {                                                         \
    const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();  \
    tm[i] += now_ - tl;                                                \
    tl = now_;                                                         \
  }
  // S0. inputs
  for (int i = t; i < UPD_RC * a.DX; i += UPD_THREADS) {
    const int r = i / a.DX, d = i % a.DX;
    a.X[i] = (r < rc && d < D) ? Sg[(row0 + r) * D + d] : 0.0f;
  }
  const int Aw = n.discrete ? 1 : A;
  for (int i = t; i < UPD_RC * a.AX; i += UPD_THREADS) {
    const int r = i / a.AX, k = i % a.AX;
    a.Ar[i] = (r < rc && k < Aw) ? actg[(row0 + r) * Aw + k] : 0.0f;
  }
  __syncthreads();
  UPD_CMARK(0)
  // Lanes = the 64 channels o of a row; wave w takes rows w and w + 4 (wave-uniform).
  const int o = t & 63, wv = t >> 6;
  // S1. trunk: H0 = X W0^T -> GroupNorm -> SiLU
  for (int r = wv; r < rc; r += 4) {
    const float* x = a.X + r * a.DX;
    const float* w = W + n.w0.lds + o * n.w0.stride;
    float acc = 0.f;
    for (int d = 0; d < D; ++d) acc += x[d] * w[d];
    upd_gn_fwd_lane(acc, W[n.g0.lds + o], W[n.b0.lds + o], a.XH0 + r * UPD_HS + o,
                    a.F + r * UPD_HS + o, a.rstd0 + r * 8 + (o >> 3), (o & 7) == 0);
  }
  __syncthreads();
  UPD_CMARK(1)
  // S2. heads: Z_h = F W1_h^T -> GroupNorm -> SiLU (rows w and w + 4 share each W1 read)
  for (int h = 0; h < nh; ++h) {
    const float* wrow = W + n.w1[h].lds + o * UPD_HS;
    const int r0 = wv, r1 = wv + 4;
    const bool two = r1 < rc;
    if (r0 >= rc) break;
    const float* f0 = a.F + r0 * UPD_HS;
    const float* f1 = a.F + (two ? r1 : r0) * UPD_HS;
    float z0 = 0.f, z1 = 0.f;
#pragma unroll 4
    for (int i = 0; i < UPD_H; i += 4) {
      const float4 w4 = *reinterpret_cast<const float4*>(wrow + i);
      const float4 a4 = *reinterpret_cast<const float4*>(f0 + i);
      const float4 b4 = *reinterpret_cast<const float4*>(f1 + i);
      z0 += a4.x * w4.x; z0 += a4.y * w4.y; z0 += a4.z * w4.z; z0 += a4.w * w4.w;
      z1 += b4.x * w4.x; z1 += b4.y * w4.y; z1 += b4.z * w4.z; z1 += b4.w * w4.w;
    }
    const float gw = W[n.g1[h].lds + o], gb = W[n.b1[h].lds + o];
    upd_gn_fwd_lane(z0, gw, gb, a.XH(h) + r0 * UPD_HS + o, a.Gh(h) + r0 * UPD_HS + o,
                    a.rstd(h) + r0 * 8 + (o >> 3), (o & 7) == 0);
    if (two)
      upd_gn_fwd_lane(z1, gw, gb, a.XH(h) + r1 * UPD_HS + o, a.Gh(h) + r1 * UPD_HS + o,
                      a.rstd(h) + r1 * 8 + (o >> 3), (o & 7) == 0);
  }
  __syncthreads();
  UPD_CMARK(2)
  // S3. head outputs + loss: one half-wave per row; lane l = (output j % 8, quarter of the 64
  //     inputs); quarter sums combined by shuffles, gathered by the row's leader lane, which
  //     writes O, evaluates the loss and writes d(loss)/d(outputs)
  {
    const int r = t >> 5, l = t & 31, jl = l >> 2, part = l & 3;
    for (int j0 = 0; j0 < n.nout; j0 += 8) {
      const int j = j0 + jl;
      float acc = 0.f;
      if (r < rc && j < n.nout) {
        const int h = upd_head_of(n, j), k = j - n.ocol[h];
        const float* wv = W + n.w2[h].lds + k * UPD_HS + part * 16;
        const float* gv = a.Gh(h) + r * UPD_HS + part * 16;
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
          const float4 w4 = *reinterpret_cast<const float4*>(wv + i);
          const float4 g4 = *reinterpret_cast<const float4*>(gv + i);
          acc += g4.x * w4.x;
          acc += g4.y * w4.y;
          acc += g4.z * w4.z;
          acc += g4.w * w4.w;
        }
      }
      acc += upd_xor1(acc);
      acc += upd_xor2(acc);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {    // gather to the row leaders: two scalar reads per j
        const float vlo = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc), 4 * jj));
        const float vhi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc), 32 + 4 * jj));
        const float v = (t & 32) ? vhi : vlo;
        const int jo = j0 + jj;
        if (l == 0 && r < rc && jo < n.nout) {
          const int h = upd_head_of(n, jo);
          a.O[r * a.OX + jo] = v + W[n.b2[h].lds + (jo - n.ocol[h])];
        }
      }
    }
  }
#undef UPD_CMARK
}

// One chunk of rc <= RC rows: forward, loss, backward; gradients accumulated into Ga (LDS
// image).  Eight barrier-separated stages; each Linear is fused with the GroupNorm that follows
// it (one thread per (row, group) owns 8 channels end to end).
template <int KD, int KA>
__device__ void upd_chunk(const UpdArgs& args, const float* W, float* Ga, const UpdAct& a,
                          int64_t row0, int rc, float invB, unsigned long long* tm) {
  const UpdNet& n = args.net;
  const int t = threadIdx.x;
  const int D = n.D, A = n.A, nh = n.nh;
  const bool timer = blockIdx.x == 0 && t == 0;
  unsigned long long tl = timer ? __builtin_amdgcn_s_memrealtime() : 0ull;
#define UPD_CMARK(i)                                                   \
  if (timer) {                                                         \
    const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();  \
    tm[i] += now_ - tl;                                                \
    tl = now_;                                                         \
  }
  if (t < UPD_RC) {
    const bool ok = t < rc;
    a.oldlp[t] = ok ? args.old_logp[row0 + t] : 0.0f;
    a.adv[t] = ok ? args.adv[row0 + t] : 0.0f;
    a.ret[t] = ok ? args.ret[row0 + t] : 0.0f;
  }
  upd_forward(n, W, a, args.S, args.act, row0, rc, tm, timer, tl);
  const int o = t & 63, wv = t >> 6;
  {
    const int r = t >> 5, l = t & 31;
    if (l == 0 && r < rc) upd_row_loss<KD, KA>(n, a, r, invB, args.clip, args.vf_coef);
  }
  __syncthreads();
  UPD_CMARK(3)
  // S4. dG_h = dO_h W2_h -> head GroupNorm + SiLU backward (lanes = channels)
  for (int h = 0; h < nh; ++h) {
    const float gw = W[n.g1[h].lds + o], gb = W[n.b1[h].lds + o];
    for (int r = wv; r < rc; r += 4) {
      const float* dO = a.dO + r * a.OX + n.ocol[h];
      float dg = 0.f;
      for (int k = 0; k < n.out[h]; ++k) dg += dO[k] * W[n.w2[h].lds + k * UPD_HS + o];
      a.DU(h)[r * UPD_HS + o] =
          upd_gn_bwd_lane(dg, a.XH(h)[r * UPD_HS + o], gw, gb, a.rstd(h)[r * 8 + (o >> 3)],
                          a.ZB(h) + r * UPD_HS + o);
    }
  }
  __syncthreads();
  UPD_CMARK(4)
  // S5. weight gradients of the heads + per-head parts of dF
  {
    // dW1_h += dZ_h^T F   (thread: 4 contiguous input columns x 4 output rows, per head)
    const int i4 = (t & 15) * 4, ob = t >> 4;
    for (int h = 0; h < nh; ++h) {
      float acc[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[k][c] = 0.f;
#pragma unroll 4
      for (int r = 0; r < UPD_RC; ++r) {
        if (r >= rc) break;
        const float4 f = *reinterpret_cast<const float4*>(a.F + r * UPD_HS + i4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float dz = a.ZB(h)[r * UPD_HS + ob + 16 * k];
          acc[k][0] += dz * f.x;
          acc[k][1] += dz * f.y;
          acc[k][2] += dz * f.z;
          acc[k][3] += dz * f.w;
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float4* gp = reinterpret_cast<float4*>(Ga + n.w1[h].lds + (ob + 16 * k) * UPD_HS + i4);
        float4 gv = *gp;
        gv.x += acc[k][0];
        gv.y += acc[k][1];
        gv.z += acc[k][2];
        gv.w += acc[k][3];
        *gp = gv;
      }
    }
  }
  if (t < nh * UPD_H) {   // head GroupNorm weight / bias
    const int h = t >> 6, c = t & 63;
    float sw = 0.f, sb = 0.f;
#pragma unroll
    for (int r = 0; r < UPD_RC; ++r) {
      if (r >= rc) break;
      const float du = a.DU(h)[r * UPD_HS + c];
      sw += du * a.XH(h)[r * UPD_HS + c];
      sb += du;
    }
    Ga[n.g1[h].lds + c] += sw;
    Ga[n.b1[h].lds + c] += sb;
  }
  for (int i = t; i < n.nout * UPD_H; i += UPD_THREADS) {   // dW2 += dO^T G
    const int j = i >> 6, c = i & 63;
    const int h = upd_head_of(n, j), k = j - n.ocol[h];
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < UPD_RC; ++r)
      if (r < rc) acc += a.dO[r * a.OX + j] * a.Gh(h)[r * UPD_HS + c];
    Ga[n.w2[h].lds + k * UPD_HS + c] += acc;
  }
  if (t < n.nout) {   // db2
    const int h = upd_head_of(n, t);
    float acc = 0.f;
    for (int r = 0; r < rc; ++r) acc += a.dO[r * a.OX + t];
    Ga[n.b2[h].lds + (t - n.ocol[h])] += acc;
  }
  if (t >= 64 && t < 64 + 3) {   // loss partials
    const int which = t - 64;
    float acc = 0.f;
    for (int r = 0; r < rc; ++r) acc += a.lossp[r * 4 + which];
    Ga[n.Lp + which] += acc;
  }
  for (int it = t; it < nh * rc * 16; it += UPD_THREADS) {   // dF_h = dZ_h W1_h
    const int h = it / (rc * 16), rem = it % (rc * 16), r = rem >> 4, c4 = (rem & 15) * 4;
    const float* dz = a.ZB(h) + r * UPD_HS;
    const float* w = W + n.w1[h].lds + c4;
    float4 acc = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int o = 0; o < UPD_H; o += 4) {
      const float4 z4 = *reinterpret_cast<const float4*>(dz + o);
      const float zz[4] = {z4.x, z4.y, z4.z, z4.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 w4 = *reinterpret_cast<const float4*>(w + (o + u) * UPD_HS);
        acc.x += zz[u] * w4.x;
        acc.y += zz[u] * w4.y;
        acc.z += zz[u] * w4.z;
        acc.w += zz[u] * w4.w;
      }
    }
    *reinterpret_cast<float4*>(a.dF(h) + r * UPD_HS + c4) = acc;
  }
  __syncthreads();
  UPD_CMARK(5)
  // S6. trunk GroupNorm + SiLU backward (lanes = channels): dF = sum_h dF_h
  for (int r = wv; r < rc; r += 4) {
    float df = 0.f;
    for (int h = 0; h < nh; ++h) df += a.dF(h)[r * UPD_HS + o];
    a.DU0[r * UPD_HS + o] = upd_gn_bwd_lane(df, a.XH0[r * UPD_HS + o], W[n.g0.lds + o],
                                            W[n.b0.lds + o], a.rstd0[r * 8 + (o >> 3)],
                                            a.T0 + r * UPD_HS + o);
  }
  __syncthreads();
  UPD_CMARK(6)
  // S7. dW0 += dH0^T X;  trunk GroupNorm weight / bias
  for (int i = t; i < UPD_H * D; i += UPD_THREADS) {
    const int o = i / D, d = i % D;
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < UPD_RC; ++r)
      if (r < rc) acc += a.T0[r * UPD_HS + o] * a.X[r * a.DX + d];
    Ga[n.w0.lds + o * n.w0.stride + d] += acc;
  }
  if (t < UPD_H) {
    float sw = 0.f, sb = 0.f;
#pragma unroll
    for (int r = 0; r < UPD_RC; ++r) {
      if (r >= rc) break;
      const float du = a.DU0[r * UPD_HS + t];
      sw += du * a.XH0[r * UPD_HS + t];
      sb += du;
    }
    Ga[n.g0.lds + t] += sw;
    Ga[n.b0.lds + t] += sb;
  }
  __syncthreads();
  UPD_CMARK(7)
#undef UPD_CMARK
}

__device__ inline float f4get(const float4& v, int e) {
  return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}
__device__ inline void f4set(float4& v, int e, float x) {
  if (e == 0) v.x = x; else if (e == 1) v.y = x; else if (e == 2) v.z = x; else v.w = x;
}

// NQ = parameter quads per thread (ceil(Lp / 4 / 256)): AdamW's moments live in registers.
template <int NQ, int KD, int KA>
__global__ __launch_bounds__(UPD_THREADS, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void
ppo_update_kernel(UpdArgs args) {
  extern __shared__ __align__(16) float upd_lds[];
  const UpdNet& n = args.net;
  const int t = threadIdx.x, g = blockIdx.x, G = args.G;
  const int Lp = n.Lp;
  const int Qp = Lp / 4;            // parameter quads
  const int Qtot = Qp + 1;          // + one quad of loss partials
  float* hdr = upd_lds;             // [64] broadcast words + chunk stage timers
  float* W = upd_lds + 64;          // [Lp]
  float* Ga = W + Lp;               // [Lp + 4]
  float* scratch = Ga + Lp + 4;     // activations / reduction scratch
  const UpdAct a = upd_carve(scratch, n);
  float* s_bcast = hdr;             // [0] clip coefficient, [1] loss
  float* s_ssq = hdr + 4;           // [4] per-wave sums of squares
  int* s_abort = reinterpret_cast<int*>(hdr + 8);

  // ---- load parameters (LDS image) and this thread's moments (quad q = t + 256 i, registers);
  //      the moments are scattered into the LDS image layout through Ga (free until phase A) ---
  float4 mreg[NQ], vreg[NQ];
  for (int k = t; k < Lp; k += UPD_THREADS) {
    const int f = upd_flat_of(n, k);
    W[k] = f >= 0 ? args.params[f] : 0.0f;
    Ga[k] = f >= 0 ? args.exp_avg[f] : 0.0f;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = t + i * UPD_THREADS;
    mreg[i] = q < Qp ? *reinterpret_cast<const float4*>(Ga + 4 * q) : float4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  for (int k = t; k < Lp; k += UPD_THREADS) {
    const int f = upd_flat_of(n, k);
    Ga[k] = f >= 0 ? args.exp_avg_sq[f] : 0.0f;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = t + i * UPD_THREADS;
    vreg[i] = q < Qp ? *reinterpret_cast<const float4*>(Ga + 4 * q) : float4{0.f, 0.f, 0.f, 0.f};
  }
  const float step0 = args.adam_step[0];
  if (t < 24) reinterpret_cast<unsigned long long*>(hdr + 16)[t] = 0ull;
  __syncthreads();

  const int R = args.R;
  float loss_last = 0.f;
  unsigned long long pt[7] = {0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = __builtin_amdgcn_s_memrealtime();
  const unsigned long long rt0 = tp, ck0 = __builtin_amdgcn_s_memtime();
  auto mark = [&](int i) {
    if (g == 0 && t == 0) {
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      pt[i] += now - tp;
      tp = now;
    }
  };
  for (int s = 0; s < args.total_steps; ++s) {
    const int j = s % args.nb;
    const int64_t mb0 = (int64_t)j * args.mb;
    const int B = (int)std::min<int64_t>(args.mb, args.N - mb0);
    const float invB = 1.0f / (float)B;
    const int myrows = std::max(0, std::min(R, B - g * R));
    // ---- phase A: partial gradient of this workgroup's rows ------------------------------------
    for (int k = t; k < Lp + 4; k += UPD_THREADS) Ga[k] = 0.0f;
    __syncthreads();
    for (int c0 = 0; c0 < myrows; c0 += UPD_RC)
      upd_chunk<KD, KA>(args, W, Ga, a, mb0 + (int64_t)g * R + c0, std::min(UPD_RC, myrows - c0), invB,
                reinterpret_cast<unsigned long long*>(hdr + 16));
    mark(0);   // phase A compute
    const __amdgpu_buffer_rsrc_t rs_part = upd_rsrc(args.part), rs_red = upd_rsrc(args.red);
    for (int q = t; q < Qtot; q += UPD_THREADS)
      st4_sc1(rs_part, ((size_t)g * Qtot + q) * 4, *reinterpret_cast<const float4*>(Ga + 4 * q));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    mark(1);   // publish partials
    if (t == 0) {
      __hip_atomic_fetch_add(args.ctr + 0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_abort = upd_wait(args.ctr, 0, (unsigned)G * (unsigned)(s + 1)) ? 0 : 1;
    }
    __syncthreads();
    if (*s_abort) return;
    mark(2);   // wait A
    // ---- phase B: reduce slice [qlo, qhi) over the G partials (workgroup order) ---------------
    {
      const int qlo = (int)((int64_t)Qtot * g / G), qhi = (int)((int64_t)Qtot * (g + 1) / G);
      const int nq = qhi - qlo;
      float ssq = 0.f;
      if (nq > UPD_THREADS / 2) {
        // wide slices (few workgroups): each thread owns whole quads, partials summed in order
        for (int qi = t; qi < nq; qi += UPD_THREADS) {
          float4 acc = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
          for (int gg = 0; gg < G; ++gg) {
            const float4 v = ld4_sc1(rs_part, ((size_t)gg * Qtot + qlo + qi) * 4);
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
          }
          st4_sc1(rs_red, (size_t)(qlo + qi) * 4, acc);
          if (qlo + qi < Qp) ssq += acc.x * acc.x + acc.y * acc.y + acc.z * acc.z + acc.w * acc.w;
        }
      } else if (nq > 0) {
        // narrow slices: split the G partials of each quad over spl threads, combine in LDS
        int spl = 1;
        while (spl * 2 * nq <= UPD_THREADS && spl * 2 <= G) spl *= 2;
        float4* red4 = reinterpret_cast<float4*>(scratch);   // [spl][nq]
        if (t < spl * nq) {
          const int qi = t % nq, sub = t / nq;
          float4 acc = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 16
          for (int gg = sub; gg < G; gg += spl) {
            const float4 v = ld4_sc1(rs_part, ((size_t)gg * Qtot + qlo + qi) * 4);
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
          }
          red4[sub * nq + qi] = acc;
        }
        __syncthreads();
        if (t < nq) {
          float4 acc = red4[t];
          for (int sub = 1; sub < spl; ++sub) {
            const float4 v = red4[sub * nq + t];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
          }
          st4_sc1(rs_red, (size_t)(qlo + t) * 4, acc);
          if (qlo + t < Qp) ssq = acc.x * acc.x + acc.y * acc.y + acc.z * acc.z + acc.w * acc.w;
        }
      }
      // block sum of ssq (threads < nq hold the pieces; fixed order)
      ssq = wave_sum_f32_to63(ssq);
      if ((t & 63) == 63) s_ssq[t >> 6] = ssq;
      __syncthreads();
      if (t == 0) {
        float tot = 0.f;
        for (int w = 0; w < UPD_THREADS / 64; ++w) tot += s_ssq[w];
        st_sc1f(args.sq + g, tot);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      mark(3);   // slice reduce
      if (t == 0) {
        __hip_atomic_fetch_add(args.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *s_abort = upd_wait(args.ctr, 1, (unsigned)G * (unsigned)(s + 1)) ? 0 : 1;
      }
      __syncthreads();
      if (*s_abort) return;
      mark(4);   // wait B
    }
    // ---- phase C: clip_grad_norm_(2.0) + AdamW on every workgroup's own copy ------------------
    float4 gq[NQ];   // this thread's gradient quads: loads issued first, in flight under the norm
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int q = t + i * UPD_THREADS;
      if (q < Qp) gq[i] = ld4_sc1(rs_red, (size_t)q * 4);
    }
    {
      float piece = t < G ? ld_sc1f(args.sq + t) : 0.f;     // every workgroup: same tree
      piece = wave_sum_f32_to63(piece);
      if ((t & 63) == 63) s_ssq[t >> 6] = piece;
      __syncthreads();
      if (t == 0) {
        float tot = 0.f;
        for (int w = 0; w < UPD_THREADS / 64; ++w) tot += s_ssq[w];
        const float norm = sqrtf(tot);
        const float coef = args.max_norm / (norm + 1e-6f);
        s_bcast[0] = coef < 1.0f ? coef : 1.0f;
        const float4 lp = ld4_sc1(rs_red, (size_t)Qp * 4);
        s_bcast[1] = lp.x * invB + args.vf_coef * (lp.y * invB) - args.ent_coef * (lp.z * invB);
      }
      __syncthreads();
    }
    mark(5);   // norm + loss
    const float clipc = s_bcast[0];
    loss_last = s_bcast[1];
    {
      const double tstep = (double)step0 + (double)(s + 1);
      const double bc1 = 1.0 - pow((double)args.beta1, tstep);
      const double bc2 = 1.0 - pow((double)args.beta2, tstep);
      const float step_size = (float)((double)args.lr / bc1);
      const float inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));   // scalar divide -> one multiply
      const float decay = (float)(1.0 - (double)args.lr * (double)args.wd);
      const float b2 = args.beta2;
      const float omb1 = (float)(1.0 - (double)args.beta1), omb2 = (float)(1.0 - (double)args.beta2);
      constexpr int BATCH = NQ;
#pragma unroll
      for (int i0 = 0; i0 < NQ; i0 += BATCH) {
#pragma unroll
        for (int b = 0; b < BATCH; ++b) {
          const int i = i0 + b;
          const int q = t + i * UPD_THREADS;
          if (i < NQ && q < Qp) {
            float4 pw = *reinterpret_cast<float4*>(W + 4 * q);
            float4 m4 = mreg[i], v4 = vreg[i];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float gr = f4get(gq[i], e) * clipc;
              float m = f4get(m4, e), v = f4get(v4, e), p = f4get(pw, e);
              p = p * decay;
              m = m + omb1 * (gr - m);
              v = v * b2 + omb2 * gr * gr;
              const float denom = __builtin_amdgcn_sqrtf(v) * inv_bc2_sqrt + args.eps;
              float rq = __builtin_amdgcn_rcpf(denom);
              rq = rq * (2.0f - denom * rq);              // one Newton step: ~0.5 ulp
              p = p - step_size * (m * rq);
              f4set(m4, e, m);
              f4set(v4, e, v);
              f4set(pw, e, p);
            }
            mreg[i] = m4;
            vreg[i] = v4;
            *reinterpret_cast<float4*>(W + 4 * q) = pw;
          }
        }
      }
    }
    __syncthreads();
    mark(6);   // AdamW
  }
  // ---- write back (workgroup 0): parameters, moments, step count, last loss -------------------
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int q = t + i * UPD_THREADS;
      if (q < Qp) *reinterpret_cast<float4*>(Ga + 4 * q) = mreg[i];
    }
    __syncthreads();
    for (int k = t; k < Lp; k += UPD_THREADS) {
      const int f = upd_flat_of(n, k);
      if (f >= 0) {
        args.params[f] = W[k];
        args.exp_avg[f] = Ga[k];
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int q = t + i * UPD_THREADS;
      if (q < Qp) *reinterpret_cast<float4*>(Ga + 4 * q) = vreg[i];
    }
    __syncthreads();
    for (int k = t; k < Lp; k += UPD_THREADS) {
      const int f = upd_flat_of(n, k);
      if (f >= 0) args.exp_avg_sq[f] = Ga[k];
    }
    if (t == 0) {
      for (int i = 0; i < 7; ++i) args.prof[i] = pt[i];
      args.prof[7] = (unsigned long long)args.total_steps;
      args.prof[30] = __builtin_amdgcn_s_memrealtime() - rt0;
      args.prof[31] = __builtin_amdgcn_s_memtime() - ck0;
      for (int i = 0; i < 22; ++i) args.prof[8 + i] = reinterpret_cast<unsigned long long*>(hdr + 16)[i];
      args.adam_step[0] = step0 + (float)args.total_steps;
      if (args.loss_out) args.loss_out[0] = loss_last;
    }
  }
}

// ActorCritic.get_evaluate over N rows (PPO.learn's policy_old pass, PPO.py:127-154):
// log_prob, state value and (optionally) entropy per row, with exactly the update kernel's
// forward arithmetic, so the first minibatch of learn() sees ratio == 1 exactly, as in the
// reference.  Workgroups stride over 8-row chunks; parameters are staged once into LDS.
template <int KD, int KA>
__global__ __launch_bounds__(UPD_THREADS, 1) void ppo_evaluate_kernel(UpdArgs args, float* logp_out,
                                                                    float* V_out, float* H_out) {
  extern __shared__ __align__(16) float upd_lds[];
  const UpdNet& n = args.net;
  const int t = threadIdx.x;
  float* W = upd_lds + 64;
  const UpdAct a = upd_carve(W + n.Lp, n);
  for (int k = t; k < n.Lp; k += UPD_THREADS) {
    const int f = upd_flat_of(n, k);
    W[k] = f >= 0 ? args.params[f] : 0.0f;
  }
  __syncthreads();
  unsigned long long tl = 0;
  const int64_t nchunks = (args.N + UPD_RC - 1) / UPD_RC;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t row0 = c * UPD_RC;
    const int rc = (int)std::min<int64_t>(UPD_RC, args.N - row0);
    upd_forward(n, W, a, args.S, args.act, row0, rc, nullptr, false, tl);
    const int r = t >> 5, l = t & 31;
    if (l == 0 && r < rc) {
      UpdDist d;
      upd_row_dist<KD, KA>(n, a.O + r * a.OX, a.Ar + r * a.AX, d);
      logp_out[row0 + r] = d.logp;
      V_out[row0 + r] = a.O[r * a.OX + n.ocol[n.nh - 1]];
      if (H_out) H_out[row0 + r] = d.H;
    }
    __syncthreads();
  }
}

// ---- stepped mode (world_size > 1): one optimizer step = grad kernel -> RCCL all-reduce of the
// flat gradient (caller) -> AdamW kernel.  Parameters and moments live in HBM in the LDS-image
// layout between launches ("images"); prl_ppo_image converts to / from torch's flat vectors.

// Phase A + B of one step for this rank's rows [row0, row0 + B_local) of global minibatch j:
// partial gradients per workgroup, then the in-GPU reduction into grad_out[Lp + 4] (the last
// quad: loss partials {sum -min(s1,s2), sum SmoothL1, sum H}).  inv_count = 1 / (rows of the
// union minibatch over all ranks), so the all-reduced sum is the union's gradient.
template <int KD, int KA>
__global__ __launch_bounds__(UPD_THREADS, 1) void ppo_grad_kernel(UpdArgs args, const float* img,
                                                                float* grad_out, int64_t row0,
                                                                int B_local, float inv_count) {
  extern __shared__ __align__(16) float upd_lds[];
  const UpdNet& n = args.net;
  const int t = threadIdx.x, g = blockIdx.x, G = args.G;
  const int Lp = n.Lp, Qp = Lp / 4, Qtot = Qp + 1;
  float* hdr = upd_lds;
  float* W = upd_lds + 64;
  float* Ga = W + Lp;
  float* scratch = Ga + Lp + 4;
  const UpdAct a = upd_carve(scratch, n);
  float* s_ssq = hdr + 4;
  int* s_abort = reinterpret_cast<int*>(hdr + 8);
  unsigned long long* tm = reinterpret_cast<unsigned long long*>(hdr + 16);
  for (int q = t; q < Qp; q += UPD_THREADS)   // written by the previous launch: plain loads
    *reinterpret_cast<float4*>(W + 4 * q) = *reinterpret_cast<const float4*>(img + 4 * q);
  for (int k = t; k < Lp + 4; k += UPD_THREADS) Ga[k] = 0.0f;
  if (t < 24) tm[t] = 0ull;
  __syncthreads();
  const int R = args.R;
  const int myrows = std::max(0, std::min(R, B_local - g * R));
  for (int c0 = 0; c0 < myrows; c0 += UPD_RC)
    upd_chunk<KD, KA>(args, W, Ga, a, row0 + (int64_t)g * R + c0, std::min(UPD_RC, myrows - c0),
                      inv_count, tm);
  const __amdgpu_buffer_rsrc_t rs_part = upd_rsrc(args.part), rs_red = upd_rsrc(grad_out);
  for (int q = t; q < Qtot; q += UPD_THREADS)
    st4_sc1(rs_part, ((size_t)g * Qtot + q) * 4, *reinterpret_cast<const float4*>(Ga + 4 * q));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __hip_atomic_fetch_add(args.ctr + 0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_abort = upd_wait(args.ctr, 0, (unsigned)G) ? 0 : 1;
  }
  __syncthreads();
  if (*s_abort) return;
  const int qlo = (int)((int64_t)Qtot * g / G), qhi = (int)((int64_t)Qtot * (g + 1) / G);
  const int nq = qhi - qlo;
  if (nq > UPD_THREADS / 2) {
    for (int qi = t; qi < nq; qi += UPD_THREADS) {
      float4 acc = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int gg = 0; gg < G; ++gg) {
        const float4 v = ld4_sc1(rs_part, ((size_t)gg * Qtot + qlo + qi) * 4);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      st4_sc1(rs_red, (size_t)(qlo + qi) * 4, acc);
    }
  } else if (nq > 0) {
    int spl = 1;
    while (spl * 2 * nq <= UPD_THREADS && spl * 2 <= G) spl *= 2;
    float4* red4 = reinterpret_cast<float4*>(scratch);
    if (t < spl * nq) {
      const int qi = t % nq, sub = t / nq;
      float4 acc = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int gg = sub; gg < G; gg += spl) {
        const float4 v = ld4_sc1(rs_part, ((size_t)gg * Qtot + qlo + qi) * 4);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      red4[sub * nq + qi] = acc;
    }
    __syncthreads();
    if (t < nq) {
      float4 acc = red4[t];
      for (int sub = 1; sub < spl; ++sub) {
        const float4 v = red4[sub * nq + t];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      st4_sc1(rs_red, (size_t)(qlo + t) * 4, acc);
    }
  }
  (void)s_ssq;
}

// clip_grad_norm_(max_norm) + AdamW on the images, one parameter quad per thread.  Every
// workgroup forms the same norm (same order), so no hand-off is needed.
__global__ __launch_bounds__(UPD_THREADS) void ppo_adam_kernel(int Lp, float* img_p, float* img_m,
                                                             float* img_v, const float* grad,
                                                             double tstep, float lr, float beta1,
                                                             float beta2, float eps, float wd,
                                                             float max_norm, float inv_count,
                                                             float vf_coef, float ent_coef,
                                                             float* loss_out) {
  __shared__ float s_part[UPD_THREADS / 64];
  const int t = threadIdx.x, Qp = Lp / 4;
  float acc = 0.f;
  for (int q = t; q < Qp; q += UPD_THREADS) {
    const float4 r = *reinterpret_cast<const float4*>(grad + 4 * q);
    acc += r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w;
  }
  acc = wave_sum(acc);
  if ((t & 63) == 0) s_part[t >> 6] = acc;
  __syncthreads();
  float tot = 0.f;
  for (int w = 0; w < UPD_THREADS / 64; ++w) tot += s_part[w];
  const float coef = max_norm / (sqrtf(tot) + 1e-6f);
  const float clipc = coef < 1.0f ? coef : 1.0f;
  const double bc1 = 1.0 - pow((double)beta1, tstep);
  const double bc2 = 1.0 - pow((double)beta2, tstep);
  const float step_size = (float)((double)lr / bc1);
  const float inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
  const float decay = (float)(1.0 - (double)lr * (double)wd);
  const float omb1 = (float)(1.0 - (double)beta1), omb2 = (float)(1.0 - (double)beta2);
  const int q = blockIdx.x * UPD_THREADS + t;
  if (q < Qp) {
    const float4 g4 = *reinterpret_cast<const float4*>(grad + 4 * q);
    float4 m4 = *reinterpret_cast<const float4*>(img_m + 4 * q);
    float4 v4 = *reinterpret_cast<const float4*>(img_v + 4 * q);
    float4 pw = *reinterpret_cast<const float4*>(img_p + 4 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gr = f4get(g4, e) * clipc;
      float m = f4get(m4, e), v = f4get(v4, e), p = f4get(pw, e);
      p = p * decay;
      m = m + omb1 * (gr - m);
      v = v * beta2 + omb2 * gr * gr;
      const float denom = __builtin_amdgcn_sqrtf(v) * inv_bc2_sqrt + eps;
      float rq = __builtin_amdgcn_rcpf(denom);
      rq = rq * (2.0f - denom * rq);
      p = p - step_size * (m * rq);
      f4set(m4, e, m);
      f4set(v4, e, v);
      f4set(pw, e, p);
    }
    *reinterpret_cast<float4*>(img_m + 4 * q) = m4;
    *reinterpret_cast<float4*>(img_v + 4 * q) = v4;
    *reinterpret_cast<float4*>(img_p + 4 * q) = pw;
  }
  if (blockIdx.x == 0 && t == 0 && loss_out) {
    const float4 lp = *reinterpret_cast<const float4*>(grad + Lp);
    loss_out[0] = lp.x * inv_count + vf_coef * (lp.y * inv_count) - ent_coef * (lp.z * inv_count);
  }
}

// torch flat vectors <-> images (to_image: flat -> image, else image -> flat)
__global__ __launch_bounds__(UPD_THREADS) void ppo_image_kernel(UpdNet n, float* fp, float* fm,
                                                              float* fv, float* ip, float* im,
                                                              float* iv, int to_image) {
  const int k = blockIdx.x * UPD_THREADS + threadIdx.x;
  if (k >= n.Lp) return;
  const int f = upd_flat_of(n, k);
  if (to_image) {
    ip[k] = f >= 0 ? fp[f] : 0.0f;
    im[k] = f >= 0 ? fm[f] : 0.0f;
    iv[k] = f >= 0 ? fv[f] : 0.0f;
  } else if (f >= 0) {
    fp[f] = ip[k];
    fm[f] = im[k];
    fv[f] = iv[k];
  }
}

}  // namespace prl

using namespace prl;

namespace {

// LDS image + flat offsets of the reference's parameter tensors, torch parameters() order.
bool upd_layout(int D, int A, int discrete, UpdNet& n) {
  if (D < 1 || D > UPD_MAXD || A < 1 || A > UPD_MAXA) return false;
  n = UpdNet{};
  n.D = D;
  n.A = A;
  n.discrete = discrete ? 1 : 0;
  n.nh = discrete ? 2 : 3;
  int flat = 0, lds = 0;
  auto add = [&](UpdTensor& t, int rows, int cols, int stride) {
    t.flat = flat;
    t.lds = lds;
    t.rows = rows;
    t.cols = cols;
    t.stride = stride;
    flat += rows * cols;
    lds += (rows * stride + 3) & ~3;
  };
  add(n.w0, UPD_H, D, D | 1);
  add(n.g0, 1, UPD_H, UPD_H);
  add(n.b0, 1, UPD_H, UPD_H);
  int col = 0;
  for (int h = 0; h < n.nh; ++h) {
    const int out = (h == n.nh - 1) ? 1 : A;
    n.out[h] = out;
    n.ocol[h] = col;
    col += out;
    add(n.w1[h], UPD_H, UPD_H, UPD_HS);
    add(n.g1[h], 1, UPD_H, UPD_H);
    add(n.b1[h], 1, UPD_H, UPD_H);
    add(n.w2[h], out, UPD_H, UPD_HS);
    add(n.b2[h], 1, out, out);
  }
  n.nout = col;
  n.P = flat;
  n.Lp = lds;
  return true;
}

int upd_nq(const UpdNet& n) { return (int)cdiv(n.Lp / 4, UPD_THREADS); }
// Specialisations for the configs' shapes (CartPole: discrete, A = 2; Pendulum: continuous,
// A = 1); every other shape runs the generic (runtime head configuration) kernel.
const void* upd_kernel_for(const UpdNet& n) {
  const int nq = upd_nq(n);
  if (n.discrete && n.A == 2 && nq <= 10) return reinterpret_cast<const void*>(ppo_update_kernel<10, 1, 2>);
  if (!n.discrete && n.A == 1 && nq <= 14) return reinterpret_cast<const void*>(ppo_update_kernel<14, 0, 1>);
  if (nq <= 20) return reinterpret_cast<const void*>(ppo_update_kernel<20, -1, 0>);
  return nullptr;
}
const void* upd_grad_kernel_for(const UpdNet& n) {
  if (n.discrete && n.A == 2) return reinterpret_cast<const void*>(ppo_grad_kernel<1, 2>);
  if (!n.discrete && n.A == 1) return reinterpret_cast<const void*>(ppo_grad_kernel<0, 1>);
  return reinterpret_cast<const void*>(ppo_grad_kernel<-1, 0>);
}
const void* upd_eval_kernel_for(const UpdNet& n) {
  if (n.discrete && n.A == 2) return reinterpret_cast<const void*>(ppo_evaluate_kernel<1, 2>);
  if (!n.discrete && n.A == 1) return reinterpret_cast<const void*>(ppo_evaluate_kernel<0, 1>);
  return reinterpret_cast<const void*>(ppo_evaluate_kernel<-1, 0>);
}

int upd_grid(int64_t mb) { return (int)std::min<int64_t>(256, cdiv(mb, UPD_RC)); }

size_t upd_lds_bytes(const UpdNet& n) {
  int DX, AX, OX;
  const int act = upd_act_floats(n.D, n.A, n.nout, DX, AX, OX);
  return sizeof(float) * (size_t)(64 + 2 * n.Lp + 4 + act);
}

struct UpdWs {
  unsigned* ctr;
  unsigned long long* prof;
  float* sq;
  float* red;
  float* part;
};

// workspace: ctr[4] (16 B, zeroed per launch) | prof[32] | sq[256] | red[Qtot*4] | part[G][Qtot*4]
size_t upd_ws_carve(const UpdNet& n, int G, char* base, UpdWs* ws) {
  const size_t Qtot = (size_t)n.Lp / 4 + 1;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
  const size_t o_ctr = take(16), o_prof = take(256), o_sq = take(256 * 4), o_red = take(Qtot * 16),
               o_part = take((size_t)G * Qtot * 16);
  if (ws) {
    ws->ctr = reinterpret_cast<unsigned*>(base + o_ctr);
    ws->prof = reinterpret_cast<unsigned long long*>(base + o_prof);
    ws->sq = reinterpret_cast<float*>(base + o_sq);
    ws->red = reinterpret_cast<float*>(base + o_red);
    ws->part = reinterpret_cast<float*>(base + o_part);
  }
  return off;
}

}  // namespace

extern "C" int prl_ppo_update_info(int32_t D, int32_t A, int32_t discrete, int64_t mini_batch,
                                   int64_t* n_params, int64_t* workspace_bytes, int32_t* grid) {
  UpdNet n;
  PRL_REQUIRE(mini_batch > 0, "prl_ppo_update_info: mini_batch must be > 0");
  if (!upd_layout(D, A, discrete, n)) {
    if (n_params) *n_params = 0;
    if (workspace_bytes) *workspace_bytes = 0;
    if (grid) *grid = 0;
    return PRL_ERR_ARG;   // shape not supported by the fused engine (caller uses the graph path)
  }
  const int G = upd_grid(mini_batch);
  if (n_params) *n_params = n.P;
  if (workspace_bytes) *workspace_bytes = (int64_t)upd_ws_carve(n, G, nullptr, nullptr);
  if (grid) *grid = G;
  return (upd_lds_bytes(n) <= 160 * 1024 && upd_kernel_for(n)) ? PRL_OK : PRL_ERR_ARG;
}

extern "C" int prl_ppo_update(float* params, float* exp_avg, float* exp_avg_sq, float* adam_step,
                              int32_t D, int32_t A, int32_t discrete, const float* S,
                              const float* actions, const float* old_logp, const float* adv,
                              const float* ret, int64_t N, int32_t mini_batch, int32_t k_epochs,
                              float clip, float vf_coef, float ent_coef, float lr, float beta1,
                              float beta2, float eps, float weight_decay, float max_norm,
                              float* loss_out, void* workspace, int64_t workspace_bytes,
                              void* stream) {
  UpdArgs args{};
  PRL_REQUIRE(upd_layout(D, A, discrete, args.net), "prl_ppo_update: D=%d A=%d not supported", D, A);
  PRL_REQUIRE(N > 0 && mini_batch > 0 && k_epochs >= 0, "prl_ppo_update: bad sizes");
  PRL_REQUIRE(params && exp_avg && exp_avg_sq && adam_step && S && actions && old_logp && adv && ret &&
                  workspace, "prl_ppo_update: null pointer");
  const int G = upd_grid(mini_batch);
  UpdWs ws;
  const size_t need = upd_ws_carve(args.net, G, reinterpret_cast<char*>(workspace), &ws);
  PRL_REQUIRE((size_t)workspace_bytes >= need, "prl_ppo_update: workspace %lld < %zu bytes",
              (long long)workspace_bytes, need);
  const int64_t nb = cdiv(N, (int64_t)mini_batch);
  PRL_REQUIRE(nb * (int64_t)k_epochs < (int64_t)(1u << 31) / 256, "prl_ppo_update: too many steps");
  if (k_epochs == 0) return PRL_OK;
  args.S = S;
  args.act = actions;
  args.old_logp = old_logp;
  args.adv = adv;
  args.ret = ret;
  args.N = N;
  args.mb = mini_batch;
  args.nb = (int)nb;
  args.total_steps = (int)(nb * k_epochs);
  args.G = G;
  args.R = (int)cdiv(cdiv((int64_t)mini_batch, (int64_t)G), (int64_t)UPD_RC) * UPD_RC;
  args.clip = clip;
  args.vf_coef = vf_coef;
  args.ent_coef = ent_coef;
  args.lr = lr;
  args.beta1 = beta1;
  args.beta2 = beta2;
  args.eps = eps;
  args.wd = weight_decay;
  args.max_norm = max_norm;
  args.params = params;
  args.exp_avg = exp_avg;
  args.exp_avg_sq = exp_avg_sq;
  args.adam_step = adam_step;
  args.loss_out = loss_out;
  args.part = ws.part;
  args.red = ws.red;
  args.sq = ws.sq;
  args.ctr = ws.ctr;
  args.prof = ws.prof;
  const size_t lds = upd_lds_bytes(args.net);
  PRL_REQUIRE(lds <= 160 * 1024, "prl_ppo_update: %zu B of LDS needed", lds);
  hipStream_t st = as_stream(stream);
  const void* kern = upd_kernel_for(args.net);
  PRL_REQUIRE(kern, "prl_ppo_update: %d parameter quads per thread not built", upd_nq(args.net));
  PRL_HIP_TRY(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  PRL_HIP_TRY(hipMemsetAsync(ws.ctr, 0, 16, st));
  void* kargs[] = {&args};
  PRL_HIP_TRY(hipLaunchCooperativeKernel(kern, dim3(G), dim3(UPD_THREADS), kargs, (unsigned)lds, st));
  return PRL_OK;
}

extern "C" int prl_ppo_evaluate(const float* params, int32_t D, int32_t A, int32_t discrete,
                                const float* S, const float* actions, int64_t N, float* logp,
                                float* V, float* entropy, void* stream) {
  UpdArgs args{};
  PRL_REQUIRE(upd_layout(D, A, discrete, args.net), "prl_ppo_evaluate: D=%d A=%d not supported", D, A);
  PRL_REQUIRE(N >= 0, "prl_ppo_evaluate: N < 0");
  if (N == 0) return PRL_OK;
  PRL_REQUIRE(params && S && actions && logp && V, "prl_ppo_evaluate: null pointer");
  args.params = const_cast<float*>(params);
  args.S = S;
  args.act = actions;
  args.N = N;
  int DX, AX, OX;
  const size_t lds = sizeof(float) * (size_t)(64 + args.net.Lp +
                                              upd_act_floats(D, A, args.net.nout, DX, AX, OX));
  PRL_REQUIRE(lds <= 160 * 1024, "prl_ppo_evaluate: %zu B of LDS needed", lds);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(N, UPD_RC), 2 * 256);
  const void* kern = upd_eval_kernel_for(args.net);
  PRL_HIP_TRY(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  void* kargs[] = {&args, &logp, &V, &entropy};
  PRL_HIP_TRY(hipLaunchKernel(kern, dim3(grid), dim3(UPD_THREADS), kargs, lds, as_stream(stream)));
  return PRL_OK;
}

extern "C" int64_t prl_ppo_image_floats(int32_t D, int32_t A, int32_t discrete) {
  UpdNet n;
  if (!upd_layout(D, A, discrete, n)) return -1;
  return (int64_t)n.Lp + 4;
}

extern "C" int prl_ppo_image(int32_t D, int32_t A, int32_t discrete, float* params, float* exp_avg,
                             float* exp_avg_sq, float* img_params, float* img_m, float* img_v,
                             int32_t to_image, void* stream) {
  UpdNet n;
  PRL_REQUIRE(upd_layout(D, A, discrete, n), "prl_ppo_image: D=%d A=%d not supported", D, A);
  PRL_REQUIRE(params && exp_avg && exp_avg_sq && img_params && img_m && img_v,
              "prl_ppo_image: null pointer");
  hipLaunchKernelGGL(ppo_image_kernel, dim3((unsigned)cdiv(n.Lp, UPD_THREADS)), dim3(UPD_THREADS),
                     0, as_stream(stream), n, params, exp_avg, exp_avg_sq, img_params, img_m, img_v,
                     to_image ? 1 : 0);
  PRL_LAUNCH_CHECK("ppo_image");
  return PRL_OK;
}

extern "C" int prl_ppo_grad_step(const float* img_params, int32_t D, int32_t A, int32_t discrete,
                                 const float* S, const float* actions, const float* old_logp,
                                 const float* adv, const float* ret, int64_t N, int32_t mini_batch,
                                 int64_t minibatch_index, float inv_count, float clip,
                                 float vf_coef, float* grad_out, void* workspace,
                                 int64_t workspace_bytes, void* stream) {
  UpdArgs args{};
  PRL_REQUIRE(upd_layout(D, A, discrete, args.net), "prl_ppo_grad_step: D=%d A=%d not supported", D, A);
  PRL_REQUIRE(N >= 0 && mini_batch > 0 && minibatch_index >= 0, "prl_ppo_grad_step: bad sizes");
  PRL_REQUIRE(img_params && grad_out && workspace, "prl_ppo_grad_step: null pointer");
  const int G = upd_grid(mini_batch);
  UpdWs ws;
  const size_t need = upd_ws_carve(args.net, G, reinterpret_cast<char*>(workspace), &ws);
  PRL_REQUIRE((size_t)workspace_bytes >= need, "prl_ppo_grad_step: workspace too small");
  const int64_t row0 = minibatch_index * (int64_t)mini_batch;
  const int B_local = (int)std::max<int64_t>(0, std::min<int64_t>(mini_batch, N - row0));
  PRL_REQUIRE(B_local == 0 || (S && actions && old_logp && adv && ret), "prl_ppo_grad_step: null input");
  args.S = S;
  args.act = actions;
  args.old_logp = old_logp;
  args.adv = adv;
  args.ret = ret;
  args.N = N;
  args.mb = mini_batch;
  args.G = G;
  args.R = (int)cdiv(cdiv((int64_t)mini_batch, (int64_t)G), (int64_t)UPD_RC) * UPD_RC;
  args.clip = clip;
  args.vf_coef = vf_coef;
  args.part = ws.part;
  args.ctr = ws.ctr;
  const size_t lds = upd_lds_bytes(args.net);
  hipStream_t st = as_stream(stream);
  const void* kern = upd_grad_kernel_for(args.net);
  PRL_HIP_TRY(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  PRL_HIP_TRY(hipMemsetAsync(ws.ctr, 0, 16, st));
  float inv = inv_count;
  int64_t r0 = row0;
  int bl = B_local;
  const float* img = img_params;
  void* kargs[] = {&args, &img, &grad_out, &r0, &bl, &inv};
  // plain launch: G <= 256 workgroups of 1 per CU are co-resident in practice; the in-kernel
  // wait is bounded and reports a timeout through the status word like the persistent kernel
  PRL_HIP_TRY(hipLaunchKernel(kern, dim3(G), dim3(UPD_THREADS), kargs, lds, st));
  return PRL_OK;
}

extern "C" int prl_ppo_adam_step(float* img_params, float* img_m, float* img_v, int32_t D,
                                 int32_t A, int32_t discrete, const float* grad, int64_t step,
                                 float lr, float beta1, float beta2, float eps, float weight_decay,
                                 float max_norm, float inv_count, float vf_coef, float ent_coef,
                                 float* loss_out, void* stream) {
  UpdNet n;
  PRL_REQUIRE(upd_layout(D, A, discrete, n), "prl_ppo_adam_step: D=%d A=%d not supported", D, A);
  PRL_REQUIRE(img_params && img_m && img_v && grad && step >= 1, "prl_ppo_adam_step: bad arguments");
  hipLaunchKernelGGL(ppo_adam_kernel, dim3((unsigned)cdiv(n.Lp / 4, UPD_THREADS)), dim3(UPD_THREADS),
                     0, as_stream(stream), n.Lp, img_params, img_m, img_v, grad, (double)step, lr,
                     beta1, beta2, eps, weight_decay, max_norm, inv_count, vf_coef, ent_coef, loss_out);
  PRL_LAUNCH_CHECK("ppo_adam_step");
  return PRL_OK;
}

// status word of the last launch on this workspace (device u32: 0 ok, 1 = in-kernel timeout)
extern "C" int prl_ppo_update_status_ptr(void* workspace, uint32_t** status) {
  PRL_REQUIRE(workspace && status, "prl_ppo_update_status_ptr: null pointer");
  *status = reinterpret_cast<uint32_t*>(workspace) + 3;
  return PRL_OK;
}
