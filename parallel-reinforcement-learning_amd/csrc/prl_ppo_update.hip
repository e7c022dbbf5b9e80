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
  float* priv;      // [G][2][Lp]
  unsigned* ctr;    // [0] arrivals A, [1] arrivals B, [2] abort, [3] status
};

// ---- sc1 (write-through / L1-bypassing) accessors -------------------------------------------
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ inline __amdgpu_buffer_rsrc_t upd_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ inline float4 ld4_sc1(const float* p) {
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(upd_rsrc(p), 0, 0, 16);
  return float4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                __uint_as_float(v.w)};
}
__device__ inline void st4_sc1(float* p, float4 x) {
  v4u v;
  v.x = __float_as_uint(x.x);
  v.y = __float_as_uint(x.y);
  v.z = __float_as_uint(x.z);
  v.w = __float_as_uint(x.w);
  __builtin_amdgcn_raw_buffer_store_b128(v, upd_rsrc(p), 0, 0, 16);
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
  float* T0;      // [RC][HS]  H0 raw -> dF -> dH0
  float* XH0;     // [RC][HS]
  float* F;       // [RC][HS]
  float* DU0;     // [RC][HS]
  float* rstd0;   // [RC][8]
  float* heads;   // per head h at heads + h * UPD_HEAD_FLOATS:
                  //   ZB [RC][HS] (Z raw -> dG -> dZ), XH, Gh, DU [RC][HS], rstd [RC][8]
  __device__ float* ZB(int h) const { return heads + h * UPD_HEAD_FLOATS; }
  __device__ float* XH(int h) const { return heads + h * UPD_HEAD_FLOATS + UPD_RC * UPD_HS; }
  __device__ float* Gh(int h) const { return heads + h * UPD_HEAD_FLOATS + 2 * UPD_RC * UPD_HS; }
  __device__ float* DU(int h) const { return heads + h * UPD_HEAD_FLOATS + 3 * UPD_RC * UPD_HS; }
  __device__ float* rstd(int h) const { return heads + h * UPD_HEAD_FLOATS + 4 * UPD_RC * UPD_HS; }
  float* O;       // [RC][OX]
  float* dO;      // [RC][OX]
  int DX, AX, OX;
};

__host__ __device__ inline int upd_act_floats(int D, int A, int nout, int& DX, int& AX, int& OX) {
  DX = (D + 3) & ~3;
  AX = (A + 3) & ~3;
  OX = (nout + 3) & ~3;
  return UPD_RC * (DX + AX + 4 + 4 + 4 * UPD_HS + 8 + UPD_MAXH * (4 * UPD_HS + 8) + 2 * OX) + 16;
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
  a.O = take(UPD_RC * a.OX);
  a.dO = take(UPD_RC * a.OX);
  return a;
}

// GroupNorm(8 groups of 8) + SiLU forward of one (row, group): same arithmetic as gn_silu_fwd.
__device__ inline void upd_gn_fwd(const float* raw, const float* gw, const float* gb, float* xh_out,
                                  float* y_out, float* rstd_out) {
  float v[8];
  const float4 a = *reinterpret_cast<const float4*>(raw);
  const float4 b = *reinterpret_cast<const float4*>(raw + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
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

// backward of the above for one (row, group): dio holds dOut on entry, dX on exit; du_out = dy
__device__ inline void upd_gn_bwd(float* dio, const float* xh_in, const float* gw, const float* gb,
                                  float rstd, float* du_out) {
  float go[8], xh[8];
  {
    const float4 a = *reinterpret_cast<const float4*>(dio);
    const float4 b = *reinterpret_cast<const float4*>(dio + 4);
    go[0] = a.x; go[1] = a.y; go[2] = a.z; go[3] = a.w; go[4] = b.x; go[5] = b.y; go[6] = b.z; go[7] = b.w;
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
  *reinterpret_cast<float4*>(dio) = float4{dx[0], dx[1], dx[2], dx[3]};
  *reinterpret_cast<float4*>(dio + 4) = float4{dx[4], dx[5], dx[6], dx[7]};
  *reinterpret_cast<float4*>(du_out) = float4{dy[0], dy[1], dy[2], dy[3]};
  *reinterpret_cast<float4*>(du_out + 4) = float4{dy[4], dy[5], dy[6], dy[7]};
}

// Per-row loss (surrogate, prl_loss.hip semantics) and the gradient w.r.t. the head outputs.
// Loops run to the compile-time UPD_MAXA with `k < A` guards so everything stays in registers.
__device__ inline void upd_row_loss(const UpdNet& n, const UpdAct& a, int r, float invB, float clip,
                                    float vf_coef) {
  const float* O = a.O + r * a.OX;
  float* dO = a.dO + r * a.OX;
  const int A = n.A;
  float logp = 0.f, H = 0.f;
  float p[UPD_MAXA], q[UPD_MAXA];
  float S2 = 0.f, qa = 1.f;
  int ai = 0;
  if (n.discrete) {
    float mx = O[0];
#pragma unroll
    for (int k = 1; k < UPD_MAXA; ++k)
      if (k < A) mx = fmaxf(mx, O[k]);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      p[k] = k < A ? expf(O[k] - mx) : 0.f;
      s += p[k];
    }
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      p[k] = k < A ? p[k] / s : 0.f;
      S2 += p[k];
    }
    ai = (int)a.Ar[r * a.AX];
    const bool bad = ai < 0 || ai >= A;   // torch's gather would raise: poison the step instead
    float la = 0.f;
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      q[k] = p[k] / S2;
      if (k < A) {
        const float c = q[k] < FLT_EPSILON ? FLT_EPSILON : (q[k] > 1.0f - FLT_EPSILON ? 1.0f - FLT_EPSILON : q[k]);
        const float l = logf(c);
        H += l * q[k];
        if (k == ai) { la = l; qa = q[k]; }
      }
    }
    H = -H;
    logp = bad ? __builtin_nanf("") : la;
  } else {
    const float half_log_2pi = 0.91893853320467274f;  // log(sqrt(2 pi))
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      if (k < A) {
        const float mu = O[k];
        const float lsr = O[A + k];
        const float lsc = lsr < -2.0f ? -2.0f : (lsr > 2.0f ? 2.0f : lsr);
        const float sd = log1pf(expf(lsc));               // softplus, beta 1 (lsc <= 2 < 20)
        const float d = a.Ar[r * a.AX + k] - mu;
        const float lsd = logf(sd);
        logp += -(d * d) / (2.0f * (sd * sd)) - lsd - half_log_2pi;
        H += 0.5f + half_log_2pi + lsd;
      }
    }
  }
  const float V = O[n.ocol[n.nh - 1]];
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
  dO[n.ocol[n.nh - 1]] = vf_coef * invB * gx;
  a.lossp[r * 4 + 0] = -m;
  a.lossp[r * 4 + 1] = sl;
  a.lossp[r * 4 + 2] = H;
  // d logp / d head outputs
  if (n.discrete) {
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

// one chunk of rc <= RC rows: forward, loss, backward; gradients accumulated into Ga (LDS image)
__device__ void upd_chunk(const UpdArgs& args, const float* W, float* Ga, const UpdAct& a,
                          int64_t row0, int rc, float invB) {
  const UpdNet& n = args.net;
  const int t = threadIdx.x;
  const int D = n.D, A = n.A, nh = n.nh;
  // 0. inputs
  for (int i = t; i < UPD_RC * a.DX; i += UPD_THREADS) {
    const int r = i / a.DX, d = i % a.DX;
    a.X[i] = (r < rc && d < D) ? args.S[(row0 + r) * D + d] : 0.0f;
  }
  const int Aw = n.discrete ? 1 : A;
  for (int i = t; i < UPD_RC * a.AX; i += UPD_THREADS) {
    const int r = i / a.AX, k = i % a.AX;
    a.Ar[i] = (r < rc && k < Aw) ? args.act[(row0 + r) * Aw + k] : 0.0f;
  }
  if (t < UPD_RC) {
    const bool ok = t < rc;
    a.oldlp[t] = ok ? args.old_logp[row0 + t] : 0.0f;
    a.adv[t] = ok ? args.adv[row0 + t] : 0.0f;
    a.ret[t] = ok ? args.ret[row0 + t] : 0.0f;
  }
  __syncthreads();
  // 1. H0 = X W0^T
  for (int i = t; i < rc * UPD_H; i += UPD_THREADS) {
    const int r = i >> 6, o = i & 63;
    const float* w = W + n.w0.lds + o * n.w0.stride;
    const float* x = a.X + r * a.DX;
    float acc = 0.f;
    for (int d = 0; d < D; ++d) acc += x[d] * w[d];
    a.T0[r * UPD_HS + o] = acc;
  }
  __syncthreads();
  // 2. trunk GroupNorm + SiLU
  if (t < rc * 8) {
    const int r = t >> 3, g = t & 7;
    upd_gn_fwd(a.T0 + r * UPD_HS + g * 8, W + n.g0.lds + g * 8, W + n.b0.lds + g * 8,
               a.XH0 + r * UPD_HS + g * 8, a.F + r * UPD_HS + g * 8, a.rstd0 + r * 8 + g);
  }
  __syncthreads();
  // 3. Z_h = F W1_h^T   (thread = (head, output column), all rows)
  if (t < nh * UPD_H) {
    const int h = t >> 6, o = t & 63;
    const float* w = W + n.w1[h].lds + o * UPD_HS;
    float acc[UPD_RC];
#pragma unroll
    for (int r = 0; r < UPD_RC; ++r) acc[r] = 0.f;
    for (int i = 0; i < UPD_H; i += 4) {
      const float4 wv = *reinterpret_cast<const float4*>(w + i);
#pragma unroll
      for (int r = 0; r < UPD_RC; ++r) {
        const float4 f = *reinterpret_cast<const float4*>(a.F + r * UPD_HS + i);
        acc[r] += f.x * wv.x;
        acc[r] += f.y * wv.y;
        acc[r] += f.z * wv.z;
        acc[r] += f.w * wv.w;
      }
    }
#pragma unroll
    for (int r = 0; r < UPD_RC; ++r)
      if (r < rc) a.ZB(h)[r * UPD_HS + o] = acc[r];
  }
  __syncthreads();
  // 4. head GroupNorm + SiLU
  if (t < nh * rc * 8) {
    const int h = t / (rc * 8), rg = t % (rc * 8), r = rg >> 3, g = rg & 7;
    upd_gn_fwd(a.ZB(h) + r * UPD_HS + g * 8, W + n.g1[h].lds + g * 8, W + n.b1[h].lds + g * 8,
               a.XH(h) + r * UPD_HS + g * 8, a.Gh(h) + r * UPD_HS + g * 8, a.rstd(h) + r * 8 + g);
  }
  __syncthreads();
  // 5. outputs O[r][col] = G_h W2_h^T + b2_h
  for (int i = t; i < rc * n.nout; i += UPD_THREADS) {
    const int r = i / n.nout, j = i % n.nout;
    int h = 0;
    while (h + 1 < nh && j >= n.ocol[h + 1]) ++h;
    const int k = j - n.ocol[h];
    const float* w = W + n.w2[h].lds + k * n.w2[h].stride;
    const float* gv = a.Gh(h) + r * UPD_HS;
    float acc = 0.f;
    for (int c = 0; c < UPD_H; c += 4) {
      const float4 wv = *reinterpret_cast<const float4*>(w + c);
      const float4 g4 = *reinterpret_cast<const float4*>(gv + c);
      acc += g4.x * wv.x;
      acc += g4.y * wv.y;
      acc += g4.z * wv.z;
      acc += g4.w * wv.w;
    }
    a.O[r * a.OX + j] = acc + W[n.b2[h].lds + k];
  }
  __syncthreads();
  // 6. loss + d(head outputs)
  if (t < rc) upd_row_loss(n, a, t, invB, args.clip, args.vf_coef);
  __syncthreads();
  // 7. dG_h = dO_h W2_h;  dW2_h += dO_h^T G_h;  db2_h;  loss partials
  for (int i = t; i < nh * rc * UPD_H; i += UPD_THREADS) {
    const int h = i / (rc * UPD_H), ri = i % (rc * UPD_H), r = ri >> 6, c = ri & 63;
    const float* dO = a.dO + r * a.OX + n.ocol[h];
    float acc = 0.f;
    for (int k = 0; k < n.out[h]; ++k) acc += dO[k] * W[n.w2[h].lds + k * n.w2[h].stride + c];
    a.ZB(h)[r * UPD_HS + c] = acc;
  }
  for (int i = t; i < n.nout * UPD_H; i += UPD_THREADS) {
    const int j = i >> 6, c = i & 63;
    int h = 0;
    while (h + 1 < nh && j >= n.ocol[h + 1]) ++h;
    const int k = j - n.ocol[h];
    float acc = 0.f;
    for (int r = 0; r < rc; ++r) acc += a.dO[r * a.OX + j] * a.Gh(h)[r * UPD_HS + c];
    Ga[n.w2[h].lds + k * n.w2[h].stride + c] += acc;
  }
  if (t < n.nout) {
    int h = 0;
    while (h + 1 < nh && t >= n.ocol[h + 1]) ++h;
    float acc = 0.f;
    for (int r = 0; r < rc; ++r) acc += a.dO[r * a.OX + t];
    Ga[n.b2[h].lds + (t - n.ocol[h])] += acc;
  }
  if (t >= 64 && t < 64 + 3) {
    const int which = t - 64;
    float acc = 0.f;
    for (int r = 0; r < rc; ++r) acc += a.lossp[r * 4 + which];
    Ga[n.Lp + which] += acc;
  }
  __syncthreads();
  // 8. head GroupNorm + SiLU backward (ZB: dG -> dZ)
  if (t < nh * rc * 8) {
    const int h = t / (rc * 8), rg = t % (rc * 8), r = rg >> 3, g = rg & 7;
    upd_gn_bwd(a.ZB(h) + r * UPD_HS + g * 8, a.XH(h) + r * UPD_HS + g * 8,
               W + n.g1[h].lds + g * 8, W + n.b1[h].lds + g * 8, a.rstd(h)[r * 8 + g],
               a.DU(h) + r * UPD_HS + g * 8);
  }
  __syncthreads();
  // 9a. dW1_h += dZ_h^T F   (thread: 4 contiguous input columns x 4 output rows, per head)
  {
    const int i4 = (t & 15) * 4, ob = t >> 4;
    for (int h = 0; h < nh; ++h) {
      float acc[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[k][c] = 0.f;
      for (int r = 0; r < rc; ++r) {
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
  // 9b. head GroupNorm weight/bias grads (column sums)
  if (t < nh * UPD_H) {
    const int h = t >> 6, c = t & 63;
    float sw = 0.f, sb = 0.f;
    for (int r = 0; r < rc; ++r) {
      const float du = a.DU(h)[r * UPD_HS + c];
      sw += du * a.XH(h)[r * UPD_HS + c];
      sb += du;
    }
    Ga[n.g1[h].lds + c] += sw;
    Ga[n.b1[h].lds + c] += sb;
  }
  // 9c. dF = sum_h dZ_h W1_h   (thread: one row, 2 adjacent columns)
  for (int i = t; i < rc * 32; i += UPD_THREADS) {
    const int r = i >> 5, c2 = (i & 31) * 2;
    float s0 = 0.f, s1 = 0.f;
    for (int h = 0; h < nh; ++h) {
      const float* dz = a.ZB(h) + r * UPD_HS;
      const float* w = W + n.w1[h].lds + c2;
      for (int o = 0; o < UPD_H; ++o) {
        const float2 wv = *reinterpret_cast<const float2*>(w + o * UPD_HS);
        const float z = dz[o];
        s0 += z * wv.x;
        s1 += z * wv.y;
      }
    }
    a.T0[r * UPD_HS + c2] = s0;
    a.T0[r * UPD_HS + c2 + 1] = s1;
  }
  __syncthreads();
  // 10. trunk GroupNorm + SiLU backward (T0: dF -> dH0)
  if (t < rc * 8) {
    const int r = t >> 3, g = t & 7;
    upd_gn_bwd(a.T0 + r * UPD_HS + g * 8, a.XH0 + r * UPD_HS + g * 8, W + n.g0.lds + g * 8,
               W + n.b0.lds + g * 8, a.rstd0[r * 8 + g], a.DU0 + r * UPD_HS + g * 8);
  }
  __syncthreads();
  // 11. dW0 += dH0^T X;  trunk GroupNorm weight/bias grads
  for (int i = t; i < UPD_H * D; i += UPD_THREADS) {
    const int o = i / D, d = i % D;
    float acc = 0.f;
    for (int r = 0; r < rc; ++r) acc += a.T0[r * UPD_HS + o] * a.X[r * a.DX + d];
    Ga[n.w0.lds + o * n.w0.stride + d] += acc;
  }
  if (t < UPD_H) {
    float sw = 0.f, sb = 0.f;
    for (int r = 0; r < rc; ++r) {
      const float du = a.DU0[r * UPD_HS + t];
      sw += du * a.XH0[r * UPD_HS + t];
      sb += du;
    }
    Ga[n.g0.lds + t] += sw;
    Ga[n.b0.lds + t] += sb;
  }
  __syncthreads();
}

__global__ __launch_bounds__(UPD_THREADS, 1) void ppo_update_kernel(UpdArgs args) {
  extern __shared__ __align__(16) float upd_lds[];
  const UpdNet& n = args.net;
  const int t = threadIdx.x, g = blockIdx.x, G = args.G;
  const int Lp = n.Lp;
  const int Qp = Lp / 4;            // parameter quads
  const int Qtot = Qp + 1;          // + one quad of loss partials
  float* hdr = upd_lds;             // [16] broadcast words
  float* W = upd_lds + 16;          // [Lp]
  float* Ga = W + Lp;               // [Lp + 4]
  float* scratch = Ga + Lp + 4;     // activations / reduction scratch
  const UpdAct a = upd_carve(scratch, n);
  float* s_bcast = hdr;             // [0] clip coefficient, [1] loss
  float* s_ssq = hdr + 4;           // [4] per-wave sums of squares
  int* s_abort = reinterpret_cast<int*>(hdr + 8);
  float* pm = args.priv + (size_t)g * 2 * Lp;
  float* pv = pm + Lp;

  // ---- load parameters (LDS image) and this workgroup's private moments -----------------------
  for (int k = t; k < Lp; k += UPD_THREADS) {
    const int f = upd_flat_of(n, k);
    W[k] = f >= 0 ? args.params[f] : 0.0f;
    pm[k] = f >= 0 ? args.exp_avg[f] : 0.0f;   // thread-private entries (same k mapping below)
    pv[k] = f >= 0 ? args.exp_avg_sq[f] : 0.0f;
  }
  const float step0 = args.adam_step[0];
  __syncthreads();

  const int R = args.R;
  float loss_last = 0.f;
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
      upd_chunk(args, W, Ga, a, mb0 + (int64_t)g * R + c0, std::min(UPD_RC, myrows - c0), invB);
    float* mypart = args.part + (size_t)g * Qtot * 4;
    for (int q = t; q < Qtot; q += UPD_THREADS)
      st4_sc1(mypart + 4 * q, *reinterpret_cast<const float4*>(Ga + 4 * q));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      __hip_atomic_fetch_add(args.ctr + 0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_abort = upd_wait(args.ctr, 0, (unsigned)G * (unsigned)(s + 1)) ? 0 : 1;
    }
    __syncthreads();
    if (*s_abort) return;
    // ---- phase B: reduce slice [qlo, qhi) over the G partials (workgroup order) ---------------
    {
      const int qlo = (int)((int64_t)Qtot * g / G), qhi = (int)((int64_t)Qtot * (g + 1) / G);
      const int nq = qhi - qlo;
      float ssq = 0.f;
      if (nq > UPD_THREADS / 2) {
        // wide slices (few workgroups): each thread owns whole quads, partials summed in order
        for (int qi = t; qi < nq; qi += UPD_THREADS) {
          float4 acc = float4{0.f, 0.f, 0.f, 0.f};
          for (int gg = 0; gg < G; ++gg) {
            const float4 v = ld4_sc1(args.part + ((size_t)gg * Qtot + qlo + qi) * 4);
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
          }
          st4_sc1(args.red + (size_t)(qlo + qi) * 4, acc);
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
          for (int gg = sub; gg < G; gg += spl) {
            const float4 v = ld4_sc1(args.part + ((size_t)gg * Qtot + qlo + qi) * 4);
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
          st4_sc1(args.red + (size_t)(qlo + t) * 4, acc);
          if (qlo + t < Qp) ssq = acc.x * acc.x + acc.y * acc.y + acc.z * acc.z + acc.w * acc.w;
        }
      }
      // block sum of ssq (threads < nq hold the pieces; fixed order)
      ssq = wave_sum(ssq);
      if ((t & 63) == 0) s_ssq[t >> 6] = ssq;
      __syncthreads();
      if (t == 0) {
        float tot = 0.f;
        for (int w = 0; w < UPD_THREADS / 64; ++w) tot += s_ssq[w];
        st_sc1f(args.sq + g, tot);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) {
        __hip_atomic_fetch_add(args.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *s_abort = upd_wait(args.ctr, 1, (unsigned)G * (unsigned)(s + 1)) ? 0 : 1;
      }
      __syncthreads();
      if (*s_abort) return;
    }
    // ---- phase C: clip_grad_norm_(2.0) + AdamW on every workgroup's own copy ------------------
    if (t == 0) {
      float tot = 0.f;
      for (int gg = 0; gg < G; ++gg) tot += ld_sc1f(args.sq + gg);
      const float norm = sqrtf(tot);
      const float coef = args.max_norm / (norm + 1e-6f);
      s_bcast[0] = coef < 1.0f ? coef : 1.0f;
      const float4 lp = ld4_sc1(args.red + (size_t)Qp * 4);
      s_bcast[1] = lp.x * invB + args.vf_coef * (lp.y * invB) - args.ent_coef * (lp.z * invB);
    }
    __syncthreads();
    const float clipc = s_bcast[0];
    loss_last = s_bcast[1];
    {
      const double tstep = (double)step0 + (double)(s + 1);
      const double bc1 = 1.0 - pow((double)args.beta1, tstep);
      const double bc2 = 1.0 - pow((double)args.beta2, tstep);
      const float step_size = (float)((double)args.lr / bc1);
      const float bc2_sqrt = (float)sqrt(bc2);
      const float decay = (float)(1.0 - (double)args.lr * (double)args.wd);
      const float b2 = args.beta2;
      const float omb1 = (float)(1.0 - (double)args.beta1), omb2 = (float)(1.0 - (double)args.beta2);
      for (int k = t; k < Lp; k += UPD_THREADS) {
        const float gr = ld_sc1f(args.red + k) * clipc;
        float m = pm[k], v = pv[k], p = W[k];
        p = p * decay;
        m = m + omb1 * (gr - m);
        v = v * b2 + omb2 * gr * gr;
        const float denom = sqrtf(v) / bc2_sqrt + args.eps;
        p = p - step_size * (m / denom);
        pm[k] = m;
        pv[k] = v;
        W[k] = p;
      }
    }
    __syncthreads();
  }
  // ---- write back (workgroup 0): parameters, moments, step count, last loss -------------------
  if (g == 0) {
    for (int k = t; k < Lp; k += UPD_THREADS) {
      const int f = upd_flat_of(n, k);
      if (f >= 0) {
        args.params[f] = W[k];
        args.exp_avg[f] = pm[k];
        args.exp_avg_sq[f] = pv[k];
      }
    }
    if (t == 0) {
      args.adam_step[0] = step0 + (float)args.total_steps;
      if (args.loss_out) args.loss_out[0] = loss_last;
    }
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

int upd_grid(int64_t mb) { return (int)std::min<int64_t>(256, cdiv(mb, UPD_RC)); }

size_t upd_lds_bytes(const UpdNet& n) {
  int DX, AX, OX;
  const int act = upd_act_floats(n.D, n.A, n.nout, DX, AX, OX);
  return sizeof(float) * (size_t)(16 + 2 * n.Lp + 4 + act);
}

struct UpdWs {
  unsigned* ctr;
  float* sq;
  float* red;
  float* part;
  float* priv;
};

// workspace: ctr[4] (16 B, zeroed per launch) | sq[256] | red[Qtot*4] | part[G][Qtot*4] | priv
size_t upd_ws_carve(const UpdNet& n, int G, char* base, UpdWs* ws) {
  const size_t Qtot = (size_t)n.Lp / 4 + 1;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
  const size_t o_ctr = take(16), o_sq = take(256 * 4), o_red = take(Qtot * 16),
               o_part = take((size_t)G * Qtot * 16), o_priv = take((size_t)G * 2 * n.Lp * 4);
  if (ws) {
    ws->ctr = reinterpret_cast<unsigned*>(base + o_ctr);
    ws->sq = reinterpret_cast<float*>(base + o_sq);
    ws->red = reinterpret_cast<float*>(base + o_red);
    ws->part = reinterpret_cast<float*>(base + o_part);
    ws->priv = reinterpret_cast<float*>(base + o_priv);
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
  return upd_lds_bytes(n) <= 160 * 1024 ? PRL_OK : PRL_ERR_ARG;
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
  args.priv = ws.priv;
  args.ctr = ws.ctr;
  const size_t lds = upd_lds_bytes(args.net);
  PRL_REQUIRE(lds <= 160 * 1024, "prl_ppo_update: %zu B of LDS needed", lds);
  hipStream_t st = as_stream(stream);
  PRL_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(ppo_update_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  PRL_HIP_TRY(hipMemsetAsync(ws.ctr, 0, 16, st));
  void* kargs[] = {&args};
  PRL_HIP_TRY(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(ppo_update_kernel), dim3(G),
                                     dim3(UPD_THREADS), kargs, (unsigned)lds, st));
  return PRL_OK;
}

// status word of the last launch on this workspace (device u32: 0 ok, 1 = in-kernel timeout)
extern "C" int prl_ppo_update_status_ptr(void* workspace, uint32_t** status) {
  PRL_REQUIRE(workspace && status, "prl_ppo_update_status_ptr: null pointer");
  *status = reinterpret_cast<uint32_t*>(workspace) + 3;
  return PRL_OK;
}
