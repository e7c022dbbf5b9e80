// prl_ppo_wide.hip — one optimizer step's gradient for the wide nets the persistent engine cannot
// hold (observation dim D up to 352, up to 48 head outputs: C5's D = 348 synthetic Humanoid with
// A = 17, i.e. mu 17 + log_std 17 + critic 1).  Forward (ActorCritic.get_evaluate,
// PPO/ActorCritic.py:118-146) -> clipped surrogate + 0.5 SmoothL1 (PPO/PPO.py:225-245; entropy
// detached) -> backward of the whole net for the minibatch of `cursor`, in ONE kernel, then a
// deterministic fold of the per-workgroup partial gradients (second kernel).  clip_grad_norm_ and
// AdamW stay torch's (capturable, fused) on the flat gradient, as in the graphed per-step path.
//
// Why its own kernel: the persistent engine keeps the parameters AND the gradient image in one
// CU's LDS (~2 x 150 KB for C5: does not fit), and C5's per-step graph was ~60 kernels, 1.3 ms per
// 65,536-row step.  Here the minibatch is wide (65,536 rows = 4,096 16-row tiles), so there is no
// hand-off inside the step: workgroup g walks tiles g, g + G, ... and accumulates ITS gradient in
// registers (MFMA accumulators), writes it once to part[g], and a second kernel sums part[0..G)
// in workgroup order.
//
// Per workgroup (256 threads = 4 waves, one per SIMD; wave w owns channel block w = channels
// 16w .. 16w+15 of every 64-wide layer; activations live in v_mfma_f32_16x16x4_f32 C fragments,
// lane (x = l & 15, q = l >> 4) register i = [row x][channel 16w + 4q + i]):
//   registers: W0 block w as A fragments (KSM k-steps, read once), dW0 block w (KSM / 4 16-column
//              accumulators), dW1 / dW2 blocks, GroupNorm gamma / beta gradient quads;
//   LDS:       the heads' parameters (W1, GN, W2, b2, trunk GN), the tile's inputs (double
//              buffered: the next tile stages while a slower wave still reads this one's), trunk
//              output F, head outputs G, the outputs O / dO, head dZ, per-wave transpose slots.
// Per 16-row tile, 5 workgroup barriers: stage X | trunk fwd -> F | heads fwd -> G | output layer
// -> O | row loss -> dO | heads bwd (dW2, dZ) | dW1, dF, trunk GN bwd, dW0.
#include "prl_common.h"

#include <float.h>

#include <algorithm>

#include <stdlib.h>

namespace prl {
namespace {

constexpr int WD_THREADS = 256;
constexpr int WD_H = 64;
constexpr int WD_HS = 68;      // LDS row stride of the [*][64] weight matrices
constexpr int WD_RT = 16;      // rows per tile
constexpr int WD_MAXH = 3;
constexpr int WD_MAXO = 48;    // outputs of all heads (three 16-row output tiles)
constexpr int WD_MAXHO = 32;   // outputs of one head (two 16-row tiles)
constexpr int WD_MAXA = 32;
constexpr int WD_FS = 80;      // row stride of F and dZ tiles [16][64]
constexpr int WD_GS = 196;     // row stride of the head outputs [16][3 * 64] (== 4 mod 64)
constexpr int WD_OS = 52;      // row stride of O / dO [16][48]
constexpr int WD_RS = 36;      // row-input record: act[32], old_logp, adv, ret, pad
constexpr int WD_GRID_MAX = 256;

struct WdNet {
  int D, A, nh, discrete, nout, P, Pq;      // Pq: P rounded up to 4 (loss slots at Pq .. Pq+2)
  int out[WD_MAXH], ocol[WD_MAXH];
  // flat offsets (torch parameters() order: model.0.weight, model.1.{weight,bias}, then every
  // head's 0.weight, 1.weight, 1.bias, 3.weight, 3.bias)
  int w0, g0, b0, w1[WD_MAXH], g1[WD_MAXH], b1[WD_MAXH], w2[WD_MAXH], b2[WD_MAXH];
  // LDS offsets of the head parameter image (floats)
  int Lg0, Lb0, Lw1[WD_MAXH], Lg1[WD_MAXH], Lb1[WD_MAXH], Lw2[WD_MAXH], Lb2[WD_MAXH], Lp;
};

__host__ __device__ constexpr bool wd_layout(int D, int A, int discrete, WdNet& n) {
  n = WdNet{};
  if (D < 1 || A < 1 || A > WD_MAXA) return false;
  n.D = D;
  n.A = A;
  n.discrete = discrete ? 1 : 0;
  n.nh = discrete ? 2 : 3;
  int flat = 0, lds = 0;
  auto lds_add = [&](int floats) {
    const int o = lds;
    lds += (floats + 3) & ~3;
    return o;
  };
  n.w0 = flat; flat += WD_H * D;
  n.g0 = flat; flat += WD_H;
  n.b0 = flat; flat += WD_H;
  n.Lg0 = lds_add(WD_H);
  n.Lb0 = lds_add(WD_H);
  int col = 0;
  for (int h = 0; h < n.nh; ++h) {
    const int out = (h == n.nh - 1) ? 1 : A;
    if (out > WD_MAXHO) return false;
    n.out[h] = out;
    n.ocol[h] = col;
    col += out;
    n.w1[h] = flat; flat += WD_H * WD_H;
    n.g1[h] = flat; flat += WD_H;
    n.b1[h] = flat; flat += WD_H;
    n.w2[h] = flat; flat += out * WD_H;
    n.b2[h] = flat; flat += out;
    n.Lw1[h] = lds_add(WD_H * WD_HS);
    n.Lg1[h] = lds_add(WD_H);
    n.Lb1[h] = lds_add(WD_H);
    n.Lw2[h] = lds_add(out * WD_HS);
    n.Lb2[h] = lds_add(out);
  }
  n.nout = col;
  if (n.nout > WD_MAXO) return false;
  n.P = flat;
  n.Pq = (flat + 3) & ~3;
  n.Lp = lds;
  return true;
}
__host__ __device__ constexpr WdNet wd_make(int D, int A, int discrete) {
  WdNet n{};
  wd_layout(D, A, discrete, n);
  return n;
}
// the specialised shape: C5's Humanoid-shaped net (D 348, A 17, continuous): its whole layout a
// compile-time constant (every LDS / flat offset an immediate, no net struct in SGPRs)
constexpr int WD_C5_D = 348, WD_C5_A = 17;

// tile scratch after the parameter image (floats)
__host__ __device__ inline int wd_xs(int KSM) { return 4 * KSM + 4; }   // X row stride (== 4 mod 32)
__host__ __device__ inline int wd_scratch_floats(int KSM) {
  return 2 * WD_RT * wd_xs(KSM)      // Xs  [2][16][XS]   tile inputs (double-buffered)
         + 2 * WD_RT * WD_RS         // Rin [2][16][36]   row inputs (double-buffered)
         + WD_RT * WD_FS             // Fs  [16][80]      trunk output
         + WD_RT * WD_GS             // Gs  [16][196]     head outputs (3 x 64 channels)
         + 2 * WD_RT * WD_OS         // Os, dOs [16][52]  outputs, d loss / d outputs
         + WD_MAXH * WD_RT * WD_FS   // Zs  [3][16][80]   head dZ
         + 4 * WD_RT * 16            // Tw  [4][16][16]   per-wave dH0 transpose slot
         + 8 * WD_H;                 // Gn  [8][64]       GroupNorm gamma / beta gradients
}
inline size_t wd_lds_bytes(const WdNet& n, int KSM) {
  return sizeof(float) * (size_t)(n.Lp + wd_scratch_floats(KSM));
}

struct WdArgs {
  WdNet net;
  const float* params;     // flat, torch parameters() order
  const float* S;          // [N][D]
  const float* act;        // [N][Aw]
  const float* old_logp;   // [N]
  const float* adv;        // [N]
  const float* ret;        // [N]
  const int64_t* cursor;   // device: minibatch index j (rows j*mb .. min((j+1)*mb, N))
  const float* scales;     // device [nb] loss scale per minibatch (data-parallel ranks) or null
  int64_t N, mb;
  float clip, vf_coef;
  float* part;             // [G][Pq + 4]
  int G;
  unsigned long long* prof;   // [8] workgroup 0's s_memrealtime ticks per tile stage (or null)
  float* dh0;              // split form: [mb][64] trunk pre-activation gradients (dW0 kernel input)
  float* eval_logp;        // evaluate form: [N] log-prob and state value per row
  float* eval_V;
  float* dist_out;         // distribution form: [N][A] probs or [N][2A] mu | std per row
};

typedef float wd_v4 __attribute__((ext_vector_type(4)));
__device__ inline wd_v4 wd_mma(float a, float b, wd_v4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ inline wd_v4 wd_ld4(const float* p) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  return wd_v4{v.x, v.y, v.z, v.w};
}
__device__ inline void wd_st4(float* p, wd_v4 v) {
  *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
}
__device__ inline void wd_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ inline float wd_exp(float x) { return __expf(x); }
__device__ inline float wd_log(float x) { return __logf(x); }
__device__ inline float wd_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ inline float wd_sigmoid(float y) { return wd_rcp(1.0f + wd_exp(-y)); }
template <int CTRL>
__device__ inline float wd_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
// sum over the 16 lanes of a DPP row (the tile's 16 rows, for one channel quad)
__device__ inline float wd_rsum16(float v) {
  v += wd_dpp<0xB1>(v);
  v += wd_dpp<0x4E>(v);
  v += wd_dpp<0x141>(v);
  v += wd_dpp<0x140>(v);
  return v;
}
// v + the partner lane l ^ 16's v (the other 4 channels of the lane's GroupNorm group)
__device__ inline float wd_pair_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// GroupNorm(8 groups of 8, eps 1e-5) + SiLU on a C fragment (PPO/ActorCritic.py:19-22)
__device__ inline void wd_gn_fwd(wd_v4 z, wd_v4 gw, wd_v4 gb, wd_v4& xh, float& rstd, wd_v4& y) {
  const float s4 = (z[0] + z[1]) + (z[2] + z[3]);
  const float mean = wd_pair_sum(s4) * 0.125f;
  wd_v4 d;
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = z[i] - mean;
  const float q4 = (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
  rstd = __builtin_amdgcn_rsqf(wd_pair_sum(q4) * 0.125f + 1e-5f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xh[i] = d[i] * rstd;
    const float u = xh[i] * gw[i] + gb[i];
    y[i] = u * wd_sigmoid(u);
  }
}
__device__ inline wd_v4 wd_gn_bwd(wd_v4 go, wd_v4 xh, wd_v4 gw, wd_v4 gb, float rstd, wd_v4& dy) {
  wd_v4 dxh;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float u = xh[i] * gw[i] + gb[i];
    const float sg = wd_sigmoid(u);
    dy[i] = go[i] * (sg * (1.0f + u * (1.0f - sg)));
    dxh[i] = dy[i] * gw[i];
  }
  const float a4 = (dxh[0] + dxh[1]) + (dxh[2] + dxh[3]);
  const float b4 = (dxh[0] * xh[0] + dxh[1] * xh[1]) + (dxh[2] * xh[2] + dxh[3] * xh[3]);
  const float m1 = wd_pair_sum(a4) * 0.125f;
  const float m2 = wd_pair_sum(b4) * 0.125f;
  wd_v4 dx;
#pragma unroll
  for (int i = 0; i < 4; ++i) dx[i] = rstd * (dxh[i] - m1 - xh[i] * m2);
  return dx;
}

// head h's offsets, selected over compile-time indices (no dynamic indexing of the kernarg struct)
struct WdHead {
  int Lw1, Lg1, Lb1, Lw2, Lb2, oc, no;
};
__device__ inline WdHead wd_head(const WdNet& n, int h) {
  WdHead r{n.Lw1[0], n.Lg1[0], n.Lb1[0], n.Lw2[0], n.Lb2[0], n.ocol[0], n.out[0]};
#pragma unroll
  for (int k = 1; k < WD_MAXH; ++k)
    if (h == k) r = WdHead{n.Lw1[k], n.Lg1[k], n.Lb1[k], n.Lw2[k], n.Lb2[k], n.ocol[k], n.out[k]};
  return r;
}

// max over the 16 lanes of a DPP row
__device__ inline float wd_rmax16(float v) {
  v = fmaxf(v, wd_dpp<0xB1>(v));
  v = fmaxf(v, wd_dpp<0x4E>(v));
  v = fmaxf(v, wd_dpp<0x141>(v));
  v = fmaxf(v, wd_dpp<0x140>(v));
  return v;
}

// The tile's row losses on all 256 threads: row r = t >> 4 is one DPP row of 16 lanes, lane c
// takes the actions / classes k = c and c + 16 (A <= 32); per-row sums are DPP row sums, so every
// lane of a row holds the same bits.  Same arithmetic as upd_row_loss (prl_ppo_update.hip) up to
// the order of the per-action sums.  Writes dO[r][0 .. 48) and returns {-min(s1, s2), SmoothL1,
// H} of row r (every lane of the row).
__device__ inline void wd_tile_loss(const WdNet& n, const float* Os, const float* Rin, float* dOs,
                                    float invB, float clip, float vf_coef, float (&lp)[3],
                                    float& logp_row, float& v_row) {
  const int t = threadIdx.x, r = t >> 4, c = t & 15;
  const int A = n.A;
  const bool discrete = n.discrete != 0;
  const int vcol = discrete ? A : 2 * A;
  const float* O = Os + r * WD_OS;
  const float* rin = Rin + r * WD_RS;
  float* dO = dOs + r * WD_OS;
  dO[c] = 0.f;
  dO[c + 16] = 0.f;
  dO[c + 32] = 0.f;
  float logp, H;
  // per-lane state of its (up to) two actions
  float e0 = 0.f, e1 = 0.f, mx = 0.f, rs = 1.f, rS2 = 1.f, qa = 1.f;
  float sd0 = 1.f, sd1 = 1.f, dd0 = 0.f, dd1 = 0.f, ls0 = 0.f, ls1 = 0.f, lc0 = 0.f, lc1 = 0.f;
  const int k0 = c, k1 = c + 16;
  const bool ok0 = k0 < A, ok1 = k1 < A;
  int ai = 0;
  if (discrete) {
    const float o0 = ok0 ? O[k0] : -FLT_MAX, o1 = ok1 ? O[k1] : -FLT_MAX;
    mx = wd_rmax16(fmaxf(o0, o1));
    e0 = ok0 ? wd_exp(o0 - mx) : 0.f;
    e1 = ok1 ? wd_exp(o1 - mx) : 0.f;
    rs = wd_rcp(wd_rsum16(e0 + e1));
    const float p0 = e0 * rs, p1 = e1 * rs;
    rS2 = wd_rcp(wd_rsum16(p0 + p1));
    const float q0 = p0 * rS2, q1 = p1 * rS2;
    ai = (int)rin[0];
    const bool bad = ai < 0 || ai >= A;
    const float c0 = q0 < FLT_EPSILON ? FLT_EPSILON : (q0 > 1.0f - FLT_EPSILON ? 1.0f - FLT_EPSILON : q0);
    const float c1 = q1 < FLT_EPSILON ? FLT_EPSILON : (q1 > 1.0f - FLT_EPSILON ? 1.0f - FLT_EPSILON : q1);
    const float l0 = wd_log(c0), l1 = wd_log(c1);
    H = -wd_rsum16((ok0 ? l0 * q0 : 0.f) + (ok1 ? l1 * q1 : 0.f));
    const float la = wd_rsum16((k0 == ai ? l0 : 0.f) + (k1 == ai ? l1 : 0.f));
    qa = bad ? 1.f : wd_rsum16((k0 == ai ? q0 : 0.f) + (k1 == ai ? q1 : 0.f));
    logp = bad ? __builtin_nanf("") : la;
  } else {
    const float half_log_2pi = 0.91893853320467274f;
    float lpart = 0.f, hpart = 0.f;
    if (ok0) {
      const float lsr = O[A + k0];
      lc0 = lsr;
      const float lsc = lsr < -2.0f ? -2.0f : (lsr > 2.0f ? 2.0f : lsr);
      ls0 = lsc;
      sd0 = wd_log(1.0f + wd_exp(lsc));
      dd0 = rin[k0] - O[k0];
      const float lsd = wd_log(sd0);
      lpart += -(dd0 * dd0) * wd_rcp(2.0f * (sd0 * sd0)) - lsd - half_log_2pi;
      hpart += 0.5f + half_log_2pi + lsd;
    }
    if (ok1) {
      const float lsr = O[A + k1];
      lc1 = lsr;
      const float lsc = lsr < -2.0f ? -2.0f : (lsr > 2.0f ? 2.0f : lsr);
      ls1 = lsc;
      sd1 = wd_log(1.0f + wd_exp(lsc));
      dd1 = rin[k1] - O[k1];
      const float lsd = wd_log(sd1);
      lpart += -(dd1 * dd1) * wd_rcp(2.0f * (sd1 * sd1)) - lsd - half_log_2pi;
      hpart += 0.5f + half_log_2pi + lsd;
    }
    logp = wd_rsum16(lpart);
    H = wd_rsum16(hpart);
  }
  const float V = O[vcol];
  logp_row = logp;
  v_row = V;
  const float diff = logp - rin[32];
  const float cl = diff < -20.0f ? -20.0f : (diff > 20.0f ? 20.0f : diff);
  const float ratio = wd_exp(cl);
  const float adv = rin[33];
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
  const float x = V - rin[34];
  const float ax = fabsf(x);
  const float sl = ax < 1.0f ? 0.5f * ax * ax : ax - 0.5f;
  const float gx = ax < 1.0f ? x : (x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f));
  lp[0] = -m;
  lp[1] = sl;
  lp[2] = H;
  if (c == 0) dO[vcol] = vf_coef * invB * gx;
  if (discrete) {
    const float mk = (qa >= FLT_EPSILON && qa <= 1.0f - FLT_EPSILON) ? 1.0f : 0.0f;
    const float gq = (logp != logp) ? logp : dlogp * mk;
    const float rqa = wd_rcp(qa);
    const float p0 = e0 * rs, p1 = e1 * rs;
    const float dp0 = ok0 ? gq * (((k0 == ai) ? rqa : 0.0f) - 1.0f) * rS2 : 0.f;
    const float dp1 = ok1 ? gq * (((k1 == ai) ? rqa : 0.0f) - 1.0f) * rS2 : 0.f;
    const float dot = wd_rsum16(p0 * dp0 + p1 * dp1);
    if (ok0) dO[k0] = p0 * (dp0 - dot);
    if (ok1) dO[k1] = p1 * (dp1 - dot);
  } else {
    if (ok0) {
      const float var = sd0 * sd0, rvar = wd_rcp(var), rsd = wd_rcp(sd0);
      dO[k0] = dlogp * (dd0 * rvar);
      const float dsd = dlogp * ((dd0 * dd0) * (rvar * rsd) - rsd);
      const float pass = (lc0 >= -2.0f && lc0 <= 2.0f) ? 1.0f : 0.0f;
      dO[A + k0] = dsd * wd_sigmoid(ls0) * pass;
    }
    if (ok1) {
      const float var = sd1 * sd1, rvar = wd_rcp(var), rsd = wd_rcp(sd1);
      dO[k1] = dlogp * (dd1 * rvar);
      const float dsd = dlogp * ((dd1 * dd1) * (rvar * rsd) - rsd);
      const float pass = (lc1 >= -2.0f && lc1 <= 2.0f) ? 1.0f : 0.0f;
      dO[A + k1] = dsd * wd_sigmoid(ls1) * pass;
    }
  }
}

// The distribution form's row output (ActorCritic.dist_params, the rollout's sampling input):
// row r = t >> 4 on its DPP row of 16 lanes, lane c taking outputs k = c and c + 16: discrete
// softmax probabilities (max-shifted exp, DPP row sums), continuous [mu | softplus(clamp(log_std,
// -2, 2))].  Rows >= rc are not written.
__device__ inline void wd_tile_dist(const WdNet& n, const float* Os, float* out, int64_t row0, int rc) {
  const int t = threadIdx.x, r = t >> 4, c = t & 15;
  const int A = n.A;
  const int k0 = c, k1 = c + 16;
  const bool ok0 = k0 < A, ok1 = k1 < A;
  const float* O = Os + r * WD_OS;
  if (n.discrete) {
    const float o0 = ok0 ? O[k0] : -FLT_MAX, o1 = ok1 ? O[k1] : -FLT_MAX;
    const float mx = wd_rmax16(fmaxf(o0, o1));
    const float e0 = ok0 ? wd_exp(o0 - mx) : 0.f, e1 = ok1 ? wd_exp(o1 - mx) : 0.f;
    const float rs = wd_rcp(wd_rsum16(e0 + e1));
    if (r < rc) {
      float* o = out + (row0 + r) * A;
      if (ok0) o[k0] = e0 * rs;
      if (ok1) o[k1] = e1 * rs;
    }
  } else if (r < rc) {
    float* o = out + (row0 + r) * 2 * A;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = u ? k1 : k0;
      if (u ? ok1 : ok0) {
        const float lsr = O[A + k];
        const float lsc = lsr < -2.0f ? -2.0f : (lsr > 2.0f ? 2.0f : lsr);
        o[k] = O[k];
        o[A + k] = wd_log(1.0f + wd_exp(lsc));
      }
    }
  }
}

// Next-tile prefetch (D % 4 == 0, 16-B aligned S; the X buffers then have row stride D): the X
// tile — 16 consecutive rows of S, one contiguous block — is copied global -> LDS by 16-B
// global_load_lds (no VGPR destination; a wave-instruction writes 1 KiB contiguously), issued
// by one wave after the heads' forward and drained at the barrier after the loss; the row
// records go through 3 registers (loaded at the same point by every wave).
__device__ inline void wd_glds_x(const WdNet& n, const WdArgs& a, int64_t row0, int rc, float* Xs) {
  const int t = threadIdx.x, l = t & 63;
  const int tot = WD_RT * n.D, have = rc * n.D;
  const float* src = a.S + row0 * n.D;
  const int nchunk = (tot + 255) >> 8;   // 256-float chunks, one wave-instruction each
  for (int c = 0; c < nchunk; ++c) {     // one wave issues them all (the caller's)
    const int f = (c << 8) + 4 * l;
    const int fs = f < have ? f : 0;     // past the minibatch's rows / the tile: any valid row
    // inline asm, not __builtin_amdgcn_global_load_lds: the compiler puts an s_waitcnt vmcnt(0)
    // in front of the next LDS read after the builtin (the copy writes LDS it cannot tell apart),
    // which exposed the whole copy wherever it was issued; the explicit wait before the barrier
    // after the loss is the only one it needs (no instruction reads the other X buffer before)
    const unsigned m = __builtin_amdgcn_readfirstlane(
        (unsigned)reinterpret_cast<uintptr_t>(Xs + (c << 8)));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // m0: nothing else in these kernels uses it
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(src + fs), "s"(m) : "memory", "m0");
#pragma clang diagnostic pop
  }
}
// The row records' slots a thread loads: slot i (e = t + 256 i) is row r, column k of the
// [16][36] record; its source column (act[k] / old_logp / adv / ret) depends only on the thread,
// so it is resolved once per launch: base == nullptr for an empty slot.  (Loaded by one wave
// instead — 9 slots per lane — the outputs stage waited for that wave: 268 vs 253 us per step.)
struct WdRinSlots {
  const float* base[3];
  int stride[3], r[3];
};
__device__ inline WdRinSlots wd_rin_slots(const WdNet& n, const WdArgs& a) {
  const int t = threadIdx.x;
  const int Aw = n.discrete ? 1 : n.A;
  WdRinSlots sl;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int e = t + WD_THREADS * i;
    const int r = e / WD_RS, k = e - r * WD_RS;
    const float* b = nullptr;
    int st = 1;
    if (e < WD_RT * WD_RS) {
      if (k < WD_MAXA) { b = (k < Aw && a.act) ? a.act + k : nullptr; st = Aw; }
      else if (a.old_logp == nullptr) b = nullptr;   // evaluate / distribution forms
      else if (k == 32) b = a.old_logp;
      else if (k == 33) b = a.adv;
      else if (k == 34) b = a.ret;
    }
    sl.base[i] = b;
    sl.stride[i] = st;
    sl.r[i] = r;
  }
  return sl;
}
// pr[i] = the raw loaded words; bit i of *ok says whether slot i is real (else 0 is stored): the
// select happens where pr is stored, so nothing waits for the loads before then.  One load per
// slot from a selected address (a valid dummy when the slot is empty): no branches, so no
// write-after-write wait on the destination between divergent paths.
__device__ inline void wd_rin_load(const WdRinSlots& sl, const WdArgs& a, int64_t row0, int rc,
                                   float (&pr)[3], unsigned* ok) {
  unsigned m = 0u;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const bool real = sl.base[i] != nullptr && sl.r[i] < rc;
    pr[i] = *(real ? sl.base[i] + (row0 + sl.r[i]) * sl.stride[i] : a.S);
    m |= real ? 1u << i : 0u;
  }
  *ok = m;
}

// Stage tile rows [row0, row0 + rc) of S into Xs (rows >= rc and columns >= D stay / become 0)
// and the row records into Rin.
__device__ inline void wd_stage(const WdNet& n, const WdArgs& a, int64_t row0, int rc, int XS,
                                float* Xs, float* Rin) {
  const int t = threadIdx.x, D = n.D;
  const float* src = a.S + row0 * D;
  const int tot = WD_RT * D, have = rc * D;
  if ((D & 3) == 0 && ((reinterpret_cast<uintptr_t>(a.S) & 15u) == 0)) {
    for (int f = 4 * t; f < tot; f += 4 * WD_THREADS) {
      const int r = f / D, d = f - r * D;
      const float4 v = f < have ? *reinterpret_cast<const float4*>(src + f) : float4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<float4*>(Xs + r * XS + d) = v;
    }
  } else {
    for (int f = t; f < tot; f += WD_THREADS) {
      const int r = f / D, d = f - r * D;
      Xs[r * XS + d] = f < have ? src[f] : 0.f;
    }
  }
  const int Aw = n.discrete ? 1 : n.A;
  for (int e = t; e < WD_RT * WD_RS; e += WD_THREADS) {
    const int r = e / WD_RS, k = e - r * WD_RS;
    float v = 0.f;
    if (r < rc) {
      const int64_t row = row0 + r;
      if (k < WD_MAXA) v = (k < Aw && a.act) ? a.act[row * Aw + k] : 0.f;
      else if (a.old_logp == nullptr) v = 0.f;   // evaluate / distribution forms
      else if (k == 32) v = a.old_logp[row];
      else if (k == 33) v = a.adv[row];
      else if (k == 34) v = a.ret[row];
    }
    Rin[e] = v;
  }
}

// SPLIT: dW0 is left to ppo_wide_dw0_kernel (dH0 goes to HBM); the ~90 registers of its
// accumulators hold the W0 fragments instead, loaded once per workgroup.
// the X half of wd_stage (rows >= rc zero; columns >= D untouched)
__device__ inline void wd_stage_x(const WdNet& n, const WdArgs& a, int64_t row0, int rc, int XS,
                                  float* Xs) {
  const int t = threadIdx.x, D = n.D;
  const float* src = a.S + row0 * D;
  const int tot = WD_RT * D, have = rc * D;
  if ((D & 3) == 0 && ((reinterpret_cast<uintptr_t>(a.S) & 15u) == 0)) {
    for (int f = 4 * t; f < tot; f += 4 * WD_THREADS) {
      const int r = f / D, d = f - r * D;
      const float4 v = f < have ? *reinterpret_cast<const float4*>(src + f) : float4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<float4*>(Xs + r * XS + d) = v;
    }
  } else {
    for (int f = t; f < tot; f += WD_THREADS) {
      const int r = f / D, d = f - r * D;
      Xs[r * XS + d] = f < have ? src[f] : 0.f;
    }
  }
}

// EVAL: the evaluate form (prl_ppo_wide_evaluate): the same tile forward and row arithmetic over
// all N rows, writing each row's log-prob and value instead of a gradient — PPO.learn's
// policy_old pass for the rows the wide step then updates on, so the first minibatch's ratio is
// exactly 1 (as in the reference, where both come from one get_evaluate).
template <int KSM, bool SPLIT, bool EVAL, bool DIST = false>
__device__ __forceinline__ void ppo_wide_grad_body(const WdNet& n, const WdArgs& a) {
  static_assert(!DIST || EVAL, "the distribution form is an evaluate form");
  constexpr int KE = SPLIT ? 1 : KSM / 4;   // 16-column blocks of dW0
  extern __shared__ float4 wd_lds4[];
  float* lds = reinterpret_cast<float*>(wd_lds4);
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4, w = t >> 6;
  const int D = n.D, nh = n.nh;
  // X buffers: row stride D (unpadded, global_load_lds prefetch) when D % 4 == 0 and S is 16-B
  // aligned, else wd_xs(KSM) (zero pad columns, register staging)
  const bool pfv = (D & 3) == 0 && (reinterpret_cast<uintptr_t>(a.S) & 15u) == 0;
  const int XS = pfv ? D : wd_xs(KSM);
  constexpr int XBUF = WD_RT * (4 * KSM + 4);   // floats per X buffer (>= 16 D + 64 spill-over)
  float* W = lds;
  float* p = lds + n.Lp;
  float* Xs0 = p; p += 2 * XBUF;
  float* Rin0 = p; p += 2 * WD_RT * WD_RS;
  float* Fs = p; p += WD_RT * WD_FS;
  float* Gs = p; p += WD_RT * WD_GS;
  float* Os = p; p += WD_RT * WD_OS;
  float* dOs = p; p += WD_RT * WD_OS;
  float* Zs = p; p += WD_MAXH * WD_RT * WD_FS;
  float* Tw = p + w * WD_RT * 16;
  p += 4 * WD_RT * 16;
  // GroupNorm gradient accumulators: [2h] gamma_h, [2h + 1] beta_h (heads), [6] gamma_0, [7] beta_0;
  // entry 16w + 4q + i is owned by lane (x = 0, q) of wave w
  float* Gn = p;

  // ---- minibatch of this step
  // (distribution form: an optional device step index selects rows [j*mb, (j+1)*mb) of S, the
  // rollout's traj_obs[k] read in place; out rows are relative to row_lo)
  const int64_t j = DIST ? (a.cursor ? *a.cursor : 0) : EVAL ? 0 : *a.cursor;
  const int64_t row_lo = j * a.mb;
  const int64_t rows = row_lo < a.N ? (a.N - row_lo < a.mb ? a.N - row_lo : a.mb) : 0;
  const float invB = rows > 0 ? (a.scales ? a.scales[j] : 1.0f) / (float)rows : 0.f;
  const int ntile = (int)((rows + WD_RT - 1) / WD_RT);

  // ---- head parameters -> LDS (padding entries 0); both X buffers' pad columns -> 0
  for (int k = t; k < n.Lp; k += WD_THREADS) W[k] = 0.f;
  for (int k = t; k < 2 * XBUF; k += WD_THREADS) Xs0[k] = 0.f;
  for (int k = t; k < 8 * WD_H; k += WD_THREADS) Gn[k] = 0.f;
  __syncthreads();
  for (int k = t; k < WD_H; k += WD_THREADS) {
    W[n.Lg0 + k] = a.params[n.g0 + k];
    W[n.Lb0 + k] = a.params[n.b0 + k];
  }
#pragma unroll
  for (int h = 0; h < WD_MAXH; ++h) {
    if (h < nh) {
      const WdHead hi = wd_head(n, h);
      int fw1 = n.w1[0], fg1 = n.g1[0], fb1 = n.b1[0], fw2 = n.w2[0], fb2 = n.b2[0];
      if (h == 1) { fw1 = n.w1[1]; fg1 = n.g1[1]; fb1 = n.b1[1]; fw2 = n.w2[1]; fb2 = n.b2[1]; }
      if (h == 2) { fw1 = n.w1[2]; fg1 = n.g1[2]; fb1 = n.b1[2]; fw2 = n.w2[2]; fb2 = n.b2[2]; }
      for (int k = t; k < WD_H * WD_H; k += WD_THREADS)
        W[hi.Lw1 + (k >> 6) * WD_HS + (k & 63)] = a.params[fw1 + k];
      for (int k = t; k < WD_H; k += WD_THREADS) {
        W[hi.Lg1 + k] = a.params[fg1 + k];
        W[hi.Lb1 + k] = a.params[fb1 + k];
      }
      for (int k = t; k < hi.no * WD_H; k += WD_THREADS)
        W[hi.Lw2 + (k >> 6) * WD_HS + (k & 63)] = a.params[fw2 + k];
      for (int k = t; k < hi.no; k += WD_THREADS) W[hi.Lb2 + k] = a.params[fb2 + k];
    }
  }
  // trunk weight block w: rows 16w + x of W0, read per tile from L2 as 16-B A fragments (K order
  // permuted so a lane's four k-steps of a 16-column group are 4 consecutive columns: step
  // (sg, i) <-> column 16 sg + 4 q + i, the same permutation on the X side); registers hold the
  // dW0 accumulators instead
  const float* w0row = a.params + n.w0 + (int64_t)(16 * w + x) * D;
  const bool w0vec = (D & 3) == 0 && ((reinterpret_cast<uintptr_t>(a.params) & 15u) == 0);
  float4 w0v[SPLIT ? KSM / 4 : 1];
  if (SPLIT) {
#pragma unroll
    for (int sg = 0; sg < (SPLIT ? KSM / 4 : 1); ++sg) {
      const int d0 = 16 * sg + 4 * q;
      float4 wv;
      if (w0vec) {
        wv = d0 < D ? *reinterpret_cast<const float4*>(w0row + d0) : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        wv.x = d0 < D ? w0row[d0] : 0.f;
        wv.y = d0 + 1 < D ? w0row[d0 + 1] : 0.f;
        wv.z = d0 + 2 < D ? w0row[d0 + 2] : 0.f;
        wv.w = d0 + 3 < D ? w0row[d0 + 3] : 0.f;
      }
      w0v[sg] = wv;
    }
    // landed before the tile loop: the trunk's MFMAs then carry no vmcnt wait for them, which
    // would also wait out the stores / prefetches the loop leaves in flight
    __builtin_amdgcn_s_waitcnt(0);
  }
  // gradient accumulators
  wd_v4 gW0[KE];
  wd_v4 gW1[WD_MAXH][4];
  wd_v4 gW2[WD_MAXH][2];
  const wd_v4 z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < KE; ++e) gW0[e] = z4;
#pragma unroll
  for (int h = 0; h < WD_MAXH; ++h) {
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) gW1[h][bb] = z4;
    gW2[h][0] = z4;
    gW2[h][1] = z4;
  }
  double gbias = 0.0;                 // wave 3, lane l < nout: output bias l
  double lpacc[3] = {0.0, 0.0, 0.0};  // threads t % 16 == 0: loss terms of row t >> 4

  const bool timer = a.prof != nullptr && blockIdx.x == 0 && t == 0;
  unsigned long long tm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tl = timer ? __builtin_amdgcn_s_memrealtime() : 0ull;
#define WD_MARK(i)                                                     \
  if (timer) {                                                         \
    const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();  \
    tm[i] += now_ - tl;                                                \
    tl = now_;                                                         \
  }
  const WdRinSlots rin_slots = wd_rin_slots(n, a);
  int it = 0;
  for (int tile = blockIdx.x; tile < ntile; tile += a.G, ++it) {
    const int64_t row0 = row_lo + (int64_t)tile * WD_RT;
    const int rc = (int)(rows - (int64_t)tile * WD_RT < WD_RT ? rows - (int64_t)tile * WD_RT : WD_RT);
    float* Xs = Xs0 + (it & 1) * XBUF;
    float* Rin = Rin0 + (it & 1) * WD_RT * WD_RS;
    if (it == 0 || !pfv) wd_stage(n, a, row0, rc, XS, Xs, Rin);   // else prefetched last tile
    __syncthreads();   // #1: Xs, Rin (and, on the first tile, the parameter image)
    WD_MARK(0)

    // ---- trunk: H0^T block w = W0 block w X^T, GroupNorm + SiLU
    wd_v4 xh0, Fw;
    float r0;
    {
      wd_v4 acc[4] = {z4, z4, z4, z4};
#pragma unroll
      for (int sg = 0; sg < KSM / 4; ++sg) {
        const int d0 = 16 * sg + 4 * q;
        if (16 * sg < D) {
          float4 wv;
          if (SPLIT) {
            wv = w0v[SPLIT ? sg : 0];
          } else if (w0vec) {
            wv = d0 < D ? *reinterpret_cast<const float4*>(w0row + d0) : float4{0.f, 0.f, 0.f, 0.f};
          } else {
            wv.x = d0 < D ? w0row[d0] : 0.f;
            wv.y = d0 + 1 < D ? w0row[d0 + 1] : 0.f;
            wv.z = d0 + 2 < D ? w0row[d0 + 2] : 0.f;
            wv.w = d0 + 3 < D ? w0row[d0 + 3] : 0.f;
          }
          float4 xv = *reinterpret_cast<const float4*>(Xs + x * XS + d0);
          if (16 * sg + 16 > D) {
            // the last, partial column group (D % 16 != 0): with the unpadded row stride
            // (XS == D) columns >= D are the NEXT row's first columns.  Their weights are 0, but
            // 0 x NaN is NaN: a non-finite value there (a terminal env's unwritten observation
            // row in the rollout's distribution pass) leaked into this row's outputs.  Zero them.
            xv.x = d0 < D ? xv.x : 0.f;
            xv.y = d0 + 1 < D ? xv.y : 0.f;
            xv.z = d0 + 2 < D ? xv.z : 0.f;
            xv.w = d0 + 3 < D ? xv.w : 0.f;
          }
          acc[0] = wd_mma(wv.x, xv.x, acc[0]);
          acc[1] = wd_mma(wv.y, xv.y, acc[1]);
          acc[2] = wd_mma(wv.z, xv.z, acc[2]);
          acc[3] = wd_mma(wv.w, xv.w, acc[3]);
        }
      }
      wd_v4 z;
#pragma unroll
      for (int i = 0; i < 4; ++i) z[i] = (acc[0][i] + acc[1][i]) + (acc[2][i] + acc[3][i]);
      wd_gn_fwd(z, wd_ld4(W + n.Lg0 + 16 * w + 4 * q), wd_ld4(W + n.Lb0 + 16 * w + 4 * q), xh0, r0, Fw);
      wd_st4(Fs + x * WD_FS + 16 * w + 4 * q, Fw);
    }
    __syncthreads();   // #2: Fs
    WD_MARK(1)
    // ---- next tile's inputs go in flight after the heads' forward (the other X buffer was last
    //      read by the previous tile's trunk); issued before the loss, as in round 2, its first
    //      wait exposed the whole copy
    const int tile_n = tile + a.G;
    const bool has_next = pfv && tile_n < ntile;
    // ---- heads: Z_h^T block w = W1_h block w F^T, GroupNorm + SiLU -> G_h
    wd_v4 F[4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) F[bb] = wd_ld4(Fs + x * WD_FS + 16 * bb + 4 * q);
    wd_v4 xhh[WD_MAXH], Gh[WD_MAXH];
    float rh[WD_MAXH];
#pragma unroll
    for (int h = 0; h < WD_MAXH; ++h) {
      xhh[h] = z4;
      Gh[h] = z4;
      rh[h] = 0.f;
      if (h < nh) {
        const WdHead hi = wd_head(n, h);
        wd_v4 z = z4;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
          const wd_v4 wa = wd_ld4(W + hi.Lw1 + (16 * w + x) * WD_HS + 16 * bb + 4 * q);
          z = wd_mma(wa[0], F[bb][0], z);
          z = wd_mma(wa[1], F[bb][1], z);
          z = wd_mma(wa[2], F[bb][2], z);
          z = wd_mma(wa[3], F[bb][3], z);
        }
        wd_gn_fwd(z, wd_ld4(W + hi.Lg1 + 16 * w + 4 * q), wd_ld4(W + hi.Lb1 + 16 * w + 4 * q),
                  xhh[h], rh[h], Gh[h]);
        wd_st4(Gs + x * WD_GS + 64 * h + 16 * w + 4 * q, Gh[h]);
      }
    }
    __syncthreads();   // #3: Gs
    WD_MARK(2)
    // the next tile's X copy, issued by wave 3, which forms no outputs: a wave's LDS reads queue
    // behind its own in-flight LDS copies (issued by all four waves at the heads' start, the
    // copy's latency moved into the heads' forward), and here it lands under the outputs
    float pr[3];
    unsigned pr_ok = 0u;
    if (has_next) {
      const int64_t rn = rows - (int64_t)tile_n * WD_RT;
      const int rcn = (int)(rn < WD_RT ? rn : WD_RT);
      const int64_t r0n = row_lo + (int64_t)tile_n * WD_RT;
      if (w == 3) wd_glds_x(n, a, r0n, rcn, Xs0 + ((it + 1) & 1) * XBUF);
      wd_rin_load(rin_slots, a, r0n, rcn, pr, &pr_ok);
    }
    // ---- output layer: wave m < 3 forms outputs 16m .. 16m+15 of every row (K = each
    //      overlapping head's 64 channels): lane (x = row, q) reg i = O[row x][16m + 4q + i]
    if (w < 3 && 16 * w < n.nout) {
      const int jA = 16 * w + x;   // the A row this lane supplies
      wd_v4 o = z4;
#pragma unroll
      for (int h = 0; h < WD_MAXH; ++h) {
        if (h < nh) {
          const WdHead hi = wd_head(n, h);
          if (hi.oc < 16 * w + 16 && hi.oc + hi.no > 16 * w) {
            const bool mine = jA >= hi.oc && jA < hi.oc + hi.no;
            const float* wr = W + hi.Lw2 + (mine ? jA - hi.oc : 0) * WD_HS;
            const float* gr = Gs + x * WD_GS + 64 * h;
            // K order per step (sg, i): lane q <-> channel 16 sg + 4 q + i, so each operand is
            // one 16-B LDS read per four MFMAs (was a 4-B read per MFMA and operand)
#pragma unroll
            for (int sg = 0; sg < 4; ++sg) {
              const wd_v4 av = mine ? wd_ld4(wr + 16 * sg + 4 * q) : z4;
              const wd_v4 bv = wd_ld4(gr + 16 * sg + 4 * q);
#pragma unroll
              for (int i = 0; i < 4; ++i) o = wd_mma(av[i], bv[i], o);
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int jo = 16 * w + 4 * q + i;
        float bias = 0.f;
#pragma unroll
        for (int h = 0; h < WD_MAXH; ++h) {
          if (h < nh) {
            const WdHead hi = wd_head(n, h);
            if (jo >= hi.oc && jo < hi.oc + hi.no) bias = W[hi.Lb2 + jo - hi.oc];
          }
        }
        o[i] += bias;
      }
      wd_st4(Os + x * WD_OS + 16 * w + 4 * q, o);
    }
    __syncthreads();   // #4: Os
    WD_MARK(3)
    // ---- per-row loss and dO: row t >> 4, 16 lanes per row
    if (DIST) {
      wd_tile_dist(n, Os, a.dist_out, row0 - row_lo, rc);
    } else {
      float lp[3], logp_r, v_r;
      wd_tile_loss(n, Os, Rin, dOs, invB, a.clip, a.vf_coef, lp, logp_r, v_r);
      if (EVAL) {
        if ((t & 15) == 0 && (t >> 4) < rc) {
          a.eval_logp[row0 + (t >> 4)] = logp_r;
          a.eval_V[row0 + (t >> 4)] = v_r;
        }
      } else if ((t & 15) == 0 && (t >> 4) < rc) {
        lpacc[0] += (double)lp[0];
        lpacc[1] += (double)lp[1];
        lpacc[2] += (double)lp[2];
      }
      if ((t >> 4) >= rc) {   // rows past the minibatch: no gradient
        float* dOr = dOs + (t >> 4) * WD_OS;
        dOr[t & 15] = 0.f;
        dOr[(t & 15) + 16] = 0.f;
        dOr[(t & 15) + 32] = 0.f;
      }
    }
    if (has_next) {
      float* Rn = Rin0 + ((it + 1) & 1) * WD_RT * WD_RS;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (t + WD_THREADS * i < WD_RT * WD_RS) Rn[t + WD_THREADS * i] = (pr_ok >> i) & 1u ? pr[i] : 0.f;
      __builtin_amdgcn_s_waitcnt(0);   // the global_load_lds copies, before the barrier
    }
    __syncthreads();   // #5: dOs
    WD_MARK(4)
    if (EVAL) continue;
    // ---- heads backward (block w): dW2, dG -> GroupNorm bwd -> dZ (to Zs), dgamma / dbeta
#pragma unroll
    for (int h = 0; h < WD_MAXH; ++h) {
      if (h < nh) {
        const WdHead hi = wd_head(n, h);
        const int oc = hi.oc, no = hi.no;
        // dW2_h[16mt + 4q + i][16w + x] += sum_rows dO[row][oc + 16mt + x'] G_h[row][16w + x]
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          if (16 * mt < no) {
            const int jj = 16 * mt + x;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const int r = 4 * s + q;
              gW2[h][mt] = wd_mma(jj < no ? dOs[r * WD_OS + oc + jj] : 0.f,
                                  Gs[r * WD_GS + 64 * h + 16 * w + x], gW2[h][mt]);
            }
          }
        }
        // dG_h^T block w = W2_h^T dO_h^T (K = the head's outputs)
        wd_v4 dg = z4;
#pragma unroll
        for (int s = 0; s < WD_MAXHO / 4; ++s) {
          if (4 * s < no) {
            const int jj = 4 * s + q;
            const float av = jj < no ? W[hi.Lw2 + jj * WD_HS + 16 * w + x] : 0.f;
            const float bv = jj < no ? dOs[x * WD_OS + oc + jj] : 0.f;
            dg = wd_mma(av, bv, dg);
          }
        }
        wd_v4 dy;
        const wd_v4 dz = wd_gn_bwd(dg, xhh[h], wd_ld4(W + hi.Lg1 + 16 * w + 4 * q),
                                   wd_ld4(W + hi.Lb1 + 16 * w + 4 * q), rh[h], dy);
        wd_st4(Zs + h * WD_RT * WD_FS + x * WD_FS + 16 * w + 4 * q, dz);
        {
          wd_v4 sg, sb;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            sg[i] = wd_rsum16(dy[i] * xhh[h][i]);
            sb[i] = wd_rsum16(dy[i]);
          }
          if (x == 0) {
            float* pg = Gn + 2 * h * WD_H + 16 * w + 4 * q;
            wd_st4(pg, wd_ld4(pg) + sg);
            wd_st4(pg + WD_H, wd_ld4(pg + WD_H) + sb);
          }
        }
      }
    }
    if (w == 3 && l < n.nout) {   // output biases: f64 row sums (softmax dO cancel across rows)
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < WD_RT; ++r) s += (double)dOs[r * WD_OS + l];
      gbias += s;
    }
    __syncthreads();   // #6: Zs
    WD_MARK(5)
    // ---- dW1_h[16w + 4q + i][16bb + x] += sum_rows dZ_h[row][16w + ..] F[row][16bb + x]
#pragma unroll
    for (int h = 0; h < WD_MAXH; ++h) {
      if (h < nh) {
        const float* Zh = Zs + h * WD_RT * WD_FS;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int r = 4 * s + q;
          const float av = Zh[r * WD_FS + 16 * w + x];
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) gW1[h][bb] = wd_mma(av, Fs[r * WD_FS + 16 * bb + x], gW1[h][bb]);
        }
      }
    }
    // ---- dF^T block w = sum_h W1_h^T dZ_h^T (K permuted: step s, lane q <-> channel
    //      16 (s & 3) + 4 q + (s >> 2)), trunk GroupNorm backward -> dH0
    wd_v4 dF;
    {
      wd_v4 d0 = z4, d1 = z4;
#pragma unroll
      for (int h = 0; h < WD_MAXH; ++h) {
        if (h < nh) {
          const WdHead hi = wd_head(n, h);
          const float* Zh = Zs + h * WD_RT * WD_FS + x * WD_FS;
          const float* Wh = W + hi.Lw1 + 16 * w + x;
          // B operands: four 16-B reads up front (a lane's steps read 4 runs of 4 channels)
          wd_v4 zb[4];
#pragma unroll
          for (int sg = 0; sg < 4; ++sg) zb[sg] = wd_ld4(Zh + 16 * sg + 4 * q);
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            const int o = 16 * (s & 3) + 4 * q + (s >> 2);
            if (s & 1) d1 = wd_mma(Wh[o * WD_HS], zb[s & 3][s >> 2], d1);
            else d0 = wd_mma(Wh[o * WD_HS], zb[s & 3][s >> 2], d0);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) dF[i] = d0[i] + d1[i];
    }
    wd_v4 dy0;
    const wd_v4 dH0 = wd_gn_bwd(dF, xh0, wd_ld4(W + n.Lg0 + 16 * w + 4 * q),
                                wd_ld4(W + n.Lb0 + 16 * w + 4 * q), r0, dy0);
    {
      wd_v4 sg, sb;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sg[i] = wd_rsum16(dy0[i] * xh0[i]);
        sb[i] = wd_rsum16(dy0[i]);
      }
      if (x == 0) {
        float* pg = Gn + 6 * WD_H + 16 * w + 4 * q;
        wd_st4(pg, wd_ld4(pg) + sg);
        wd_st4(pg + WD_H, wd_ld4(pg + WD_H) + sb);
      }
    }
    // ---- dW0[16w + 4q + i][16e + x] += sum_rows dH0[row][ch] X[row][16e + x]
    WD_MARK(6)
    if (SPLIT) {
      if (x < rc) wd_st4(a.dh0 + (row0 - row_lo + x) * WD_H + 16 * w + 4 * q, dH0);
    } else {
    wd_st4(Tw + x * 16 + 4 * q, dH0);
    wd_wave_sync();
    {
      float ta[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) ta[s] = Tw[(4 * s + q) * 16 + x];
#pragma unroll
      for (int e = 0; e < KE; ++e) {
        if (16 * e < D) {
#pragma unroll
          for (int s = 0; s < 4; ++s) gW0[e] = wd_mma(ta[s], Xs[(4 * s + q) * XS + 16 * e + x], gW0[e]);
        }
      }
    }
    }
    wd_wave_sync();   // Tw is rewritten by the next tile only after its barriers; keep order
    WD_MARK(7)
  }
#undef WD_MARK
  if (EVAL) return;
  if (timer) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a.prof[i] += tm[i];
  }

  // ---- this workgroup's partial gradient -> part[g] (flat order; every entry written once)
  float* out = a.part + (int64_t)blockIdx.x * (n.Pq + 4);
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const int d = 16 * e + x;
    if (!SPLIT && d < D) {
#pragma unroll
      for (int i = 0; i < 4; ++i) out[n.w0 + (16 * w + 4 * q + i) * D + d] = gW0[e][i];
    }
  }
#pragma unroll
  for (int h = 0; h < WD_MAXH; ++h) {
    if (h < nh) {
      int fw1 = n.w1[0], fg1 = n.g1[0], fb1 = n.b1[0], fw2 = n.w2[0], no = n.out[0];
      if (h == 1) { fw1 = n.w1[1]; fg1 = n.g1[1]; fb1 = n.b1[1]; fw2 = n.w2[1]; no = n.out[1]; }
      if (h == 2) { fw1 = n.w1[2]; fg1 = n.g1[2]; fb1 = n.b1[2]; fw2 = n.w2[2]; no = n.out[2]; }
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int i = 0; i < 4; ++i) out[fw1 + (16 * w + 4 * q + i) * WD_H + 16 * bb + x] = gW1[h][bb][i];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int jj = 16 * mt + 4 * q + i;
          if (jj < no) out[fw2 + jj * WD_H + 16 * w + x] = gW2[h][mt][i];
        }
      if (x == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          out[fg1 + 16 * w + 4 * q + i] = Gn[2 * h * WD_H + 16 * w + 4 * q + i];
          out[fb1 + 16 * w + 4 * q + i] = Gn[(2 * h + 1) * WD_H + 16 * w + 4 * q + i];
        }
      }
    }
  }
  if (x == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out[n.g0 + 16 * w + 4 * q + i] = Gn[6 * WD_H + 16 * w + 4 * q + i];
      out[n.b0 + 16 * w + 4 * q + i] = Gn[7 * WD_H + 16 * w + 4 * q + i];
    }
  }
  if (w == 3 && l < n.nout) {
    int fb = n.b2[0] + l;
#pragma unroll
    for (int h = 1; h < WD_MAXH; ++h)
      if (h < nh && l >= n.ocol[h]) fb = (h == 1 ? n.b2[1] : n.b2[2]) + (l - n.ocol[h]);
    out[fb] = (float)gbias;
  }
  // loss terms: threads t % 16 == 0 hold their rows' sums (other lanes 0); 16-lane DPP row sums,
  // then the 4 rows of each wave and the 4 waves in a fixed order through LDS
  {
    __syncthreads();   // the tile scratch is free
    float* red = Zs;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float s = wd_rsum16((float)lpacc[k]);
      if ((t & 15) == 0) red[(t >> 4) * 4 + k] = s;
    }
    __syncthreads();
    if (t == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        float s = 0.f;
        for (int r = 0; r < WD_RT; ++r) s += red[r * 4 + k];
        out[n.Pq + k] = s;
      }
      out[n.Pq + 3] = 0.f;
    }
  }
}

// KSPEC: the C5 specialisation (constexpr layout); else the runtime layout from the argument
template <int KSM, bool SPLIT, bool EVAL = false, bool KSPEC = false, bool DIST = false>
__global__ __launch_bounds__(WD_THREADS, 1) void ppo_wide_grad_kernel(WdArgs a) {
  if constexpr (KSPEC) {
    constexpr WdNet N = wd_make(WD_C5_D, WD_C5_A, 0);
    ppo_wide_grad_body<KSM, SPLIT, EVAL, DIST>(N, a);
  } else {
    ppo_wide_grad_body<KSM, SPLIT, EVAL, DIST>(a.net, a);
  }
}

// Split form, second pass: dW0[c][d] = sum over the minibatch's rows of dH0[row][c] X[row][d]
// (K = rows).  Workgroup g takes 32-row tiles g, g + G2, ...; wave w owns channels 16w .. 16w+15
// (22 16 x 16 accumulators for D = 348).  The next tile's X and dH0 rows are loaded into
// registers while the current tile's MFMAs run (D % 4 == 0, 16-B aligned S; else staged in
// place), then written to LDS between two barriers.  Two workgroups per CU.  The partial goes to
// part2[g] ([64 D] + 4 pad, flat W0 order) for the same fold as the other gradients.
constexpr int WD2_GRID_MAX = 256;
constexpr int WD2_RT = 32;
template <int KSM>
__device__ __forceinline__ void ppo_wide_dw0_body(const WdNet& n, const WdArgs& a, float* part2, int G2) {
  constexpr int KE = KSM / 4;
  constexpr int XS2 = 4 * KSM + 4;
  constexpr int HS = 68;
  constexpr int NPF = (WD2_RT * 4 * KSM / 4 + WD_THREADS - 1) / WD_THREADS;   // float4 per thread
  __shared__ float Xs[WD2_RT * XS2];
  __shared__ float Hs[WD2_RT * HS];
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4, w = t >> 6;
  const int D = n.D;
  const int64_t j = *a.cursor;
  const int64_t row_lo = j * a.mb;
  const int64_t rows = row_lo < a.N ? (a.N - row_lo < a.mb ? a.N - row_lo : a.mb) : 0;
  const int ntile = (int)((rows + WD2_RT - 1) / WD2_RT);
  const bool vec = (D & 3) == 0 && (reinterpret_cast<uintptr_t>(a.S) & 15u) == 0;
  for (int k = t; k < WD2_RT * XS2; k += WD_THREADS) Xs[k] = 0.f;
  const wd_v4 z4 = {0.f, 0.f, 0.f, 0.f};
  wd_v4 acc[KE];
#pragma unroll
  for (int e = 0; e < KE; ++e) acc[e] = z4;
  float4 px[NPF];
  float4 ph[2];   // dH0: 32 rows x 64 = 512 float4, 2 per thread
  auto load = [&](int tile) {
    const int64_t r0 = (int64_t)tile * WD2_RT;   // relative to row_lo
    const int rc = (int)(rows - r0 < WD2_RT ? rows - r0 : WD2_RT);
    const float* src = a.S + (row_lo + r0) * D;
    const int have = rc * D;
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int f = 4 * (t + WD_THREADS * i);
      px[i] = f < have ? *reinterpret_cast<const float4*>(src + f) : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int f = 4 * (t + WD_THREADS * i);
      ph[i] = (f >> 6) < rc ? *reinterpret_cast<const float4*>(a.dh0 + r0 * WD_H + f)
                            : float4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store = [&]() {
    const int tot = WD2_RT * D;
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int f = 4 * (t + WD_THREADS * i);
      if (f < tot) {
        const int r = f / D, d = f - r * D;
        *reinterpret_cast<float4*>(Xs + r * XS2 + d) = px[i];
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int f = 4 * (t + WD_THREADS * i);
      *reinterpret_cast<float4*>(Hs + (f >> 6) * HS + (f & 63)) = ph[i];
    }
  };
  __syncthreads();
  if (vec && (int)blockIdx.x < ntile) load(blockIdx.x);
  for (int tile = blockIdx.x; tile < ntile; tile += G2) {
    if (vec) {
      store();
    } else {   // scalar staging in place
      const int64_t r0 = (int64_t)tile * WD2_RT;
      const int rc = (int)(rows - r0 < WD2_RT ? rows - r0 : WD2_RT);
      const float* src = a.S + (row_lo + r0) * D;
      for (int f = t; f < WD2_RT * D; f += WD_THREADS) {
        const int r = f / D, d = f - r * D;
        Xs[r * XS2 + d] = r < rc ? src[f] : 0.f;
      }
      for (int e = t; e < WD2_RT * WD_H; e += WD_THREADS)
        Hs[(e >> 6) * HS + (e & 63)] = (e >> 6) < rc ? a.dh0[r0 * WD_H + e] : 0.f;
    }
    __syncthreads();
    if (vec && tile + G2 < ntile) load(tile + G2);   // in flight under the MFMAs
#pragma unroll
    for (int kk = 0; kk < WD2_RT / 16; ++kk) {
      float ta[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) ta[s] = Hs[(16 * kk + 4 * s + q) * HS + 16 * w + x];
#pragma unroll
      for (int e = 0; e < KE; ++e) {
        if (16 * e < D) {
#pragma unroll
          for (int s = 0; s < 4; ++s)
            acc[e] = wd_mma(ta[s], Xs[(16 * kk + 4 * s + q) * XS2 + 16 * e + x], acc[e]);
        }
      }
    }
    __syncthreads();
  }
  float* out = part2 + (int64_t)blockIdx.x * (WD_H * D + 4);
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const int d = 16 * e + x;
    if (d < D) {
#pragma unroll
      for (int i = 0; i < 4; ++i) out[(16 * w + 4 * q + i) * D + d] = acc[e][i];
    }
  }
}

// grad[k] = sum_g part[g][k] (f64), k < P; loss = (L0 + vf L1 - ent L2) / B.  Block = 256 / S
// quads x S workgroup slots; slot s sums workgroups s, s + S, s + 2S, ... in that order, and the S
// slot sums are added in slot order (deterministic).  The standalone fold (dW0's 256 partials)
// runs S = 16: 4x the blocks of S = 4, 6.6 vs 8.4 us at C5; inside the dW0 launch the tile
// partials' fold keeps S = 4 (with S = 16 its extra blocks slowed dW0 by 1.1 us;
// profiles/r04_wide_fold_ab.md).
struct WrArgs {
  const float* part;
  int G, P, Pq;
  float* grad;
  float* loss_out;
  const int64_t* cursor;
  const float* scales;
  int64_t N, mb;
  float vf_coef, ent_coef;
  int q0;   // first quad folded (the split form: past W0's block, which dW0's own fold writes)
};
template <int S>
__device__ __forceinline__ void ppo_wide_reduce_body(const WrArgs& r, int blk) {
  constexpr int QU = 256 / S;
  const float* __restrict__ part = r.part;
  const int G = r.G, P = r.P, Pq = r.Pq;
  float* __restrict__ grad = r.grad;
  __shared__ double4 acc_s[S][QU];
  const int t = threadIdx.x, slot = t / QU, qi = t % QU;
  const int quad = r.q0 + blk * QU + qi;
  const int stride = Pq + 4;
  const int nq = stride / 4;
  double4 acc = {0.0, 0.0, 0.0, 0.0};
  if (quad < nq) {
    const float4* src = reinterpret_cast<const float4*>(part) + quad;
    int g = slot;
    for (; g + 3 * S < G; g += 4 * S) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = src[(int64_t)(g + S * u) * nq];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += v[u].x;
        acc.y += v[u].y;
        acc.z += v[u].z;
        acc.w += v[u].w;
      }
    }
    for (; g < G; g += S) {
      const float4 v = src[(int64_t)g * nq];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  acc_s[slot][qi] = acc;
  __syncthreads();
  if (slot == 0 && quad < nq) {
    double4 s = acc_s[0][qi];
#pragma unroll
    for (int k = 1; k < S; ++k) {
      const double4 o = acc_s[k][qi];
      s.x += o.x;
      s.y += o.y;
      s.z += o.z;
      s.w += o.w;
    }
    const int k0 = 4 * quad;
    if (k0 < P) {
      grad[k0] = (float)s.x;
      if (k0 + 1 < P) grad[k0 + 1] = (float)s.y;
      if (k0 + 2 < P) grad[k0 + 2] = (float)s.z;
      if (k0 + 3 < P) grad[k0 + 3] = (float)s.w;
    } else if (k0 == Pq && r.loss_out) {
      const int64_t j = *r.cursor;
      const int64_t lo = j * r.mb;
      const int64_t rows = lo < r.N ? (r.N - lo < r.mb ? r.N - lo : r.mb) : 0;
      const float inv = rows > 0 ? (r.scales ? r.scales[j] : 1.0f) / (float)rows : 0.f;
      r.loss_out[0] = (float)s.x * inv + r.vf_coef * ((float)s.y * inv) - r.ent_coef * ((float)s.z * inv);
    }
  }
}
template <int S>
int wr_blocks(int nq) { return (int)cdiv(nq, 256 / S); }
template <int S>
__global__ __launch_bounds__(256) void ppo_wide_reduce_kernel(WrArgs r) { ppo_wide_reduce_body<S>(r, blockIdx.x); }

// dW0 (workgroups 0 .. G2-1) and, in the same launch, the fold of the tile kernel's partials
// into every other gradient (workgroups G2 ..: ppo_wide_reduce_body): the two read disjoint
// buffers, and the fold's ~38 MB stream at C5's minibatch ran alone behind the tile kernel
// before (9 us per step), while dW0 streams X at ~35 % of HBM.
template <int KSM, bool KSPEC = false, int S = 4>
__global__ __launch_bounds__(WD_THREADS, 2) void ppo_wide_dw0_kernel(WdArgs a, float* part2, int G2,
                                                                    WrArgs r) {
  static_assert(WD_THREADS == 256, "the fold body runs 256-thread workgroups");
  if ((int)blockIdx.x >= G2) {
    ppo_wide_reduce_body<S>(r, (int)blockIdx.x - G2);
    return;
  }
  if constexpr (KSPEC) {
    constexpr WdNet N = wd_make(WD_C5_D, WD_C5_A, 0);
    ppo_wide_dw0_body<KSM>(N, a, part2, G2);
  } else {
    ppo_wide_dw0_body<KSM>(a.net, a, part2, G2);
  }
}

// KSM instantiated for D <= 128 and D <= 352
int wd_ksm(int D) { return D <= 128 ? 32 : (D <= 352 ? 88 : 0); }
// the constexpr-layout kernel runs this shape (PRL_WIDE_SPEC=0: the runtime-layout kernel, A/B)
bool wd_spec(const WdNet& n) {
  static const bool on = [] {
    const char* e = getenv("PRL_WIDE_SPEC");
    return !(e && e[0] == '0');
  }();
  return on && n.D == WD_C5_D && n.A == WD_C5_A && !n.discrete;
}

int wd_grid(int64_t mb);
int wd_grid2(int64_t mb) {
  const int64_t tiles = (mb + WD2_RT - 1) / WD2_RT;
  // PRL_WIDE_G2 (A/B): cap on dW0's workgroups (its partials, 89 KB each at C5, are folded after it)
  static const int cap = [] {
    const char* e = getenv("PRL_WIDE_G2");
    const int v = e ? atoi(e) : WD2_GRID_MAX;
    return v >= 1 && v <= WD2_GRID_MAX ? v : WD2_GRID_MAX;
  }();
  return (int)std::max<int64_t>(1, std::min<int64_t>(tiles, cap));
}
bool wd_split() {
  static const int v = [] {
    const char* e = getenv("PRL_WIDE_SPLIT");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v != 0;
}
// part layout: [G][Pq + 4] kernel-1 partials | dH0 [mb][64] | [G2][64 D + 4] dW0 partials
int64_t wd_part_floats(const WdNet& n, int64_t mb) {
  return (int64_t)wd_grid(mb) * (n.Pq + 4) + mb * WD_H + (int64_t)wd_grid2(mb) * (WD_H * n.D + 4);
}

int wd_grid(int64_t mb) {
  const int64_t tiles = (mb + WD_RT - 1) / WD_RT;
  return (int)std::max<int64_t>(1, std::min<int64_t>(tiles, WD_GRID_MAX));
}

}  // namespace
}  // namespace prl

using namespace prl;

extern "C" int prl_ppo_wide_info(int32_t D, int32_t A, int32_t discrete, int64_t mini_batch,
                                 int64_t* n_params, int64_t* part_floats, int32_t* grid) {
  WdNet n;
  if (n_params) *n_params = 0;
  if (part_floats) *part_floats = 0;
  if (grid) *grid = 0;
  PRL_REQUIRE(mini_batch > 0, "prl_ppo_wide_info: mini_batch must be > 0");
  if (!wd_layout(D, A, discrete, n) || wd_ksm(D) == 0) return PRL_ERR_ARG;
  if (wd_lds_bytes(n, wd_ksm(D)) > 160 * 1024) return PRL_ERR_ARG;
  const int G = wd_grid(mini_batch);
  if (n_params) *n_params = n.P;
  if (part_floats) *part_floats = wd_part_floats(n, mini_batch);
  if (grid) *grid = G;
  return PRL_OK;
}

// ActorCritic.dist_params over N rows (the rollout's sampling input, AsyncPPO's vector step): the
// wide kernel's forward, then per row the softmax probabilities [N][A] (discrete) or
// [mu | softplus(clamp(log_std, -2, 2))] [N][2A] (continuous).  One launch; capturable.
static int wd_dist_launch(const float* params, int32_t D, int32_t A, int32_t discrete,
                          const float* S, int64_t N, int64_t rows, const int64_t* step,
                          float* out, void* stream) {
  WdNet n;
  PRL_REQUIRE(N >= 0 && rows >= 0, "prl_ppo_wide_dist: N < 0 or rows < 0");
  PRL_REQUIRE(wd_layout(D, A, discrete, n) && wd_ksm(D) > 0,
              "prl_ppo_wide_dist: shape D=%d A=%d outside the wide kernel", D, A);
  PRL_REQUIRE(params && S && out, "prl_ppo_wide_dist: null pointer");
  if (N == 0 || rows == 0) return PRL_OK;
  const int KSM = wd_ksm(D);
  const size_t lds = wd_lds_bytes(n, KSM);
  PRL_REQUIRE(lds <= 160 * 1024, "prl_ppo_wide_dist: LDS %zu bytes", lds);
  WdArgs a{};
  a.net = n;
  a.params = params;
  a.S = S;
  a.N = N;
  a.mb = rows;
  a.cursor = step;
  a.G = wd_grid(rows);
  a.dist_out = out;
  hipStream_t st = as_stream(stream);
  static unsigned long long lds_set[3] = {0ull, 0ull, 0ull};   // bit = device ordinal
  int dev_ord = 0;
  PRL_HIP_TRY(hipGetDevice(&dev_ord));
  const unsigned long long dev_bit = 1ull << (dev_ord & 63);
#define WD_DLAUNCH(K, SPEC, slot)                                                                 \
  do {                                                                                         \
    if (!(lds_set[slot] & dev_bit)) {                                                          \
      PRL_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&ppo_wide_grad_kernel<K, true, true, SPEC, true>), \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));   \
      lds_set[slot] |= dev_bit;                                                                \
    }                                                                                          \
    hipLaunchKernelGGL((ppo_wide_grad_kernel<K, true, true, SPEC, true>), dim3(a.G), dim3(WD_THREADS), lds, st, a); \
  } while (0)
  if (KSM == 32) WD_DLAUNCH(32, false, 0);
  else if (wd_spec(n)) WD_DLAUNCH(88, true, 2);
  else WD_DLAUNCH(88, false, 1);
#undef WD_DLAUNCH
  PRL_LAUNCH_CHECK("ppo_wide_dist");
  return PRL_OK;
}

extern "C" int prl_ppo_wide_dist(const float* params, int32_t D, int32_t A, int32_t discrete,
                                 const float* S, int64_t N, float* out, void* stream) {
  return wd_dist_launch(params, D, A, discrete, S, N, N, nullptr, out, stream);
}

// The rollout's graphed vector step: rows [k*rows, (k+1)*rows) of the trajectory's observation
// store S ([N][D], N = (T+1) * rows), k read from the device (step_dev[0]), so one captured graph
// serves every step without a per-step copy of traj_obs[k].  A k past the store gives no rows.
extern "C" int prl_ppo_wide_dist_at(const float* params, int32_t D, int32_t A, int32_t discrete,
                                    const float* S, int64_t N, int64_t rows,
                                    const int64_t* step_dev, float* out, void* stream) {
  PRL_REQUIRE(step_dev != nullptr, "prl_ppo_wide_dist_at: null step index");
  return wd_dist_launch(params, D, A, discrete, S, N, rows, step_dev, out, stream);
}

extern "C" int prl_ppo_wide_evaluate(const float* params, int32_t D, int32_t A, int32_t discrete,
                                     const float* S, const float* actions, int64_t N,
                                     float* logp_out, float* V_out, void* stream) {
  WdNet n;
  PRL_REQUIRE(N >= 0, "prl_ppo_wide_evaluate: N < 0");
  PRL_REQUIRE(wd_layout(D, A, discrete, n) && wd_ksm(D) > 0,
              "prl_ppo_wide_evaluate: shape D=%d A=%d outside the wide kernel", D, A);
  PRL_REQUIRE(params && S && actions && logp_out && V_out, "prl_ppo_wide_evaluate: null pointer");
  if (N == 0) return PRL_OK;
  const int KSM = wd_ksm(D);
  const size_t lds = wd_lds_bytes(n, KSM);
  PRL_REQUIRE(lds <= 160 * 1024, "prl_ppo_wide_evaluate: LDS %zu bytes", lds);
  WdArgs a{};
  a.net = n;
  a.params = params;
  a.S = S;
  a.act = actions;
  a.N = N;
  a.mb = N;
  a.G = wd_grid(N);
  a.eval_logp = logp_out;
  a.eval_V = V_out;
  hipStream_t st = as_stream(stream);
  static unsigned long long lds_set[3] = {0ull, 0ull, 0ull};   // bit = device ordinal
  int dev_ord = 0;
  PRL_HIP_TRY(hipGetDevice(&dev_ord));
  const unsigned long long dev_bit = 1ull << (dev_ord & 63);
#define WD_ELAUNCH(K, SPEC, slot)                                                                 \
  do {                                                                                         \
    if (!(lds_set[slot] & dev_bit)) {                                                          \
      PRL_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&ppo_wide_grad_kernel<K, true, true, SPEC>), \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));   \
      lds_set[slot] |= dev_bit;                                                                \
    }                                                                                          \
    hipLaunchKernelGGL((ppo_wide_grad_kernel<K, true, true, SPEC>), dim3(a.G), dim3(WD_THREADS), lds, st, a); \
  } while (0)
  if (KSM == 32) WD_ELAUNCH(32, false, 0);
  else if (wd_spec(n)) WD_ELAUNCH(88, true, 2);
  else WD_ELAUNCH(88, false, 1);
#undef WD_ELAUNCH
  PRL_LAUNCH_CHECK("ppo_wide_evaluate");
  return PRL_OK;
}

extern "C" int prl_ppo_wide_grad_prof(const float*, int32_t, int32_t, int32_t, const float*,
                                      const float*, const float*, const float*, const float*,
                                      int64_t, int64_t, const int64_t*, const float*, float, float,
                                      float, float*, float*, float*, int64_t, unsigned long long*,
                                      void*);

extern "C" int prl_ppo_wide_grad(const float* params, int32_t D, int32_t A, int32_t discrete,
                                 const float* S, const float* actions, const float* old_logp,
                                 const float* adv, const float* ret, int64_t N,
                                 int64_t mini_batch, const int64_t* cursor, const float* scales,
                                 float clip, float vf_coef, float ent_coef, float* grad,
                                 float* loss_out, float* part, int64_t part_floats, void* stream) {
  return prl_ppo_wide_grad_prof(params, D, A, discrete, S, actions, old_logp, adv, ret, N,
                                mini_batch, cursor, scales, clip, vf_coef, ent_coef, grad,
                                loss_out, part, part_floats, nullptr, stream);
}

// prl_ppo_wide_grad + workgroup 0's per-stage tick counters added into prof[8] (diagnostics:
// tools/wide_bench.py)
extern "C" int prl_ppo_wide_grad_prof(const float* params, int32_t D, int32_t A, int32_t discrete,
                                      const float* S, const float* actions, const float* old_logp,
                                      const float* adv, const float* ret, int64_t N,
                                      int64_t mini_batch, const int64_t* cursor,
                                      const float* scales, float clip, float vf_coef,
                                      float ent_coef, float* grad, float* loss_out, float* part,
                                      int64_t part_floats, unsigned long long* prof,
                                      void* stream) {
  WdNet n;
  PRL_REQUIRE(mini_batch > 0 && N >= 0, "prl_ppo_wide_grad: bad sizes");
  PRL_REQUIRE(wd_layout(D, A, discrete, n) && wd_ksm(D) > 0,
              "prl_ppo_wide_grad: shape D=%d A=%d outside the wide kernel", D, A);
  PRL_REQUIRE(params && S && actions && old_logp && adv && ret && cursor && grad && part,
              "prl_ppo_wide_grad: null pointer");
  const int G = wd_grid(mini_batch);
  PRL_REQUIRE(part_floats >= wd_part_floats(n, mini_batch), "prl_ppo_wide_grad: part buffer too small");
  const int KSM = wd_ksm(D);
  const size_t lds = wd_lds_bytes(n, KSM);
  PRL_REQUIRE(lds <= 160 * 1024, "prl_ppo_wide_grad: LDS %zu bytes", lds);
  WdArgs a{};
  a.net = n;
  a.params = params;
  a.S = S;
  a.act = actions;
  a.old_logp = old_logp;
  a.adv = adv;
  a.ret = ret;
  a.cursor = cursor;
  a.scales = scales;
  a.N = N;
  a.mb = mini_batch;
  a.clip = clip;
  a.vf_coef = vf_coef;
  a.part = part;
  a.G = G;
  a.prof = prof;
  const bool split = wd_split();
  a.dh0 = part + (int64_t)G * (n.Pq + 4);
  float* part2 = a.dh0 + mini_batch * WD_H;
  const int G2 = wd_grid2(mini_batch);
  hipStream_t st = as_stream(stream);
  // the kernels' dynamic-LDS limit is raised once per process AND device (the attribute is
  // per device; not a stream operation, but kept out of the per-step path that graphs capture)
  static unsigned long long lds_set[5] = {0ull, 0ull, 0ull, 0ull, 0ull};   // bit = device ordinal
  int dev_ord = 0;
  PRL_HIP_TRY(hipGetDevice(&dev_ord));
  const unsigned long long dev_bit = 1ull << (dev_ord & 63);
#define WD_LAUNCH(K, SP, SPEC, slot)                                                            \
  do {                                                                                       \
    if (!(lds_set[slot] & dev_bit)) {                                                        \
      PRL_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&ppo_wide_grad_kernel<K, SP, false, SPEC>), \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)); \
      lds_set[slot] |= dev_bit;                                                              \
    }                                                                                        \
    hipLaunchKernelGGL((ppo_wide_grad_kernel<K, SP, false, SPEC>), dim3(G), dim3(WD_THREADS), lds, st, a); \
  } while (0)
  if (KSM == 32) {
    if (split) WD_LAUNCH(32, true, false, 0); else WD_LAUNCH(32, false, false, 1);
  } else if (wd_spec(n) && split) {
    WD_LAUNCH(88, true, true, 4);
  } else {
    if (split) WD_LAUNCH(88, true, false, 2); else WD_LAUNCH(88, false, false, 3);
  }
#undef WD_LAUNCH
  PRL_LAUNCH_CHECK("ppo_wide_grad");
  const int nq = (n.Pq + 4) / 4;
  WrArgs fold{part, G, n.P, n.Pq, grad, loss_out, cursor, scales, N, mini_batch, vf_coef, ent_coef, 0};
  if (split) {   // dW0 = dH0^T X beside the partials' fold, then dW0's fold into grad's W0 block
    // The tile kernel leaves its partials' W0 block unwritten in the split form (dW0 comes from
    // part2): the fold starts past it instead of reading 256 x 64 D unwritten floats and writing
    // grad's W0 block twice (C5: 22.8 of the fold's 38 MB per step)
    if (n.w0 == 0) fold.q0 = (WD_H * n.D) / 4;
    const dim3 grid2((unsigned)(G2 + wr_blocks<4>(nq - fold.q0)));
    if (KSM == 32)
      hipLaunchKernelGGL(ppo_wide_dw0_kernel<32>, grid2, dim3(WD_THREADS), 0, st, a, part2, G2, fold);
    else if (wd_spec(n))
      hipLaunchKernelGGL((ppo_wide_dw0_kernel<88, true>), grid2, dim3(WD_THREADS), 0, st, a, part2, G2, fold);
    else
      hipLaunchKernelGGL((ppo_wide_dw0_kernel<88, false>), grid2, dim3(WD_THREADS), 0, st, a, part2, G2, fold);
    PRL_LAUNCH_CHECK("ppo_wide_dw0");
    const int P2 = WD_H * n.D;   // 64 D: a multiple of 4
    const WrArgs fold2{part2, G2, P2, P2, grad + n.w0, nullptr, cursor, scales, N, mini_batch, vf_coef, ent_coef};
    hipLaunchKernelGGL(ppo_wide_reduce_kernel<16>, dim3((unsigned)wr_blocks<16>((P2 + 4) / 4)), dim3(256), 0,
                       st, fold2);
    PRL_LAUNCH_CHECK("ppo_wide_reduce_dw0");
  } else {
    hipLaunchKernelGGL(ppo_wide_reduce_kernel<16>, dim3((unsigned)wr_blocks<16>(nq)), dim3(256), 0, st, fold);
    PRL_LAUNCH_CHECK("ppo_wide_reduce");
  }
  return PRL_OK;
}
