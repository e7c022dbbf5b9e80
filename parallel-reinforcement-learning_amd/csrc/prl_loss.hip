// prl_loss.hip — PPO clipped-surrogate loss, forward + gradient (PPO/PPO.py:222-249).
//
// Per sample i of a minibatch of mb:
//   ratio = exp(clamp(logp - old_logp, -20, 20))                                  (PPO.py:225-231)
//   surr1 = ratio * adv;  surr2 = clamp(ratio, 1 - clip, 1 + clip) * adv           (:232-242)
//   loss_i = -min(surr1, surr2) + vf_coef * SmoothL1(V, ret) - ent_coef * H        (:245)
// and the reference back-propagates loss.mean() (:249), so
//   loss = mean_i(-min) + vf_coef * mean_i(smoothl1_i) - ent_coef * H.
// Gradients follow torch's autograd rules exactly: clamp passes the gradient on the closed
// interval, minimum() splits it 1/2-1/2 on ties, SmoothL1 (beta 1) backward is clip(x, -1, 1).
// The forward writes the per-sample gradient of `loss` (upstream 1) so the backward is a scale.
// HBM: 20 B/sample in (logp, old_logp, adv, V, ret) + 8 B/sample out (dlogp, dV).
#include "prl_common.h"

namespace prl {

constexpr int SUR_THREADS = 256;
constexpr int SUR_EPT = 4;
constexpr int SUR_TILE = SUR_THREADS * SUR_EPT;

__device__ inline float clampf_keepnan(float x, float lo, float hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}

__global__ __launch_bounds__(SUR_THREADS) void surrogate_fwd_kernel(
    const float* __restrict__ logp, const float* __restrict__ old_logp,
    const float* __restrict__ adv, const float* __restrict__ V, const float* __restrict__ ret,
    const float* __restrict__ entropy, int64_t mb, float clip, float vf_coef, float ent_coef,
    float* __restrict__ loss_out, float* __restrict__ dlogp, float* __restrict__ dV,
    double2* __restrict__ partials, unsigned* __restrict__ arrivals) {
  const float lo = 1.0f - clip, hi = 1.0f + clip;
  const float inv_mb = 1.0f / (float)mb;
  double s_pol = 0.0, s_vf = 0.0;
  const int64_t base = (int64_t)blockIdx.x * SUR_TILE;
#pragma unroll
  for (int k = 0; k < SUR_EPT; ++k) {
    const int64_t i = base + (int64_t)k * SUR_THREADS + threadIdx.x;  // coalesced
    if (i >= mb) continue;
    const float diff = logp[i] - old_logp[i];
    const float cl = clampf_keepnan(diff, -20.0f, 20.0f);
    const float ratio = expf(cl);
    const float a = adv[i];
    const float s1 = ratio * a;
    const float rc = clampf_keepnan(ratio, lo, hi);
    const float s2 = rc * a;
    const float m = (s1 != s1 || s2 != s2) ? __builtin_nanf("") : fminf(s1, s2);
    s_pol += (double)(-m);
    const float x = V[i] - ret[i];
    const float ax = fabsf(x);
    const float sl = ax < 1.0f ? 0.5f * ax * ax : ax - 0.5f;
    s_vf += (double)sl;
    if (dlogp) {
      float w1, w2;
      if (s1 < s2) { w1 = 1.0f; w2 = 0.0f; }
      else if (s2 < s1) { w1 = 0.0f; w2 = 1.0f; }
      else { w1 = 0.5f; w2 = 0.5f; }
      const float in_clip = (ratio >= lo && ratio <= hi) ? 1.0f : 0.0f;
      const float in_20 = (diff >= -20.0f && diff <= 20.0f) ? 1.0f : 0.0f;
      const float dratio = w1 * a + w2 * a * in_clip;
      dlogp[i] = -inv_mb * dratio * ratio * in_20;
    }
    if (dV) {
      const float gx = ax < 1.0f ? x : (x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f));
      dV[i] = vf_coef * inv_mb * gx;
    }
  }
  __shared__ double s_red[2][SUR_THREADS / 64];
  __shared__ int s_last;
  s_pol = wave_sum(s_pol);
  s_vf = wave_sum(s_vf);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { s_red[0][wid] = s_pol; s_red[1][wid] = s_vf; }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double bp = 0.0, bv = 0.0;
  for (int w = 0; w < SUR_THREADS / 64; ++w) { bp += s_red[0][w]; bv += s_red[1][w]; }
  const unsigned nb = gridDim.x;
  if (nb == 1) {
    const double loss = bp / (double)mb + (double)vf_coef * (bv / (double)mb) -
                        (double)ent_coef * (double)(entropy ? *entropy : 0.0f);
    *loss_out = (float)loss;
    return;
  }
  // hand-off of the block partials: write-through stores, drained, then the counter; the last
  // arriver reads them with sc1 loads (no L2 write-back / invalidate fences)
  unsigned long long* pp = reinterpret_cast<unsigned long long*>(partials + blockIdx.x);
  __hip_atomic_store(pp, __double_as_longlong(bp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(pp + 1, __double_as_longlong(bv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned old = __hip_atomic_fetch_add(arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old != nb - 1) return;
  double tp = 0.0, tv = 0.0;
  const unsigned long long* pa = reinterpret_cast<const unsigned long long*>(partials);
  for (unsigned b = 0; b < nb; ++b) {  // block order: deterministic
    tp += __longlong_as_double(__hip_atomic_load(pa + 2 * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    tv += __longlong_as_double(__hip_atomic_load(pa + 2 * b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  const double loss = tp / (double)mb + (double)vf_coef * (tv / (double)mb) -
                      (double)ent_coef * (double)(entropy ? *entropy : 0.0f);
  *loss_out = (float)loss;
  __hip_atomic_store(arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
}

__global__ __launch_bounds__(256) void surrogate_bwd_kernel(const float* __restrict__ grad_out,
                                                            const float* __restrict__ gl,
                                                            const float* __restrict__ gv, int64_t mb,
                                                            float* __restrict__ dlogp,
                                                            float* __restrict__ dV) {
  const float go = *grad_out;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < mb;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (dlogp) dlogp[i] = go * gl[i];
    if (dV) dV[i] = go * gv[i];
  }
}

}  // namespace prl

using namespace prl;

int64_t prl_surrogate_workspace_bytes(int64_t mb) {
  const int64_t nb = cdiv(mb, SUR_TILE);
  return 16 + 16 * nb;
}

extern "C" int prl_ppo_surrogate_fwd(const float* logp, const float* old_logp, const float* adv,
                                     const float* V, const float* ret, const float* entropy,
                                     int64_t mb, float clip, float vf_coef, float ent_coef,
                                     float* loss_out, float* dlogp, float* dV, void* workspace,
                                     int64_t workspace_bytes, void* stream) {
  PRL_REQUIRE(mb > 0, "prl_ppo_surrogate_fwd: empty minibatch");
  PRL_REQUIRE(logp && old_logp && adv && V && ret && loss_out, "prl_ppo_surrogate_fwd: null pointer");
  const int64_t nb = cdiv(mb, SUR_TILE);
  PRL_REQUIRE(nb < (int64_t)0x7fffffff, "prl_ppo_surrogate_fwd: minibatch too large");
  hipStream_t s = as_stream(stream);
  double2* partials = nullptr;
  unsigned* arrivals = nullptr;
  if (nb > 1) {
    PRL_REQUIRE(workspace && workspace_bytes >= prl_surrogate_workspace_bytes(mb),
                "prl_ppo_surrogate_fwd: workspace too small");
    arrivals = static_cast<unsigned*>(workspace);  // zero-initialised once; kernel re-arms it
    partials = reinterpret_cast<double2*>(static_cast<char*>(workspace) + 16);
  }
  hipLaunchKernelGGL(surrogate_fwd_kernel, dim3((unsigned)nb), dim3(SUR_THREADS), 0, s, logp,
                     old_logp, adv, V, ret, entropy, mb, clip, vf_coef, ent_coef, loss_out, dlogp,
                     dV, partials, arrivals);
  PRL_LAUNCH_CHECK("surrogate_fwd");
  return PRL_OK;
}

extern "C" int prl_ppo_surrogate_bwd(const float* grad_out, const float* dlogp_unit,
                                     const float* dV_unit, int64_t mb, float* dlogp, float* dV,
                                     void* stream) {
  PRL_REQUIRE(mb >= 0, "prl_ppo_surrogate_bwd: mb < 0");
  if (mb == 0) return PRL_OK;
  PRL_REQUIRE(grad_out, "prl_ppo_surrogate_bwd: null grad_out");
  PRL_REQUIRE((!dlogp || dlogp_unit) && (!dV || dV_unit), "prl_ppo_surrogate_bwd: null unit grads");
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(mb, 256), 1024);
  hipLaunchKernelGGL(surrogate_bwd_kernel, dim3(grid), dim3(256), 0, as_stream(stream), grad_out,
                     dlogp_unit, dV_unit, mb, dlogp, dV);
  PRL_LAUNCH_CHECK("surrogate_bwd");
  return PRL_OK;
}
