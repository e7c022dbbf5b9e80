// prl_gn.hip — fused GroupNorm(8 groups, 64 channels) + SiLU, forward and backward.
//
// Every hidden block of the reference's networks is Linear -> GroupNorm(64 // 8, 64) -> SiLU
// (PPO/ActorCritic.py:19-60, PPO/RND.py:25-30).  On the PyTorch-ROCm build in this image,
// nn.GroupNorm's backward returns wrong weight/bias gradients for N >= 512 rows (dx is right;
// measured by tools/diag_groupnorm.py against a float64 restatement), which silently corrupts
// PPO.learn().  These kernels replace GroupNorm + SiLU on device tensors with one fused pass
// each way:
//   forward:  y = (x - mean_g) * rstd_g * w + b,  out = y * sigmoid(y)      (biased variance)
//   backward: dy = dout * s * (1 + y (1 - s)),  dxhat = dy * w,
//             dx = rstd * (dxhat - mean_g(dxhat) - xhat * mean_g(dxhat * xhat)),
//             dw = sum_rows dy * xhat,  db = sum_rows dy
// One thread owns one (row, group) = 8 contiguous floats (two 16-B loads/stores, coalesced);
// the backward's per-channel column sums are reduced in LDS per workgroup and across workgroups
// by a write-through hand-off to the last-arriving workgroup (block order: deterministic).
#include "prl_common.h"

#include <algorithm>

namespace prl {

constexpr int GN_C = 64, GN_G = 8, GN_GS = 8;       // channels, groups, group size
constexpr int GN_THREADS = 256;                     // 32 rows x 8 groups per slab
constexpr int GN_ROWS = GN_THREADS / GN_G;          // 32
constexpr int GN_MAX_BLOCKS = 240;
constexpr int GN_U = 4;
constexpr int GN_FB = 16;                           // partial loads in flight per thread (fold)                             // rows per thread per backward pass

struct GnRow {
  float x[GN_GS];
};

__device__ inline void gn_load(const float* p, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[0];
  const float4 b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ inline void gn_store(float* p, const float* v) {
  reinterpret_cast<float4*>(p)[0] = float4{v[0], v[1], v[2], v[3]};
  reinterpret_cast<float4*>(p)[1] = float4{v[4], v[5], v[6], v[7]};
}

__device__ inline void gn_stats(const float* v, float eps, float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < GN_GS; ++k) s += v[k];
  mean = s * (1.0f / GN_GS);
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < GN_GS; ++k) q += (v[k] - mean) * (v[k] - mean);
  rstd = 1.0f / sqrtf(q * (1.0f / GN_GS) + eps);
}

__global__ __launch_bounds__(GN_THREADS) void gn_silu_fwd_kernel(const float* __restrict__ x,
                                                                 int64_t N,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ b,
                                                                 float eps, int silu,
                                                                 float* __restrict__ out) {
  const int grp = threadIdx.x & (GN_G - 1);
  const int c0 = grp * GN_GS;
  float wv[GN_GS], bv[GN_GS];
#pragma unroll
  for (int k = 0; k < GN_GS; ++k) { wv[k] = w[c0 + k]; bv[k] = b[c0 + k]; }
  for (int64_t row = (int64_t)blockIdx.x * GN_ROWS + (threadIdx.x >> 3); row < N;
       row += (int64_t)gridDim.x * GN_ROWS) {
    float v[GN_GS];
    gn_load(x + row * GN_C + c0, v);
    float mean, rstd;
    gn_stats(v, eps, mean, rstd);
#pragma unroll
    for (int k = 0; k < GN_GS; ++k) {
      const float y = (v[k] - mean) * rstd * wv[k] + bv[k];
      v[k] = silu ? y / (1.0f + expf(-y)) : y;
    }
    gn_store(out + row * GN_C + c0, v);
  }
}

__global__ __launch_bounds__(GN_THREADS) void gn_silu_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ dout, int64_t N,
    const float* __restrict__ w, const float* __restrict__ b, float eps, int silu,
    float* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db,
    float* __restrict__ partials /*[gridDim][128]*/, unsigned* __restrict__ arrivals) {
  __shared__ float s_col[2][GN_ROWS][GN_C + 1];
  __shared__ int s_last;
  const int grp = threadIdx.x & (GN_G - 1);
  const int rloc = threadIdx.x >> 3;
  const int c0 = grp * GN_GS;
  float wv[GN_GS], bv[GN_GS], accw[GN_GS], accb[GN_GS];
#pragma unroll
  for (int k = 0; k < GN_GS; ++k) {
    wv[k] = w[c0 + k];
    bv[k] = b[c0 + k];
    accw[k] = 0.f;
    accb[k] = 0.f;
  }
  // GN_U rows per thread per pass, all loads issued first (at 240 workgroups of 4 waves, one
  // row at a time left the kernel latency-bound at ~0.7 TB/s); rows stay in ascending order per
  // thread, so the column sums are accumulated exactly as before
  const int64_t stride = (int64_t)gridDim.x * GN_ROWS;
  for (int64_t row0 = (int64_t)blockIdx.x * GN_ROWS + rloc; row0 < N; row0 += GN_U * stride) {
    float vv[GN_U][GN_GS], gg[GN_U][GN_GS];
#pragma unroll
    for (int u = 0; u < GN_U; ++u) {
      const int64_t row = row0 + u * stride;
      if (row < N) {
        gn_load(x + row * GN_C + c0, vv[u]);
        gn_load(dout + row * GN_C + c0, gg[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < GN_U; ++u) {
    const int64_t row = row0 + u * stride;
    if (row >= N) break;
    float* v = vv[u];
    const float* go = gg[u];
    float mean, rstd;
    gn_stats(v, eps, mean, rstd);
    float xh[GN_GS], dxh[GN_GS];
    float m1 = 0.f, m2 = 0.f;
#pragma unroll
    for (int k = 0; k < GN_GS; ++k) {
      xh[k] = (v[k] - mean) * rstd;
      const float y = xh[k] * wv[k] + bv[k];
      float dy = go[k];
      if (silu) {
        const float s = 1.0f / (1.0f + expf(-y));
        dy = go[k] * (s * (1.0f + y * (1.0f - s)));
      }
      accw[k] += dy * xh[k];
      accb[k] += dy;
      dxh[k] = dy * wv[k];
      m1 += dxh[k];
      m2 += dxh[k] * xh[k];
    }
    m1 *= (1.0f / GN_GS);
    m2 *= (1.0f / GN_GS);
#pragma unroll
    for (int k = 0; k < GN_GS; ++k) v[k] = rstd * (dxh[k] - m1 - xh[k] * m2);
    gn_store(dx + row * GN_C + c0, v);
    }
  }
  // column sums: rows of this block -> one partial per channel
#pragma unroll
  for (int k = 0; k < GN_GS; ++k) {
    s_col[0][rloc][c0 + k] = accw[k];
    s_col[1][rloc][c0 + k] = accb[k];
  }
  __syncthreads();
  float colsum = 0.f;
  if (threadIdx.x < 2 * GN_C) {
    const int which = threadIdx.x >> 6, c = threadIdx.x & 63;
    for (int r = 0; r < GN_ROWS; ++r) colsum += s_col[which][r][c];
  }
  if (gridDim.x == 1) {
    if (threadIdx.x < GN_C) dw[threadIdx.x] = colsum;
    else if (threadIdx.x < 2 * GN_C) db[threadIdx.x - GN_C] = colsum;
    return;
  }
  // hand the partial to the last-arriving block: write-through stores, drained, then a counter
  if (threadIdx.x < 2 * GN_C) {
    __hip_atomic_store(reinterpret_cast<unsigned*>(partials) + blockIdx.x * 2 * GN_C + threadIdx.x,
                       __float_as_uint(colsum), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old == gridDim.x - 1) ? 1 : 0;
  }
  __syncthreads();
  if (!s_last) return;
  // the last block folds the partials in block order: both halves of the block take half of the
  // blocks each (GN_FB loads in flight per thread: one at a time, 240 dependent L2 round trips
  // made this fold ~70 us, the whole kernel's time), then the two halves add in LDS
  {
    const int col = threadIdx.x & (2 * GN_C - 1), half = threadIdx.x >> 7;
    const unsigned nb = gridDim.x, mid = (nb + 1) / 2;
    const unsigned lo = half ? mid : 0u, hi = half ? nb : mid;
    const unsigned* pp = reinterpret_cast<const unsigned*>(partials);
    float acc = 0.f;
    for (unsigned b0 = lo; b0 < hi; b0 += GN_FB) {
      float v[GN_FB];
#pragma unroll
      for (int u = 0; u < GN_FB; ++u)
        v[u] = b0 + u < hi ? __uint_as_float(__hip_atomic_load(pp + (b0 + u) * 2 * GN_C + col,
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                           : 0.f;
#pragma unroll
      for (int u = 0; u < GN_FB; ++u) acc += v[u];
    }
    (&s_col[0][0][0])[half * 2 * GN_C + col] = acc;   // s_col is free again (barriers above)
  }
  __syncthreads();
  if (threadIdx.x < 2 * GN_C) {
    const float* fold = &s_col[0][0][0];
    const float acc = fold[threadIdx.x] + fold[2 * GN_C + threadIdx.x];
    if (threadIdx.x < GN_C) dw[threadIdx.x] = acc;
    else db[threadIdx.x - GN_C] = acc;
  }
  if (threadIdx.x == 0) __hip_atomic_store(arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

inline unsigned gn_blocks(int64_t N) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(N, GN_ROWS), GN_MAX_BLOCKS));
}

}  // namespace prl

using namespace prl;

int64_t prl_gn_workspace_bytes(int64_t N) { return 16 + (int64_t)gn_blocks(N) * 2 * GN_C * 4; }

extern "C" int prl_gn_silu_fwd(const float* x, int64_t N, int32_t C, int32_t groups,
                               const float* w, const float* b, float eps, int32_t silu, float* out,
                               void* stream) {
  PRL_REQUIRE(C == GN_C && groups == GN_G, "prl_gn_silu_fwd: only GroupNorm(8, 64) is built");
  PRL_REQUIRE(N >= 0, "prl_gn_silu_fwd: N < 0");
  if (N == 0) return PRL_OK;
  PRL_REQUIRE(x && w && b && out, "prl_gn_silu_fwd: null pointer");
  PRL_REQUIRE(aligned16(x) && aligned16(out), "prl_gn_silu_fwd: x/out must be 16-B aligned");
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(N, GN_ROWS), 4096);
  hipLaunchKernelGGL(gn_silu_fwd_kernel, dim3(grid), dim3(GN_THREADS), 0, as_stream(stream), x, N,
                     w, b, eps, silu, out);
  PRL_LAUNCH_CHECK("gn_silu_fwd");
  return PRL_OK;
}

extern "C" int prl_gn_silu_bwd(const float* x, const float* dout, int64_t N, int32_t C,
                               int32_t groups, const float* w, const float* b, float eps,
                               int32_t silu, float* dx, float* dw, float* db, void* workspace,
                               int64_t workspace_bytes, void* stream) {
  PRL_REQUIRE(C == GN_C && groups == GN_G, "prl_gn_silu_bwd: only GroupNorm(8, 64) is built");
  PRL_REQUIRE(N >= 0, "prl_gn_silu_bwd: N < 0");
  PRL_REQUIRE(x && dout && w && b && dx && dw && db, "prl_gn_silu_bwd: null pointer");
  PRL_REQUIRE(aligned16(x) && aligned16(dout) && aligned16(dx), "prl_gn_silu_bwd: 16-B alignment");
  const unsigned grid = gn_blocks(N);
  unsigned* arrivals = nullptr;
  float* partials = nullptr;
  if (grid > 1) {
    PRL_REQUIRE(workspace && workspace_bytes >= prl_gn_workspace_bytes(N),
                "prl_gn_silu_bwd: workspace too small");
    arrivals = static_cast<unsigned*>(workspace);  // zero-initialised once; kernel re-arms it
    partials = reinterpret_cast<float*>(static_cast<char*>(workspace) + 16);
  }
  hipLaunchKernelGGL(gn_silu_bwd_kernel, dim3(grid), dim3(GN_THREADS), 0, as_stream(stream), x,
                     dout, N, w, b, eps, silu, dx, dw, db, partials, arrivals);
  PRL_LAUNCH_CHECK("gn_silu_bwd");
  return PRL_OK;
}
