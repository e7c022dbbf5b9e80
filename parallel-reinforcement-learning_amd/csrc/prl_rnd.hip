// prl_rnd.hip — RND intrinsic reward forward (PPO/RND.py:71-94) on fp32 MFMA.
//
//   out[i] = beta * || pred(x_i) - target(x_i) ||_2,
//   net(x) = Linear(64 -> D)(SiLU(GroupNorm(8 groups, 64, eps 1e-5)(Linear(D -> 64)(x))))
// (RND.py:25-38; both nets are independent re-initialisations of the same architecture).
//
// One workgroup = 4 waves = 64 rows.  Layer 1 for BOTH nets is one GEMM
//   H[64 x 128] = X[64 x D] . [W1_target ; W1_pred]^T       (K = D, staged in 64-deep LDS chunks)
// on v_mfma_f32_32x32x2_f32 (exact f32 FMA chain, 64 FLOP/clk/SIMD — gfx950 has no xf32), wave w
// owning rows 32*(w&1) and the 64 hidden units of net w>>1.  Bias, GroupNorm (groups of 8
// consecutive units = 8 consecutive lanes: xor-shuffle reductions) and SiLU run on the
// accumulators.  The activations go to LDS as Z = [ S_pred | -S_target ] so that the second
// layers AND their difference are one GEMM
//   Yp - Yt = Z[64 x 128] . [W2_pred^T ; W2_target^T] + (b2_pred - b2_target)   (K = 128),
// processed in 64-column chunks; squares are reduced across the 32 column lanes per row and the
// row norms never leave the chip.  FLOPs per row: 512 * D (both nets, both layers).
#include "prl_common.h"

namespace prl {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int RB_M = 64;          // rows per workgroup
constexpr int RB_KC = 64;         // layer-1 K chunk
constexpr int XP = RB_KC + 1;     // LDS pitch (floats): odd -> conflict-free ds_read_b32 columns
constexpr int ZP = 128 + 1;       // pitch of Z / W2 chunk

struct RndNet {
  const float *w1, *b1, *gw, *gb, *w2, *b2;
};

__device__ inline int c_row(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

__global__ __launch_bounds__(256) void rnd_forward_kernel(const float* __restrict__ x, int64_t n,
                                                          int D, RndNet tn, RndNet pn, float beta,
                                                          float* __restrict__ out) {
  // union of the layer-1 staging (X chunk + W1 chunk) and the layer-2 staging (Z + W2 chunk)
  __shared__ float s_buf[RB_M * ZP + RB_M * ZP];  // 2 * 64 * 129 floats = 66 KB
  __shared__ float s_rowsq[2][RB_M];
  float* s_x = s_buf;                  // [64][XP]
  float* s_w = s_buf + RB_M * XP;      // [128][XP]
  float* s_z = s_buf;                  // [64][ZP]  (after layer 1)
  float* s_w2 = s_buf + RB_M * ZP;     // [64][ZP]

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  const int64_t row0 = (int64_t)blockIdx.x * RB_M;
  const int mr = 32 * (w & 1);
  const int net = w >> 1;  // 0 target, 1 pred
  const RndNet nn = net ? pn : tn;

  // ---- layer 1 ----
  f32x16 acc0 = {}, acc1 = {};
  for (int k0 = 0; k0 < D; k0 += RB_KC) {
    const int kc = min(RB_KC, D - k0);
    const int kce = (kc + 1) & ~1;
    __syncthreads();
    for (int idx = tid; idx < RB_M * RB_KC; idx += 256) {
      const int r = idx / RB_KC, k = idx % RB_KC;
      float v = 0.f;
      if (k < kc && row0 + r < n) v = x[(row0 + r) * D + k0 + k];
      s_x[r * XP + k] = v;
    }
    for (int idx = tid; idx < 128 * RB_KC; idx += 256) {
      const int c = idx / RB_KC, k = idx % RB_KC;
      const float* W = (c < 64) ? tn.w1 : pn.w1;
      s_w[c * XP + k] = (k < kc) ? W[(c & 63) * D + k0 + k] : 0.f;
    }
    __syncthreads();
    const float* ax = s_x + (mr + lr) * XP + lh;
    const float* bw0 = s_w + (64 * net + lr) * XP + lh;
    const float* bw1 = s_w + (64 * net + 32 + lr) * XP + lh;
    for (int k = 0; k < kce; k += 2) {
      const float a = ax[k];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bw0[k], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bw1[k], acc1, 0, 0, 0);
    }
  }

  // ---- bias + GroupNorm(8 x 8) + SiLU on the accumulators ----
  const int c0 = lr, c1 = 32 + lr;  // hidden unit of acc0 / acc1 for this lane
  const float b0 = nn.b1[c0], b1v = nn.b1[c1];
  const float g0 = nn.gw[c0], g1 = nn.gw[c1], e0 = nn.gb[c0], e1 = nn.gb[c1];
  float h0[16], h1[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float v0 = acc0[i] + b0, v1 = acc1[i] + b1v;
    float s0 = v0, s1 = v1;
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {
      s0 += __shfl_xor(s0, off, 64);
      s1 += __shfl_xor(s1, off, 64);
    }
    const float m0 = s0 * 0.125f, m1 = s1 * 0.125f;
    float q0 = (v0 - m0) * (v0 - m0), q1 = (v1 - m1) * (v1 - m1);
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {
      q0 += __shfl_xor(q0, off, 64);
      q1 += __shfl_xor(q1, off, 64);
    }
    const float r0 = 1.0f / sqrtf(q0 * 0.125f + 1e-5f), r1 = 1.0f / sqrtf(q1 * 0.125f + 1e-5f);
    const float y0 = (v0 - m0) * r0 * g0 + e0, y1 = (v1 - m1) * r1 * g1 + e1;
    h0[i] = y0 / (1.0f + expf(-y0));
    h1[i] = y1 / (1.0f + expf(-y1));
  }
  __syncthreads();  // everyone is done reading the layer-1 staging
  {
    const int zoff = net ? 0 : 64;          // Z = [S_pred | -S_target]
    const float sgn = net ? 1.0f : -1.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = mr + c_row(i, lane);
      s_z[r * ZP + zoff + c0] = sgn * h0[i];
      s_z[r * ZP + zoff + c1] = sgn * h1[i];
    }
  }

  // ---- layer 2 (both nets + difference) in 64-column chunks ----
  float rowsq[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) rowsq[i] = 0.f;
  const int ct = w >> 1;  // column tile of the chunk this wave computes
  for (int col0 = 0; col0 < D; col0 += 64) {
    __syncthreads();
    for (int idx = tid; idx < 64 * 128; idx += 256) {
      const int c = idx / 128, k = idx % 128;
      const int col = col0 + c;
      float v = 0.f;
      if (col < D) v = (k < 64) ? pn.w2[col * 64 + k] : tn.w2[col * 64 + (k - 64)];
      s_w2[c * ZP + k] = v;
    }
    __syncthreads();
    f32x16 acc = {};
    const float* az = s_z + (mr + lr) * ZP + lh;
    const float* bz = s_w2 + (32 * ct + lr) * ZP + lh;
    for (int k = 0; k < 128; k += 2) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(az[k], bz[k], acc, 0, 0, 0);
    const int col = col0 + 32 * ct + lr;
    const bool cin = col < D;
    const float bd = cin ? (pn.b2[col] - tn.b2[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = cin ? acc[i] + bd : 0.f;
      float sq = v * v;
#pragma unroll
      for (int off = 1; off < 32; off <<= 1) sq += __shfl_xor(sq, off, 64);
      rowsq[i] += sq;
    }
  }
  if (lr == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s_rowsq[ct][mr + c_row(i, lane)] = rowsq[i];
  }
  __syncthreads();
  if (tid < RB_M && row0 + tid < n) out[row0 + tid] = beta * sqrtf(s_rowsq[0][tid] + s_rowsq[1][tid]);
}

}  // namespace prl

using namespace prl;

extern "C" int prl_rnd_forward(const float* x, int64_t n, int32_t D, const float* t_w1,
                               const float* t_b1, const float* t_gw, const float* t_gb,
                               const float* t_w2, const float* t_b2, const float* p_w1,
                               const float* p_b1, const float* p_gw, const float* p_gb,
                               const float* p_w2, const float* p_b2, float beta, float* out,
                               void* stream) {
  PRL_REQUIRE(n >= 0 && D > 0, "prl_rnd_forward: bad sizes");
  if (n == 0) return PRL_OK;
  PRL_REQUIRE(x && out && t_w1 && t_b1 && t_gw && t_gb && t_w2 && t_b2 && p_w1 && p_b1 && p_gw &&
                  p_gb && p_w2 && p_b2,
              "prl_rnd_forward: null pointer");
  PRL_REQUIRE(cdiv(n, RB_M) < (int64_t)0x7fffffff, "prl_rnd_forward: n too large");
  RndNet tn{t_w1, t_b1, t_gw, t_gb, t_w2, t_b2}, pn{p_w1, p_b1, p_gw, p_gb, p_w2, p_b2};
  hipLaunchKernelGGL(rnd_forward_kernel, dim3((unsigned)cdiv(n, RB_M)), dim3(256), 0,
                     as_stream(stream), x, n, (int)D, tn, pn, beta, out);
  PRL_LAUNCH_CHECK("rnd_forward");
  return PRL_OK;
}
