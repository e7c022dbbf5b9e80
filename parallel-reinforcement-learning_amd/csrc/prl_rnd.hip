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

#include <stdlib.h>

#include <algorithm>

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


// ---- the persistent fast path (D % 4 == 0: 16-B row loads) -----------------------------------
// Each workgroup (4 waves, one per SIMD, one workgroup per CU) loops over 128-row blocks.  The
// first kernel above re-staged both nets' weights (~356 KB at D = 348) through LDS with 4-B
// loads and two barriers per 64-row block, ~4x the bytes of its own rows; here the weights are
// streamed per 128-row block in double-buffered chunks with 16-B loads (the next chunk in
// registers while the current one feeds the MFMAs, one barrier per chunk), so every LDS fragment
// read feeds 2-4 MFMAs and the weight traffic per row halves.
//   layer 1: H[128 x 128] = X . [W1_target ; W1_pred]^T, K = D in 32-deep chunks; wave w owns
//            rows 32w .. 32w+31 and all 128 hidden units (4 accumulators of 32 x 32);
//   bias + GroupNorm + SiLU on the accumulators (a group = 8 consecutive lanes: DPP sums), into
//            Z = [S_pred | -S_target] (LDS, 128 x 128);
//   layer 2: Yp - Yt = Z . [W2_pred^T ; W2_target^T] + (b2_pred - b2_target) in 64-column chunks
//            (2 accumulators per wave), squares accumulated per lane across all chunks and
//            reduced over the 32 column lanes once per block.
constexpr int RF_M = 128;         // rows per block
constexpr int RF_KC = 32;         // layer-1 K chunk
constexpr int RF_P1 = RF_KC + 4;  // pitch of the X / W1 chunks (16-B rows: ds_write_b128 staging;
                                  // column reads see at most a 2-way bank conflict)
constexpr int RF_CC = 64;         // layer-2 column chunk
constexpr int RF_PZ = 129;        // pitch of Z (odd: conflict-free row-fragment reads)
constexpr int RF_PW = 132;        // pitch of the W2 chunk (16-B rows)
constexpr int RF_STAGE = 2 * 2 * RF_M * RF_P1;          // layer-1 double buffer: [2][X | W1]
constexpr int RF_STAGE2 = 2 * RF_CC * RF_PW;            // layer-2 double buffer: [2][64][132]
constexpr int RF_LDS = (RF_STAGE > RF_STAGE2 ? RF_STAGE : RF_STAGE2) + RF_M * RF_PZ + 2 * RF_M;

// sum over the 8 consecutive lanes of a GroupNorm group (every lane gets the same bits)
__device__ inline float rf_sum8(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));   // xor 1
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));   // xor 2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));  // half mirror
  return v;
}

struct RfChunk {
  float4 v[8];
};
// layer-1 chunk c of block rows [row0, row0 + 128): X[128][32] and [W1_t ; W1_p][128][32], thread
// tid takes float4 slots tid + 256 i (i < 4) of each (row = slot >> 3, quad = slot & 7)
__device__ inline void rf_load1(RfChunk& ch, const float* x, int64_t n, int D, int64_t row0, int k0,
                                const float* wt, const float* wp) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int slot = tid + 256 * i, r = slot >> 3, k = k0 + 4 * (slot & 7);
    const bool kin = k < D;
    ch.v[i] = (kin && row0 + r < n) ? *reinterpret_cast<const float4*>(x + (row0 + r) * D + k)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
    const float* W = r < 64 ? wt : wp;
    ch.v[4 + i] = kin ? *reinterpret_cast<const float4*>(W + (r & 63) * D + k) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
__device__ inline void rf_store1(const RfChunk& ch, float* buf) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int slot = tid + 256 * (i & 3), r = slot >> 3, k = 4 * (slot & 7);
    *reinterpret_cast<float4*>(buf + (i >> 2) * RF_M * RF_P1 + r * RF_P1 + k) = ch.v[i];
  }
}
// layer-2 chunk of output columns [col0, col0 + 64): W2cat[k][col] = k < 64 ? W2_p[col][k] :
// W2_t[col][k - 64], stored [col][k]; thread tid takes slots tid + 256 i (i < 8): col = slot >> 5,
// k = 4 (slot & 31)
__device__ inline void rf_load2(RfChunk& ch, int D, int col0, const float* w2t, const float* w2p) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int slot = tid + 256 * i, c = slot >> 5, k = 4 * (slot & 31), col = col0 + c;
    const float* W = k < 64 ? w2p : w2t;
    ch.v[i] = col < D ? *reinterpret_cast<const float4*>(W + col * 64 + (k & 63)) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
__device__ inline void rf_store2(const RfChunk& ch, float* buf) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int slot = tid + 256 * i, c = slot >> 5, k = 4 * (slot & 31);
    *reinterpret_cast<float4*>(buf + c * RF_PW + k) = ch.v[i];
  }
}

__global__ __launch_bounds__(256, 1) void rnd_forward_fast_kernel(const float* __restrict__ x, int64_t n,
                                                                  int D, RndNet tn, RndNet pn, float beta,
                                                                  float* __restrict__ out) {
  extern __shared__ __align__(16) float rf_lds[];
  float* stage = rf_lds;                                                       // layer 1 / 2 chunks
  float* zs = rf_lds + (RF_STAGE > RF_STAGE2 ? RF_STAGE : RF_STAGE2);          // Z [128][129]
  float* rsq = zs + RF_M * RF_PZ;                                              // [2][128]
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, lr = lane & 31, lh = lane >> 5;
  const int64_t nblocks = (n + RF_M - 1) / RF_M;
  const int nk = (D + RF_KC - 1) / RF_KC, nc = (D + RF_CC - 1) / RF_CC;
  // per-lane constants of the GroupNorm epilogue: hidden unit u = 32 j + lr of net (j >> 1)
  RfChunk ch;   // the next chunk to stage, in registers (loaded one chunk ahead, also across the
                // layer and block boundaries)
  if ((int64_t)blockIdx.x < nblocks) rf_load1(ch, x, n, D, (int64_t)blockIdx.x * RF_M, 0, tn.w1, pn.w1);
  for (int64_t blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
    const int64_t row0 = blk * RF_M;
    const bool more = blk + gridDim.x < nblocks;
    // ---- layer 1 ----
    f32x16 acc[4] = {};
    rf_store1(ch, stage);
    __syncthreads();
    for (int c = 0; c < nk; ++c) {
      if (c + 1 < nk) rf_load1(ch, x, n, D, row0, (c + 1) * RF_KC, tn.w1, pn.w1);
      else rf_load2(ch, D, 0, tn.w2, pn.w2);   // layer 2's first chunk
      const float* bx = stage + (c & 1) * 2 * RF_M * RF_P1;
      const float* ax = bx + (32 * w + lr) * RF_P1 + lh;
      const float* bw = bx + RF_M * RF_P1 + lr * RF_P1 + lh;
      // every fragment of the chunk read up front (80 VGPRs): the MFMA chain then waits only on
      // the first reads, instead of a read-wait bubble per k-pair at one wave per SIMD
      float av[RF_KC / 2], bv[4][RF_KC / 2];
#pragma unroll
      for (int k = 0; k < RF_KC / 2; ++k) {
        av[k] = ax[2 * k];
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[j][k] = bw[32 * j * RF_P1 + 2 * k];
      }
#pragma unroll
      for (int k = 0; k < RF_KC / 2; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[k], bv[j][k], acc[j], 0, 0, 0);
      if (c + 1 < nk) rf_store1(ch, stage + ((c + 1) & 1) * 2 * RF_M * RF_P1);
      __syncthreads();
    }
    // ---- bias + GroupNorm(8 x 8) + SiLU, into Z = [S_pred | -S_target] ----
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const RndNet& nn = j < 2 ? tn : pn;
      const int u = 32 * (j & 1) + lr;
      const float bb = nn.b1[u], gw = nn.gw[u], gb = nn.gb[u];
      const int zc = (j < 2 ? 64 : 0) + u;
      const float sgn = j < 2 ? -1.0f : 1.0f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float v = acc[j][i] + bb;
        const float mean = rf_sum8(v) * 0.125f;
        const float d = v - mean;
        const float var = rf_sum8(d * d) * 0.125f;
        // hardware rsq / exp / rcp (~1 ulp each; the reward is checked at 2e-5 rel): IEEE
        // division and libm expf cost ~40 VALU per value here, 64 values per lane per block
        const float y = d * __builtin_amdgcn_rsqf(var + 1e-5f) * gw + gb;
        zs[(32 * w + c_row(i, lane)) * RF_PZ + zc] = sgn * (y * __builtin_amdgcn_rcpf(1.0f + __expf(-y)));
      }
    }
    // ---- layer 2 + squared differences ----
    float rowsq[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) rowsq[i] = 0.f;
    rf_store2(ch, stage);
    __syncthreads();   // Z and the first W2 chunk
    for (int c = 0; c < nc; ++c) {
      if (c + 1 < nc) rf_load2(ch, D, (c + 1) * RF_CC, tn.w2, pn.w2);
      else if (more) rf_load1(ch, x, n, D, (blk + gridDim.x) * RF_M, 0, tn.w1, pn.w1);   // next block
      const float* bw2 = stage + (c & 1) * RF_CC * RF_PW;
      const float* az = zs + (32 * w + lr) * RF_PZ + lh;
      const float* b0 = bw2 + lr * RF_PW + lh;
      f32x16 y0 = {}, y1 = {};
#pragma unroll
      for (int k0 = 0; k0 < 128; k0 += 32) {   // fragments 16 k-steps at a time, read up front
        float a[16], c0[16], c1[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          a[k] = az[k0 + 2 * k];
          c0[k] = b0[k0 + 2 * k];
          c1[k] = b0[32 * RF_PW + k0 + 2 * k];
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          y0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], c0[k], y0, 0, 0, 0);
          y1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], c1[k], y1, 0, 0, 0);
        }
      }
      const int col_a = c * RF_CC + lr, col_b = col_a + 32;
      const float bd_a = col_a < D ? pn.b2[col_a] - tn.b2[col_a] : 0.f;
      const float bd_b = col_b < D ? pn.b2[col_b] - tn.b2[col_b] : 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float va = col_a < D ? y0[i] + bd_a : 0.f;
        const float vb = col_b < D ? y1[i] + bd_b : 0.f;
        rowsq[i] += va * va + vb * vb;
      }
      if (c + 1 < nc) rf_store2(ch, stage + ((c + 1) & 1) * RF_CC * RF_PW);
      __syncthreads();
    }
    // ---- reduce over the 32 column lanes of each half-wave, write beta * sqrt ----
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float v = rowsq[i];
      v += __shfl_xor(v, 16, 64);
      v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
      v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
      v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
      v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));
      if (lr == 0) rsq[32 * w + c_row(i, lane)] = v;
    }
    __syncthreads();
    if (tid < RF_M && row0 + tid < n) out[row0 + tid] = beta * sqrtf(rsq[tid]);
    // (the next block stages into `stage` first: the loop's last barrier has passed every read of
    // it; rsq is rewritten only after that block's own barriers)
  }
}


// ---- RND.update_pred's gradient (RND.py:96-115), fused -------------------------------------------
// One optimizer step of the predictor is MSE(pred(x), target(x).detach()) over a minibatch, its
// backward, AdamW.  This kernel forms the predictor's whole gradient for the minibatch in ONE
// launch per 128-row block (+ one fold launch), where the PyTorch step ran ~25 kernels (two
// forwards, hipBLASLt GEMMs for the three weight / input gradients, GroupNorm / SiLU backward,
// column sums), ~0.6 ms per 65,536-row minibatch at C5:
//   forward   the forward kernel's layer 1 (both nets) + GroupNorm + SiLU into Z = [S_p | -S_t],
//             layer 2 as Yp - Yt in 64-column chunks (fp32 MFMA 32x32x2);
//   dY        = scale (Yp - Yt) per chunk (scale = 2 / (rows D): MSELoss 'mean'; rows >= n: 0),
//             into LDS; then per chunk dW2 = dY^T S_p (one 32 x 32 tile per wave, K = 128 rows),
//             db2 (column sums) and dS_p += dY W2_p (the layer-1 accumulators' layout);
//   GN + SiLU backward on the fragments (the forward recomputed from the kept pre-activations,
//             the forward kernel's arithmetic), giving dH_p, dgamma, dbeta, db1;
//   dW1       = dH_p^T X: the block's X re-streamed in 32-column chunks, v_mfma_f32_16x16x4_f32
//             (wave w: units 16w .. 16w + 15), K = 128 rows.
// Every block writes its partial gradient in the flat parameter order (W1, b1, gamma, beta, W2,
// b2: torch parameters() of the predictor), and rnd_grad_fold{1,2}_kernel sum the blocks in a
// fixed order (f64): deterministic, no atomics.
constexpr int RG_PD = 65;                 // pitch of dY [128][64] (odd: conflict-free row reads)
constexpr int RG_PH = 80;                 // pitch of dH [128][64] (16-lane groups on 4 bank offsets)
constexpr int RG_PX = 48;                 // pitch of the dW1 phase's X chunk [128][32]
constexpr int RG_W2 = RF_CC * RF_PW;      // one layer-2 weight chunk [64][132]
constexpr int RG_LDS = RF_STAGE + RF_M * RF_PZ + 4 * 3 * 64 + 4 * 64;
static_assert(RG_W2 + RF_M * RG_PD <= RF_STAGE, "layer-2 chunk + dY fit the stage");
static_assert(RF_M * RG_PH <= RF_M * RF_PZ, "dH fits Z");
static_assert(RF_M * RG_PX <= RF_STAGE, "X chunk fits the stage");

__device__ inline int64_t rg_param_floats(int D) { return 129 * (int64_t)D + 192; }

// X chunk [128][32] of block rows for the dW1 phase: thread tid takes float4 slots tid + 256 i
__device__ inline void rg_loadx(float4 (&v)[4], const float* x, int64_t n, int D, int64_t row0, int k0) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int slot = tid + 256 * i, r = slot >> 3, k = k0 + 4 * (slot & 7);
    v[i] = (k < D && row0 + r < n) ? *reinterpret_cast<const float4*>(x + (row0 + r) * D + k)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
__device__ inline void rg_storex(const float4 (&v)[4], float* buf) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int slot = tid + 256 * i, r = slot >> 3, k = 4 * (slot & 7);
    *reinterpret_cast<float4*>(buf + r * RG_PX + k) = v[i];
  }
}

__global__ __launch_bounds__(256, 1) void rnd_pred_grad_kernel(const float* __restrict__ x, int64_t n, int D,
                                                               RndNet tn, RndNet pn, float scale,
                                                               float* __restrict__ partial) {
  extern __shared__ __align__(16) float rg_lds[];
  float* stage = rg_lds;                               // layer 1: [2][X | W1] chunks
  float* w2s = rg_lds;                                 // layer 2: one W2 chunk [64][132]
  float* dys = rg_lds + RG_W2;                         // layer 2: dY chunk [128][65]
  float* xs = rg_lds;                                  // dW1 phase: X chunk [128][48]
  float* zs = rg_lds + RF_STAGE;                       // Z [128][129]; then dH [128][80]
  float* cs = zs + RF_M * RF_PZ;                       // [4 waves][3][64] column sums
  float* cb = cs + 4 * 3 * 64;                         // [4 waves][64] db2 column sums
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, lr = lane & 31, lh = lane >> 5;
  const int64_t blk = blockIdx.x, row0 = blk * RF_M;
  const int nk = (D + RF_KC - 1) / RF_KC, nc = (D + RF_CC - 1) / RF_CC;
  float* part = partial + blk * rg_param_floats(D);
  float* pW1 = part;
  float* pb1 = part + 64 * (int64_t)D;
  float* pgw = pb1 + 64;
  float* pgb = pgw + 64;
  float* pW2 = pgb + 64;
  float* pb2 = pW2 + 64 * (int64_t)D;
  // ---- layer 1, both nets (the forward kernel's loop) ----
  RfChunk ch;
  rf_load1(ch, x, n, D, row0, 0, tn.w1, pn.w1);
  f32x16 acc[4] = {};
  rf_store1(ch, stage);
  __syncthreads();
  for (int c = 0; c < nk; ++c) {
    if (c + 1 < nk) rf_load1(ch, x, n, D, row0, (c + 1) * RF_KC, tn.w1, pn.w1);
    else rf_load2(ch, D, 0, tn.w2, pn.w2);
    const float* bx = stage + (c & 1) * 2 * RF_M * RF_P1;
    const float* ax = bx + (32 * w + lr) * RF_P1 + lh;
    const float* bw = bx + RF_M * RF_P1 + lr * RF_P1 + lh;
    float av[RF_KC / 2], bv[4][RF_KC / 2];
#pragma unroll
    for (int k = 0; k < RF_KC / 2; ++k) {
      av[k] = ax[2 * k];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j][k] = bw[32 * j * RF_P1 + 2 * k];
    }
#pragma unroll
    for (int k = 0; k < RF_KC / 2; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[k], bv[j][k], acc[j], 0, 0, 0);
    if (c + 1 < nk) rf_store1(ch, stage + ((c + 1) & 1) * 2 * RF_M * RF_P1);
    __syncthreads();
  }
  // ---- bias + GroupNorm + SiLU into Z = [S_pred | -S_target] (the forward kernel's epilogue) ----
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const RndNet& nn = j < 2 ? tn : pn;
    const int u = 32 * (j & 1) + lr;
    const float bb = nn.b1[u], gw = nn.gw[u], gb = nn.gb[u];
    const int zc = (j < 2 ? 64 : 0) + u;
    const float sgn = j < 2 ? -1.0f : 1.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = acc[j][i] + bb;
      const float mean = rf_sum8(v) * 0.125f;
      const float d = v - mean;
      const float var = rf_sum8(d * d) * 0.125f;
      const float y = d * __builtin_amdgcn_rsqf(var + 1e-5f) * gw + gb;
      zs[(32 * w + c_row(i, lane)) * RF_PZ + zc] = sgn * (y * __builtin_amdgcn_rcpf(1.0f + __expf(-y)));
    }
  }
  // ---- layer 2 chunks: dY, dW2, db2, dS_p ----
  f32x16 ds0 = {}, ds1 = {};   // dS_p [rows 32w ..][units lr, 32 + lr]
  for (int c = 0; c < nc; ++c) {
    rf_store2(ch, w2s);        // (the previous chunk's reads ended at the loop's last barrier)
    __syncthreads();           // Z (first chunk), this W2 chunk
    if (c + 1 < nc) rf_load2(ch, D, (c + 1) * RF_CC, tn.w2, pn.w2);
    const int col0 = c * RF_CC;
    f32x16 y0 = {}, y1 = {};
    {
      const float* az = zs + (32 * w + lr) * RF_PZ + lh;
      const float* b0 = w2s + lr * RF_PW + lh;
#pragma unroll
      for (int k0 = 0; k0 < 128; k0 += 32) {
        float a[16], c0[16], c1[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          a[k] = az[k0 + 2 * k];
          c0[k] = b0[k0 + 2 * k];
          c1[k] = b0[32 * RF_PW + k0 + 2 * k];
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          y0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], c0[k], y0, 0, 0, 0);
          y1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], c1[k], y1, 0, 0, 0);
        }
      }
    }
    const int col_a = col0 + lr, col_b = col_a + 32;
    const float bd_a = col_a < D ? pn.b2[col_a] - tn.b2[col_a] : 0.f;
    const float bd_b = col_b < D ? pn.b2[col_b] - tn.b2[col_b] : 0.f;
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = 32 * w + c_row(i, lane);
      const bool rin = row0 + r < n;
      const float da = (rin && col_a < D) ? scale * (y0[i] + bd_a) : 0.f;
      const float db = (rin && col_b < D) ? scale * (y1[i] + bd_b) : 0.f;
      dys[r * RG_PD + lr] = da;
      dys[r * RG_PD + 32 + lr] = db;
      sa += da;
      sb += db;
    }
    sa += __shfl_xor(sa, 32, 64);
    sb += __shfl_xor(sb, 32, 64);
    if (lh == 0) {
      cb[w * 64 + lr] = sa;
      cb[w * 64 + 32 + lr] = sb;
    }
    __syncthreads();           // dY, the column sums
    // dS_p += dY[rows of wave w][64 cols] . W2_p[cols][units] (K = the chunk's 64 columns)
    {
      const float* ad = dys + (32 * w + lr) * RG_PD + lh;
      const float* bw2 = w2s + lh * RF_PW + lr;
#pragma unroll
      for (int k0 = 0; k0 < 64; k0 += 16) {
        float a[8], b0v[8], b1v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          a[k] = ad[k0 + 2 * k];
          b0v[k] = bw2[(k0 + 2 * k) * RF_PW];
          b1v[k] = bw2[(k0 + 2 * k) * RF_PW + 32];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          ds0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], b0v[k], ds0, 0, 0, 0);
          ds1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], b1v[k], ds1, 0, 0, 0);
        }
      }
    }
    // dW2[col0 + 32 (w & 1) + m][32 (w >> 1) + unit] = sum over the 128 rows of dY[row][col] S_p[row][unit]
    {
      const int chf = w & 1, uh = w >> 1;
      const float* ad = dys + lh * RG_PD + 32 * chf + lr;
      const float* bz = zs + lh * RF_PZ + 32 * uh + lr;
      f32x16 t = {};
#pragma unroll
      for (int k0 = 0; k0 < 128; k0 += 32) {
        float a[16], b[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          a[k] = ad[(k0 + 2 * k) * RG_PD];
          b[k] = bz[(k0 + 2 * k) * RF_PZ];
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) t = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], b[k], t, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int col = col0 + 32 * chf + c_row(i, lane);
        if (col < D) pW2[(int64_t)col * 64 + 32 * uh + lr] = t[i];
      }
    }
    if (tid < 64 && col0 + tid < D)
      pb2[col0 + tid] = (cb[tid] + cb[64 + tid]) + (cb[128 + tid] + cb[192 + tid]);
    __syncthreads();           // every read of this W2 chunk, dY and cb done
  }
  // ---- GroupNorm + SiLU backward of the predictor's hidden layer (wave w: rows 32w .. 32w + 31) ----
  float sgw[2] = {0.f, 0.f}, sgb[2] = {0.f, 0.f}, sb1[2] = {0.f, 0.f};
  float* dhs = zs;   // Z's last reads (the last chunk's dW2) are behind the loop's last barrier
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int u = 32 * jj + lr;
    const float bb = pn.b1[u], gw = pn.gw[u], gb = pn.gb[u];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = acc[2 + jj][i] + bb;
      const float mean = rf_sum8(v) * 0.125f;
      const float d = v - mean;
      const float var = rf_sum8(d * d) * 0.125f;
      const float rs = __builtin_amdgcn_rsqf(var + 1e-5f);
      const float xh = d * rs;
      const float y = xh * gw + gb;
      const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-y));
      const float dsv = jj == 0 ? ds0[i] : ds1[i];
      const float dy = dsv * (sg * (1.0f + y * (1.0f - sg)));   // d silu(y) / dy
      const float dxh = dy * gw;
      const float m1 = rf_sum8(dxh) * 0.125f;
      const float m2 = rf_sum8(dxh * xh) * 0.125f;
      const float dv = rs * (dxh - m1 - xh * m2);
      sgw[jj] += dy * xh;
      sgb[jj] += dy;
      sb1[jj] += dv;
      dhs[(32 * w + c_row(i, lane)) * RG_PH + u] = dv;
    }
  }
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    sgw[jj] += __shfl_xor(sgw[jj], 32, 64);
    sgb[jj] += __shfl_xor(sgb[jj], 32, 64);
    sb1[jj] += __shfl_xor(sb1[jj], 32, 64);
    if (lh == 0) {
      cs[(w * 3 + 0) * 64 + 32 * jj + lr] = sb1[jj];
      cs[(w * 3 + 1) * 64 + 32 * jj + lr] = sgw[jj];
      cs[(w * 3 + 2) * 64 + 32 * jj + lr] = sgb[jj];
    }
  }
  float4 xv[4];
  rg_loadx(xv, x, n, D, row0, 0);
  __syncthreads();             // dH, the column sums
  if (tid < 3 * 64) {
    const int k = tid >> 6, u = tid & 63;
    const float v = (cs[(0 * 3 + k) * 64 + u] + cs[(1 * 3 + k) * 64 + u]) +
                    (cs[(2 * 3 + k) * 64 + u] + cs[(3 * 3 + k) * 64 + u]);
    (k == 0 ? pb1 : k == 1 ? pgw : pgb)[u] = v;
  }
  // ---- dW1[unit][col] = sum over the 128 rows of dH[row][unit] X[row][col], 32 columns a chunk ----
  const int x16 = lane & 15, q = lane >> 4;
  for (int c = 0; c < nk; ++c) {
    rg_storex(xv, xs);         // (the previous chunk's reads ended at the loop's last barrier)
    __syncthreads();
    if (c + 1 < nk) rg_loadx(xv, x, n, D, row0, (c + 1) * RF_KC);
    const float* ah = dhs + q * RG_PH + 16 * w + x16;
    const float* bxs = xs + q * RG_PX + x16;
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v u0 = {0.f, 0.f, 0.f, 0.f}, u1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < 128; k0 += 32) {
      float a[8], b0v[8], b1v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a[k] = ah[(k0 + 4 * k) * RG_PH];
        b0v[k] = bxs[(k0 + 4 * k) * RG_PX];
        b1v[k] = bxs[(k0 + 4 * k) * RG_PX + 16];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        u0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k], b0v[k], u0, 0, 0, 0);
        u1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k], b1v[k], u1, 0, 0, 0);
      }
    }
    const int colb = c * RF_KC + x16;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t urow = (int64_t)(16 * w + 4 * q + i) * D;
      if (colb < D) pW1[urow + colb] = u0[i];
      if (colb + 16 < D) pW1[urow + colb + 16] = u1[i];
    }
    __syncthreads();
  }
}

// grad[p] = sum over blocks of partial[b][p], in two passes for parallelism: pass 1, thread
// (4 consecutive p, segment g) sums blocks [g nblk / RG_SEG, (g + 1) nblk / RG_SEG) in f64 block
// order (16-B loads), into seg[g][p]; pass 2 adds the RG_SEG segments in order.  Deterministic.
constexpr int RG_SEG = 16;
__global__ __launch_bounds__(256) void rnd_grad_fold1_kernel(const float* __restrict__ partial, int64_t nblk,
                                                             int64_t P, double* __restrict__ seg) {
  const int64_t p4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int g = blockIdx.y;
  if (p4 >= P) return;
  const int64_t b0 = nblk * g / RG_SEG, b1 = nblk * (g + 1) / RG_SEG;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  for (int64_t b = b0; b < b1; ++b) {
    const float4 v = *reinterpret_cast<const float4*>(partial + b * P + p4);
    s0 += (double)v.x;
    s1 += (double)v.y;
    s2 += (double)v.z;
    s3 += (double)v.w;
  }
  double* o = seg + (int64_t)g * P + p4;
  o[0] = s0;
  o[1] = s1;
  o[2] = s2;
  o[3] = s3;
}
__global__ __launch_bounds__(256) void rnd_grad_fold2_kernel(const double* __restrict__ seg, int64_t P,
                                                             float* __restrict__ grad) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  double s = 0.0;
#pragma unroll
  for (int g = 0; g < RG_SEG; ++g) s += seg[(int64_t)g * P + p];
  grad[p] = (float)s;
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
  hipStream_t st = as_stream(stream);
  const bool fast = (D % 4) == 0 && aligned16(x) && aligned16(t_w1) && aligned16(p_w1) &&
                    aligned16(t_w2) && aligned16(p_w2) && getenv("PRL_RND_GENERIC") == nullptr;
  if (fast) {
    // persistent: one workgroup per CU (LDS-bound), each over its share of 128-row blocks
    static int cus = 0;
    if (cus == 0) {
      int dev = 0;
      PRL_HIP_TRY(hipGetDevice(&dev));
      PRL_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      PRL_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(rnd_forward_fast_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)(RF_LDS * sizeof(float))));
    }
    const int64_t nblocks = cdiv(n, RF_M);
    const unsigned grid = (unsigned)std::min<int64_t>(nblocks, cus);
    hipLaunchKernelGGL(rnd_forward_fast_kernel, dim3(grid), dim3(256), RF_LDS * sizeof(float), st, x, n,
                       (int)D, tn, pn, beta, out);
    PRL_LAUNCH_CHECK("rnd_forward_fast");
    return PRL_OK;
  }
  hipLaunchKernelGGL(rnd_forward_kernel, dim3((unsigned)cdiv(n, RB_M)), dim3(256), 0, st, x, n, (int)D,
                     tn, pn, beta, out);
  PRL_LAUNCH_CHECK("rnd_forward");
  return PRL_OK;
}

extern "C" int64_t prl_rnd_pred_grad_ws_floats(int64_t n, int32_t D) {
  if (n <= 0 || D <= 0) return 0;
  const int64_t P = 129 * (int64_t)D + 192;
  return cdiv(n, RF_M) * P + 2 * RG_SEG * P + 4;   // block partials | f64 segment sums (+ alignment)
}

extern "C" int prl_rnd_pred_grad(const float* x, int64_t n, int32_t D, const float* t_w1,
                                 const float* t_b1, const float* t_gw, const float* t_gb,
                                 const float* t_w2, const float* t_b2, const float* p_w1,
                                 const float* p_b1, const float* p_gw, const float* p_gb,
                                 const float* p_w2, const float* p_b2, float scale, float* partial,
                                 int64_t partial_floats, float* grad, void* stream) {
  PRL_REQUIRE(n >= 0 && D > 0, "prl_rnd_pred_grad: bad sizes");
  PRL_REQUIRE(D % 4 == 0, "prl_rnd_pred_grad: D = %d is not a multiple of 4", (int)D);
  const int64_t P = 129 * (int64_t)D + 192;
  PRL_REQUIRE(grad, "prl_rnd_pred_grad: null gradient");
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    PRL_HIP_TRY(hipMemsetAsync(grad, 0, P * sizeof(float), st));
    return PRL_OK;
  }
  PRL_REQUIRE(x && partial && t_w1 && t_b1 && t_gw && t_gb && t_w2 && t_b2 && p_w1 && p_b1 && p_gw &&
                  p_gb && p_w2 && p_b2,
              "prl_rnd_pred_grad: null pointer");
  PRL_REQUIRE(aligned16(x) && aligned16(t_w1) && aligned16(p_w1) && aligned16(t_w2) && aligned16(p_w2),
              "prl_rnd_pred_grad: x / W1 / W2 must be 16-B aligned");
  const int64_t nblk = cdiv(n, RF_M);
  PRL_REQUIRE(nblk < (int64_t)0x7fffffff, "prl_rnd_pred_grad: n too large");
  const int64_t need = nblk * P + 2 * RG_SEG * P + 4;
  PRL_REQUIRE(partial_floats >= need, "prl_rnd_pred_grad: partial buffer %lld < %lld floats",
              (long long)partial_floats, (long long)need);
  PRL_REQUIRE(aligned16(partial), "prl_rnd_pred_grad: partial must be 16-B aligned");
  static bool attr = false;
  if (!attr) {
    PRL_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(rnd_pred_grad_kernel),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)(RG_LDS * sizeof(float))));
    attr = true;
  }
  RndNet tn{t_w1, t_b1, t_gw, t_gb, t_w2, t_b2}, pn{p_w1, p_b1, p_gw, p_gb, p_w2, p_b2};
  hipLaunchKernelGGL(rnd_pred_grad_kernel, dim3((unsigned)nblk), dim3(256), RG_LDS * sizeof(float), st, x, n,
                     (int)D, tn, pn, scale, partial);
  PRL_LAUNCH_CHECK("rnd_pred_grad");
  // f64 segment sums after the block partials, 8-B aligned (P % 4 == 0: the partials end 16-B aligned)
  double* seg = reinterpret_cast<double*>(partial + nblk * P);
  hipLaunchKernelGGL(rnd_grad_fold1_kernel, dim3((unsigned)cdiv(P / 4, 256), RG_SEG), dim3(256), 0, st, partial,
                     nblk, P, seg);
  PRL_LAUNCH_CHECK("rnd_grad_fold1");
  hipLaunchKernelGGL(rnd_grad_fold2_kernel, dim3((unsigned)cdiv(P, 256)), dim3(256), 0, st, seg, P, grad);
  PRL_LAUNCH_CHECK("rnd_grad_fold2");
  return PRL_OK;
}
