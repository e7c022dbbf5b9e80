// prl_update.hip — pieces of the graph-captured PPO optimizer step (PPO/PPO.py:219-255).
//
// prl_gather_minibatch: the k_epochs x sequential, unshuffled minibatches of the reference
//   (batch_packer = DataLoader without shuffle, PPO.py:98-105, :202-211) are row ranges of the
//   env-major device tensors.  One captured graph serves every full minibatch: this kernel reads
//   the minibatch index from a device cursor and copies rows [cursor*mb, cursor*mb + mb) of up to
//   6 tensors into the graph's static inputs.
// prl_categorical_fwd / _bwd: Categorical(probs).log_prob(a) and .entropy() exactly as
//   torch.distributions.Categorical evaluates them (ActorCritic.py:105,136-142):
//     q = p / sum(p);  logits = log(clamp(q, eps, 1 - eps));  logp = logits[a];
//     H = -sum_k logits_k * q_k  (detached in the reference, so no gradient)
//   and d logp / d p_j = m_a * (delta_aj / q_a - 1) / sum(p), m_a = [eps <= q_a <= 1 - eps]
//   (clamp passes the gradient on the closed interval).
#include "prl_common.h"

#include <float.h>

#include <algorithm>

namespace prl {

constexpr int GATHER_MAX = 6;
struct GatherArgs {
  const float* src[GATHER_MAX];
  float* dst[GATHER_MAX];
  int32_t width[GATHER_MAX];
  int32_t count;
};

// 16-B copies (4 quads in flight per thread per pass) wherever the tensor's rows are 16-B
// aligned, element copies otherwise; rows past nrows are zero-filled (the ragged last minibatch)
__global__ __launch_bounds__(256) void gather_minibatch_kernel(GatherArgs a, const int64_t* cursor,
                                                               int64_t mb, int64_t nrows) {
  const int64_t base = cursor[0] * mb;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int t = 0; t < a.count; ++t) {
    const int w = a.width[t];
    const int64_t total = mb * w;
    const float* src = a.src[t] + base * w;
    float* dst = a.dst[t];
    const int64_t limit = (nrows - base) * w;  // never read past the source
    const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
    int64_t done = 0;
    if (vec) {
      const int64_t nq = total / 4;
      const float4* s4 = reinterpret_cast<const float4*>(src);
      float4* d4 = reinterpret_cast<float4*>(dst);
      for (int64_t q0 = tid; q0 < nq; q0 += 4 * nthreads) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t q = q0 + u * nthreads;
          if (q < nq) {
            if (4 * q + 3 < limit) {
              v[u] = s4[q];
            } else {
              const int64_t i = 4 * q;
              v[u].x = i < limit ? src[i] : 0.0f;
              v[u].y = i + 1 < limit ? src[i + 1] : 0.0f;
              v[u].z = i + 2 < limit ? src[i + 2] : 0.0f;
              v[u].w = i + 3 < limit ? src[i + 3] : 0.0f;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t q = q0 + u * nthreads;
          if (q < nq) d4[q] = v[u];
        }
      }
      done = nq * 4;
    }
    for (int64_t i = done + tid; i < total; i += nthreads) dst[i] = i < limit ? src[i] : 0.0f;
  }
}

__global__ __launch_bounds__(256) void categorical_fwd_kernel(const float* __restrict__ probs,
                                                              const float* __restrict__ actions,
                                                              int64_t n, int A,
                                                              float* __restrict__ logp,
                                                              float* __restrict__ entropy) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* p = probs + i * A;
  float S = 0.f;
  for (int k = 0; k < A; ++k) S += p[k];
  const int a = (int)(int64_t)actions[i];  // value.long()
  if (a < 0 || a >= A) {  // torch's gather would fault; flag the row instead of reading OOB
    logp[i] = __builtin_nanf("");
    if (entropy) entropy[i] = __builtin_nanf("");
    return;
  }
  float h = 0.f, la = 0.f;
  for (int k = 0; k < A; ++k) {
    const float q = p[k] / S;
    const float c = q < FLT_EPSILON ? FLT_EPSILON : (q > 1.0f - FLT_EPSILON ? 1.0f - FLT_EPSILON : q);
    const float l = logf(c);
    if (k == a) la = l;
    h += l * q;
  }
  logp[i] = la;
  if (entropy) entropy[i] = -h;
}

__global__ __launch_bounds__(256) void categorical_bwd_kernel(const float* __restrict__ probs,
                                                              const float* __restrict__ actions,
                                                              const float* __restrict__ dlogp,
                                                              int64_t n, int A,
                                                              float* __restrict__ dprobs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* p = probs + i * A;
  float S = 0.f;
  for (int k = 0; k < A; ++k) S += p[k];
  const int a = (int)(int64_t)actions[i];
  if (a < 0 || a >= A) {
    for (int k = 0; k < A; ++k) dprobs[i * A + k] = __builtin_nanf("");
    return;
  }
  const float qa = p[a] / S;
  const float m = (qa >= FLT_EPSILON && qa <= 1.0f - FLT_EPSILON) ? 1.0f : 0.0f;
  const float g = dlogp[i] * m;
  for (int k = 0; k < A; ++k) dprobs[i * A + k] = g * (((k == a) ? 1.0f / qa : 0.0f) - 1.0f) / S;
}

// Column sums of a row-major [rows][cols] f32 matrix (the bias gradient 1^T dy of a Linear over
// a large batch).  Block (window, b) sums columns [W window, W window + W) over its contiguous
// row chunk: W = cols (<= 64, 256 / W row slots) or 64 (4 row slots), so each sweep reads whole
// 64-float row segments; the slots are combined in LDS in a fixed order into partial[b][cols].
// Pass 2 is the same kernel over the [nblk][cols] partials with one row chunk.  Deterministic and
// graph-capturable.  Rows per thread in pass 1 = chunk / slots, chunk = max(slots, ceil(16384 / W))
// grown to ceil(rows / 256) once more than 256 row chunks would be needed: 64 up to 65,536 rows
// (cols > 64), max(64, rows / (256 slots)) beyond (rows = 2^20, cols = 348: 1,024); pass 2 loops
// over at most 256 / slots partial rows per thread.
constexpr int CS_THREADS = 256;
constexpr int CS_MAXBLK = 256;
__host__ __device__ inline int cs_width(int cols) { return cols <= 64 ? cols : 64; }
__global__ __launch_bounds__(CS_THREADS) void colsum_partial_kernel(const float* __restrict__ x,
                                                                    int64_t rows, int cols,
                                                                    int64_t chunk,
                                                                    float* __restrict__ partial) {
  __shared__ float s_acc[CS_THREADS];
  const int t = threadIdx.x, W = cs_width(cols), slots = CS_THREADS / W;
  const int slot = t / W, c = blockIdx.x * W + t % W;
  const int64_t r0 = (int64_t)blockIdx.y * chunk, r1 = std::min(rows, r0 + chunk);
  float acc = 0.f;
  if (slot < slots && c < cols) {
#pragma unroll 8
    for (int64_t r = r0 + slot; r < r1; r += slots) acc += x[r * cols + c];
  }
  s_acc[t] = acc;
  __syncthreads();
  if (t < W && c < cols) {
    float sum = 0.f;
    for (int k = 0; k < slots; ++k) sum += s_acc[k * W + t];
    partial[(int64_t)blockIdx.y * cols + c] = sum;
  }
}
inline int64_t colsum_chunk(int64_t rows, int cols) {
  const int W = cs_width(cols);
  int64_t chunk = std::max<int64_t>(CS_THREADS / W, (16384 + W - 1) / W);
  if ((rows + chunk - 1) / chunk > CS_MAXBLK) chunk = (rows + CS_MAXBLK - 1) / CS_MAXBLK;
  return chunk;
}
inline int colsum_blocks(int64_t rows, int cols) {
  return (int)std::max<int64_t>(1, (rows + colsum_chunk(rows, cols) - 1) / colsum_chunk(rows, cols));
}

}  // namespace prl

using namespace prl;

extern "C" int prl_gather_minibatch(const float* const* srcs, float* const* dsts,
                                    const int32_t* widths, int32_t count, const int64_t* cursor,
                                    int64_t mb, int64_t nrows, void* stream) {
  PRL_REQUIRE(count > 0 && count <= GATHER_MAX, "prl_gather_minibatch: 1..6 tensors");
  PRL_REQUIRE(srcs && dsts && widths && cursor && mb > 0, "prl_gather_minibatch: bad arguments");
  GatherArgs a{};
  a.count = count;
  for (int t = 0; t < count; ++t) {
    PRL_REQUIRE(srcs[t] && dsts[t] && widths[t] > 0, "prl_gather_minibatch: tensor %d", t);
    a.src[t] = srcs[t];
    a.dst[t] = dsts[t];
    a.width[t] = widths[t];
  }
  int64_t widest = 1;
  for (int t = 0; t < count; ++t) widest = std::max<int64_t>(widest, widths[t]);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(mb * widest, 4 * 256 * 4), 1024));
  hipLaunchKernelGGL(gather_minibatch_kernel, dim3(grid), dim3(256), 0, as_stream(stream), a,
                     cursor, mb, nrows);
  PRL_LAUNCH_CHECK("gather_minibatch");
  return PRL_OK;
}

extern "C" int prl_categorical_fwd(const float* probs, const float* actions, int64_t n, int32_t A,
                                   float* logp, float* entropy, void* stream) {
  PRL_REQUIRE(n >= 0 && A >= 1, "prl_categorical_fwd: bad sizes");
  if (n == 0) return PRL_OK;
  PRL_REQUIRE(probs && actions && logp, "prl_categorical_fwd: null pointer");
  hipLaunchKernelGGL(categorical_fwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), probs, actions, n, (int)A, logp, entropy);
  PRL_LAUNCH_CHECK("categorical_fwd");
  return PRL_OK;
}

extern "C" int prl_categorical_bwd(const float* probs, const float* actions, const float* dlogp,
                                   int64_t n, int32_t A, float* dprobs, void* stream) {
  PRL_REQUIRE(n >= 0 && A >= 1, "prl_categorical_bwd: bad sizes");
  if (n == 0) return PRL_OK;
  PRL_REQUIRE(probs && actions && dlogp && dprobs, "prl_categorical_bwd: null pointer");
  hipLaunchKernelGGL(categorical_bwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), probs, actions, dlogp, n, (int)A, dprobs);
  PRL_LAUNCH_CHECK("categorical_bwd");
  return PRL_OK;
}

extern "C" int64_t prl_colsum_partial_floats(int64_t rows, int32_t cols) {
  if (rows <= 0 || cols <= 0) return 0;
  return (int64_t)colsum_blocks(rows, cols) * cols;
}

extern "C" int prl_colsum_f32(const float* x, int64_t rows, int32_t cols, float* out,
                              float* partial, int64_t partial_floats, void* stream) {
  PRL_REQUIRE(rows >= 0 && cols > 0, "prl_colsum_f32: bad sizes");
  PRL_REQUIRE(out && (rows == 0 || (x && partial)), "prl_colsum_f32: null pointer");
  hipStream_t st = as_stream(stream);
  if (rows == 0) {
    PRL_HIP_TRY(hipMemsetAsync(out, 0, sizeof(float) * cols, st));
    return PRL_OK;
  }
  const int nblk = colsum_blocks(rows, cols);
  PRL_REQUIRE(partial_floats >= (int64_t)nblk * cols, "prl_colsum_f32: partial buffer too small");
  const unsigned windows = (unsigned)cdiv((int64_t)cols, (int64_t)cs_width(cols));
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(windows, nblk), dim3(CS_THREADS), 0, st, x, rows,
                     (int)cols, colsum_chunk(rows, cols), partial);
  PRL_LAUNCH_CHECK("colsum_partial");
  // pass 2: the same kernel over the [nblk][cols] partials as one row chunk (block order fixed)
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(windows, 1), dim3(CS_THREADS), 0, st, partial,
                     (int64_t)nblk, (int)cols, (int64_t)nblk, out);
  PRL_LAUNCH_CHECK("colsum_fold");
  return PRL_OK;
}

// ---- clip_grad_norm_ + AdamW over flat buffers (the wide step's optimizer tail) --------------
// PPO.py:248-250: nn.utils.clip_grad_norm_(policy.parameters(), max_norm) then AdamW.step()
// (torch defaults: decoupled weight decay, lerp for exp_avg, addcmul for exp_avg_sq, bias
// corrections from the incremented step count).  Parameters, gradient and both moments are flat
// vectors in parameters() order (the policy's Parameters and the optimizer's state are views of
// them, PPO/update.py FlatAdamState).  flat_adamw_kernel (below) forms the squared norm in float64
// in a fixed order in EVERY workgroup, the clip coefficient max_norm / (norm + 1e-6) clamped to 1,
// and updates its own 1,024 quads of params / exp_avg / exp_avg_sq with the persistent engine's
// arithmetic (prl_ppo_update.hip phase C); workgroup 0 stores the norm.  The gradient must then be
// left clipped (as torch leaves p.grad) and the step count advanced, which no workgroup may do
// while another is still reading the gradient for its norm or the step for its bias corrections:
// the LAST workgroup to finish (an arrival counter in the norm workspace, left at zero again) does
// both, so one launch replaces torch's foreach-norm / stack / norm / coefficient / foreach-mul /
// fused-AdamW chain.  Large P (> FA_FUSE_MAX_BLOCKS workgroups, where one workgroup's pass over
// the whole gradient would be long) keeps a second launch for it (flat_adam_clip_kernel).
constexpr int FA_THREADS = 1024;
constexpr int FA_BATCH = 8;   // gradient quads per thread in flight during the norm pass
constexpr int FA_FUSE_MAX_BLOCKS = 64;   // up to 262,144 parameters: clip + step in the last workgroup

// Every workgroup forms the whole squared norm itself, in the same fixed order (thread t: quads
// t, t + 1024, ... ascending, float64 fma; the 16 waves' sums in wave order), so all of them get
// the same clip coefficient with no exchange; workgroup b then updates quads b*1024 + t (and the
// last one the P % 4 tail).  (Until round 4 one 1024-thread workgroup did the norm AND the whole
// update: ~19 us per C5 step, most of it one CU streaming ~600 KB in and out.)
__global__ __launch_bounds__(FA_THREADS) void flat_adamw_kernel(
    float* __restrict__ p, float* __restrict__ m, float* __restrict__ v, const float* step,
    const float* grad, int64_t P, float lr, double beta1, double beta2, float eps,
    float wd, float max_norm, float* __restrict__ total_norm, float* grad_out,
    unsigned* arrive, float* step_out) {   // grad_out / step_out: grad / step (written last)
  __shared__ double s_part[FA_THREADS / 64];
  __shared__ float s_c[3];
  __shared__ unsigned s_last;
  const int t = threadIdx.x;
  const int64_t Q = P / 4;
  const float4* g4p = reinterpret_cast<const float4*>(grad);
  double acc = 0.0;
  for (int64_t q0 = t; q0 < Q; q0 += (int64_t)FA_BATCH * FA_THREADS) {
    float4 x[FA_BATCH];
#pragma unroll
    for (int i = 0; i < FA_BATCH; ++i) {
      const int64_t q = q0 + (int64_t)i * FA_THREADS;
      x[i] = q < Q ? g4p[q] : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < FA_BATCH; ++i) {
      if (q0 + (int64_t)i * FA_THREADS < Q) {
        acc = fma((double)x[i].x, (double)x[i].x, acc);
        acc = fma((double)x[i].y, (double)x[i].y, acc);
        acc = fma((double)x[i].z, (double)x[i].z, acc);
        acc = fma((double)x[i].w, (double)x[i].w, acc);
      }
    }
  }
  for (int64_t k = 4 * Q + t; k < P; k += FA_THREADS) acc = fma((double)grad[k], (double)grad[k], acc);
  acc = wave_sum(acc);
  if ((t & 63) == 0) s_part[t >> 6] = acc;
  const float step0 = step[0];
  // this workgroup's quad and its operands, loaded under the norm's reduction
  const int64_t qm = (int64_t)blockIdx.x * FA_THREADS + t;
  const bool mine = qm < Q;
  float4 g4 = {0.f, 0.f, 0.f, 0.f}, p4 = g4, m4 = g4, v4 = g4;
  if (mine) {
    g4 = g4p[qm];
    p4 = reinterpret_cast<const float4*>(p)[qm];
    m4 = reinterpret_cast<const float4*>(m)[qm];
    v4 = reinterpret_cast<const float4*>(v)[qm];
  }
  __syncthreads();
  if (t == 0) {
    double tot = 0.0;
    for (int w = 0; w < FA_THREADS / 64; ++w) tot += s_part[w];
    const float norm = (float)sqrt(tot);
    const float coef = max_norm / (norm + 1e-6f);
    s_c[0] = coef < 1.0f ? coef : 1.0f;
    if (blockIdx.x == 0) total_norm[0] = norm;
    const double tstep = (double)step0 + 1.0;
    s_c[1] = (float)((double)lr / (1.0 - pow((double)beta1, tstep)));    // step size
    s_c[2] = (float)(1.0 / sqrt(1.0 - pow((double)beta2, tstep)));       // 1 / sqrt(bc2)
  }
  __syncthreads();
  const float clipc = s_c[0], step_size = s_c[1], inv_bc2_sqrt = s_c[2];
  const float decay = (float)(1.0 - (double)lr * (double)wd);
  // 1 - beta from the caller's double betas (torch forms them in Python double precision)
  const float omb1 = (float)(1.0 - beta1), omb2 = (float)(1.0 - beta2), b2 = (float)beta2;
  auto upd = [&](float g, float& pw, float& mw, float& vw) {
    const float gr = g * clipc;
    pw = pw * decay;
    mw = fmaf(omb1, gr - mw, mw);
    vw = fmaf(omb2 * gr, gr, vw * b2);
    const float denom = fmaf(__builtin_amdgcn_sqrtf(vw), inv_bc2_sqrt, eps);
    float rq = __builtin_amdgcn_rcpf(denom);
    rq = fmaf(rq, fmaf(-denom, rq, 1.0f), rq);   // one Newton step: ~0.5 ulp
    pw = fmaf(-step_size, mw * rq, pw);
  };
  if (mine) {
    upd(g4.x, p4.x, m4.x, v4.x);
    upd(g4.y, p4.y, m4.y, v4.y);
    upd(g4.z, p4.z, m4.z, v4.z);
    upd(g4.w, p4.w, m4.w, v4.w);
    reinterpret_cast<float4*>(p)[qm] = p4;
    reinterpret_cast<float4*>(m)[qm] = m4;
    reinterpret_cast<float4*>(v)[qm] = v4;
  }
  if (blockIdx.x + 1 == gridDim.x) {   // the P % 4 tail
    for (int64_t k = 4 * Q + t; k < P; k += FA_THREADS) {
      float pw = p[k], mw = m[k], vw = v[k];
      upd(grad[k], pw, mw, vw);
      p[k] = pw;
      m[k] = mw;
      v[k] = vw;
    }
  }
  if (arrive == nullptr) return;   // the clip launch follows
  // every read of grad and step in this workgroup is complete here (all consumed above)
  __syncthreads();
  if (t == 0) {
    const unsigned old = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old + 1 == gridDim.x) ? 1u : 0u;
  }
  __syncthreads();
  if (!s_last) return;
  if (clipc != 1.0f) {   // x * 1 is x: an unclipped gradient is left as it is
    float4* go4 = reinterpret_cast<float4*>(grad_out);
    for (int64_t q = t; q < Q; q += FA_THREADS) {
      float4 x = go4[q];
      x.x *= clipc;
      x.y *= clipc;
      x.z *= clipc;
      x.w *= clipc;
      go4[q] = x;
    }
    for (int64_t k = 4 * Q + t; k < P; k += FA_THREADS) grad_out[k] *= clipc;
  }
  if (t == 0) {
    step_out[0] = step0 + 1.0f;
    __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// grad *= the clip coefficient (from the stored norm, formed as flat_adamw_kernel formed it:
// the same bits); thread 0 of workgroup 0 advances the step count
__global__ __launch_bounds__(256) void flat_adam_clip_kernel(float* __restrict__ grad, int64_t P,
                                                             float max_norm,
                                                             const float* __restrict__ total_norm,
                                                             float* __restrict__ step) {
  const float coef = max_norm / (total_norm[0] + 1e-6f);
  const float clipc = coef < 1.0f ? coef : 1.0f;
  const int64_t Q = P / 4, q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q < Q) {
    float4 g = reinterpret_cast<const float4*>(grad)[q];
    g.x *= clipc;
    g.y *= clipc;
    g.z *= clipc;
    g.w *= clipc;
    reinterpret_cast<float4*>(grad)[q] = g;
  }
  if (blockIdx.x == 0) {
    for (int64_t k = 4 * Q + threadIdx.x; k < P; k += 256) grad[k] *= clipc;
    if (threadIdx.x == 0) step[0] = step[0] + 1.0f;
  }
}

extern "C" int prl_flat_adamw(float* params, float* exp_avg, float* exp_avg_sq, float* step,
                              float* grad, int64_t P, float lr, double beta1, double beta2, float eps,
                              float weight_decay, float max_norm, float* total_norm, void* stream) {
  PRL_REQUIRE(P > 0 && P < (int64_t)1 << 30, "prl_flat_adamw: bad size %lld", (long long)P);
  PRL_REQUIRE(params && exp_avg && exp_avg_sq && step && grad && total_norm, "prl_flat_adamw: null pointer");
  PRL_REQUIRE(aligned16(params) && aligned16(exp_avg) && aligned16(exp_avg_sq) && aligned16(grad),
              "prl_flat_adamw: buffers must be 16-B aligned");
  const unsigned nblk = (unsigned)std::max<int64_t>(1, cdiv(P / 4, FA_THREADS));
  const bool fuse = nblk <= (unsigned)FA_FUSE_MAX_BLOCKS;
  // total_norm[1]: the arrival counter, zero before a buffer's first call (prl_native.flat_adamw
  // zeroes a caller's buffer once, on first use) and left zero by every call.  (Not a
  // hipMemsetAsync per call: captured into the data-parallel ranks' optimizer graph, that memset
  // node broke the step — tests/test_distributed_gpu.py::test_two_ranks_wide_step_equal_one_
  // process_on_the_union, 4.7e-3 vs 1e-3, round 6.)
  unsigned* arrive = fuse ? reinterpret_cast<unsigned*>(total_norm + 1) : nullptr;
  hipLaunchKernelGGL(flat_adamw_kernel, dim3(nblk), dim3(FA_THREADS), 0, as_stream(stream), params,
                     exp_avg, exp_avg_sq, step, grad, P, lr, beta1, beta2, eps, weight_decay,
                     max_norm, total_norm, grad, arrive, step);
  PRL_LAUNCH_CHECK("flat_adamw");
  if (fuse) return PRL_OK;
  hipLaunchKernelGGL(flat_adam_clip_kernel, dim3((unsigned)std::max<int64_t>(1, cdiv(P / 4, 256))),
                     dim3(256), 0, as_stream(stream), grad, P, max_norm, total_norm, step);
  PRL_LAUNCH_CHECK("flat_adam_clip");
  return PRL_OK;
}
