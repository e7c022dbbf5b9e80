// prl_buffers.hip — envs_active mask utilities, ordered compaction, scans and the env-major
// flatten that hands a rollout to PPO.learn.
//
// Replaces AsyncTools/utils.py:
//   indexes_of_active_environments / number_of_active_environments (:3-7)  -> prl_active_indices
//   inactive_states_dropout (:14-15)                                       -> prl_compact_rows
//   update_active_environments_list (:38-43)                               -> prl_mask_update
//   buffer_to_target_buffer_transfer (:45-51) (env-major `sum(list, [])`)  -> prl_exclusive_scan_i32
//                                                                            + prl_flatten_env_major
// Ordered (stable) compaction and scans are the classic three-phase form: per-block totals,
// one-block scan of the totals, per-block local scan + scatter.  Bit-exact by construction
// (integer work only).  The flatten is a gather: one thread (small rows) or one wave (wide rows)
// per OUTPUT row, so the env-major output is written fully coalesced; the env of a row comes from
// a binary search of the episode offsets, narrowed per block.
#include "prl_common.h"

#include <algorithm>

namespace prl {

constexpr int SC_THREADS = 256;
constexpr int SC_EPT = 8;
constexpr int SC_CHUNK = SC_THREADS * SC_EPT;

struct ScanWs {
  int64_t* bsum;   // [nb]
  int64_t* boff;   // [nb]
  int64_t* count;  // [2]
  int64_t* idx;    // [n] (mask update scratch)
};
inline int64_t scan_nb(int64_t n) { return cdiv(std::max<int64_t>(n, 1), SC_CHUNK); }
inline int64_t scan_ws_bytes(int64_t n) {
  const int64_t nb = scan_nb(n);
  return 16 * nb + 16 + 8 * std::max<int64_t>(n, 1) + 16;
}
inline ScanWs scan_ws_carve(void* ws, int64_t n) {
  const int64_t nb = scan_nb(n);
  int64_t* p = static_cast<int64_t*>(ws);
  return ScanWs{p, p + nb, p + 2 * nb, p + 2 * nb + 2};
}

// value of item i for each op
struct OpScanI32 {
  const int32_t* in;
  int64_t* offsets;
  __device__ int64_t value(int64_t i) const { return (int64_t)in[i]; }
  __device__ void emit(int64_t i, int64_t prefix, int64_t) const { offsets[i] = prefix; }
};
struct OpActive {
  const uint8_t* terminal;
  int64_t* idx_out;
  __device__ int64_t value(int64_t i) const { return terminal[i] == 0 ? 1 : 0; }
  __device__ void emit(int64_t i, int64_t prefix, int64_t v) const {
    if (v) idx_out[prefix] = i;
  }
};
struct OpCompact {
  const uint8_t* src;
  uint8_t* dst;
  const uint8_t* drop;
  int64_t row_bytes;
  __device__ int64_t value(int64_t i) const { return drop[i] == 0 ? 1 : 0; }
  __device__ void emit(int64_t i, int64_t prefix, int64_t v) const {
    if (!v) return;
    const uint8_t* s = src + i * row_bytes;
    uint8_t* d = dst + prefix * row_bytes;
    if ((row_bytes & 3) == 0 && ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 3) == 0) {
      for (int64_t b = 0; b < row_bytes; b += 4)
        *reinterpret_cast<uint32_t*>(d + b) = *reinterpret_cast<const uint32_t*>(s + b);
    } else {
      for (int64_t b = 0; b < row_bytes; ++b) d[b] = s[b];
    }
  }
};

template <class Op>
__global__ __launch_bounds__(SC_THREADS) void block_sum_kernel(Op op, int64_t n, int64_t* bsum) {
  const int64_t base = (int64_t)blockIdx.x * SC_CHUNK;
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < SC_EPT; ++k) {
    const int64_t i = base + (int64_t)k * SC_THREADS + threadIdx.x;
    if (i < n) acc += op.value(i);
  }
  __shared__ int64_t s_w[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// one block: exclusive scan of nb block totals; total -> count[0] (and, if given, extra_total)
__global__ __launch_bounds__(SC_THREADS) void scan_totals_kernel(const int64_t* bsum, int64_t nb,
                                                                 int64_t* boff, int64_t* count,
                                                                 int64_t* extra_total) {
  __shared__ int64_t s_w[4];
  const int64_t per = cdiv(nb, SC_THREADS);
  const int64_t lo = std::min<int64_t>((int64_t)threadIdx.x * per, nb);
  const int64_t hi = std::min<int64_t>(lo + per, nb);
  int64_t acc = 0;
  for (int64_t b = lo; b < hi; ++b) acc += bsum[b];
  int64_t total;
  const int64_t incl = block_inclusive_scan_256(acc, s_w, total);
  int64_t run = incl - acc;
  for (int64_t b = lo; b < hi; ++b) {
    boff[b] = run;
    run += bsum[b];
  }
  if (threadIdx.x == 0) {
    count[0] = total;
    if (extra_total) *extra_total = total;
  }
}

template <class Op>
__global__ __launch_bounds__(SC_THREADS) void scatter_kernel(Op op, int64_t n, const int64_t* boff) {
  __shared__ int64_t s_w[4];
  const int64_t base = (int64_t)blockIdx.x * SC_CHUNK + (int64_t)threadIdx.x * SC_EPT;  // blocked
  int64_t v[SC_EPT];
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < SC_EPT; ++k) {
    const int64_t i = base + k;
    v[k] = (i < n) ? op.value(i) : 0;
    acc += v[k];
  }
  int64_t total;
  const int64_t incl = block_inclusive_scan_256(acc, s_w, total);
  int64_t run = incl - acc + boff[blockIdx.x];
#pragma unroll
  for (int k = 0; k < SC_EPT; ++k) {
    const int64_t i = base + k;
    if (i < n) op.emit(i, run, v[k]);
    run += v[k];
  }
}

template <class Op>
int run_ordered_scan(Op op, int64_t n, void* workspace, int64_t* extra_total, hipStream_t s) {
  ScanWs ws = scan_ws_carve(workspace, n);
  const int64_t nb = scan_nb(n);
  if (n > 0) {
    hipLaunchKernelGGL(block_sum_kernel<Op>, dim3((unsigned)nb), dim3(SC_THREADS), 0, s, op, n, ws.bsum);
    PRL_LAUNCH_CHECK("block_sum");
  } else {
    PRL_HIP_TRY(hipMemsetAsync(ws.bsum, 0, sizeof(int64_t), s));
  }
  hipLaunchKernelGGL(scan_totals_kernel, dim3(1), dim3(SC_THREADS), 0, s, ws.bsum, nb, ws.boff,
                     ws.count, extra_total);
  PRL_LAUNCH_CHECK("scan_totals");
  if (n > 0) {
    hipLaunchKernelGGL(scatter_kernel<Op>, dim3((unsigned)nb), dim3(SC_THREADS), 0, s, op, n, ws.boff);
    PRL_LAUNCH_CHECK("scatter");
  }
  return PRL_OK;
}

__global__ void mask_update_kernel(uint8_t* terminal, const int64_t* idx, const int64_t* count,
                                   const uint8_t* dones, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t m = std::min<int64_t>(n, count[0]);
  if (i < m) terminal[idx[i]] = dones[i] ? 1 : 0;
}

// ---- flatten ------------------------------------------------------------------------------
__device__ inline int64_t upper_bound_i64(const int64_t* a, int64_t lo, int64_t hi, int64_t key) {
  // first index in [lo, hi) with a[idx] > key
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

struct FlattenArgs {
  int64_t E;
  int32_t D, Adim;
  const int64_t* offsets;  // [E+1]
  int64_t N;
  const float* traj_obs;
  const float* traj_act;
  const float* traj_rew;
  const uint8_t* traj_done;
  float *S, *A, *R, *Dn;
};

// rows handled by this block: [r0, r1); returns env search window via LDS
__device__ inline void block_env_window(const FlattenArgs& a, int64_t r0, int64_t r1, int64_t* s_win) {
  if (threadIdx.x == 0) {
    s_win[0] = upper_bound_i64(a.offsets, 0, a.E + 1, r0) - 1;
    s_win[1] = upper_bound_i64(a.offsets, 0, a.E + 1, r1 - 1);  // exclusive
  }
  __syncthreads();
}

__device__ inline void flatten_scalars(const FlattenArgs& a, int64_t row, int64_t e, int64_t t) {
  const int64_t slot = t * a.E + e;
  a.R[row] = a.traj_rew[slot];
  a.Dn[row] = a.traj_done[slot] ? 1.0f : 0.0f;
}

// thread per output row (obs rows of <= 32 floats)
__global__ __launch_bounds__(256) void flatten_rows_kernel(FlattenArgs a) {
  __shared__ int64_t s_win[2];
  const int64_t r0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t r1 = std::min<int64_t>(r0 + blockDim.x, a.N);
  block_env_window(a, r0, r1, s_win);
  const int64_t row = r0 + threadIdx.x;
  if (row >= a.N) return;
  const int64_t e = upper_bound_i64(a.offsets, s_win[0], s_win[1], row) - 1;
  const int64_t t = row - a.offsets[e];
  const float* src = a.traj_obs + (t * a.E + e) * a.D;
  float* dst = a.S + row * a.D;
  if (a.D == 4) {
    *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
  } else {
    for (int k = 0; k < a.D; ++k) dst[k] = src[k];
  }
  const float* asrc = a.traj_act + (t * a.E + e) * a.Adim;
  for (int k = 0; k < a.Adim; ++k) a.A[row * a.Adim + k] = asrc[k];
  flatten_scalars(a, row, e, t);
}

// wave per output row (wide obs rows, e.g. the 348-float synthetic env); VEC: 16-B moves (D % 4
// == 0, 16-B aligned buffers: 87 float4 per 348-float row instead of 348 4-B words — the 4-B form
// moved ~2.2 TB/s at C5's 323 K rows)
template <bool VEC>
__global__ __launch_bounds__(256) void flatten_wide_kernel(FlattenArgs a) {
  __shared__ int64_t s_win[2];
  const int64_t r0 = (int64_t)blockIdx.x * 4;
  const int64_t r1 = std::min<int64_t>(r0 + 4, a.N);
  block_env_window(a, r0, r1, s_win);
  const int64_t row = r0 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.N) return;
  const int64_t e = upper_bound_i64(a.offsets, s_win[0], s_win[1], row) - 1;
  const int64_t t = row - a.offsets[e];
  const float* src = a.traj_obs + (t * a.E + e) * a.D;
  float* dst = a.S + row * a.D;
  if (VEC) {
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int k = lane; k < (a.D >> 2); k += 64) d4[k] = s4[k];
  } else {
    for (int k = lane; k < a.D; k += 64) dst[k] = src[k];
  }
  const float* asrc = a.traj_act + (t * a.E + e) * a.Adim;
  for (int k = lane; k < a.Adim; k += 64) a.A[row * a.Adim + k] = asrc[k];
  if (lane == 0) flatten_scalars(a, row, e, t);
}

}  // namespace prl

using namespace prl;

int64_t prl_scan_workspace_bytes(int64_t n) { return scan_ws_bytes(n); }

extern "C" int prl_exclusive_scan_i32(const int32_t* in, int64_t n, int64_t* offsets,
                                      void* workspace, void* stream) {
  PRL_REQUIRE(n >= 0, "prl_exclusive_scan_i32: n < 0");
  PRL_REQUIRE(offsets && workspace && (n == 0 || in), "prl_exclusive_scan_i32: null pointer");
  return run_ordered_scan(OpScanI32{in, offsets}, n, workspace, offsets + n, as_stream(stream));
}

extern "C" int prl_active_indices(const uint8_t* terminal, int64_t E, int64_t* idx_out,
                                  int64_t* count_out, void* workspace, void* stream) {
  PRL_REQUIRE(E >= 0, "prl_active_indices: E < 0");
  PRL_REQUIRE(workspace && count_out && (E == 0 || (terminal && idx_out)),
              "prl_active_indices: null pointer");
  return run_ordered_scan(OpActive{terminal, idx_out}, E, workspace, count_out, as_stream(stream));
}

extern "C" int prl_compact_rows(const void* src, int64_t rows, int64_t row_bytes,
                                const uint8_t* drop, void* dst, int64_t* count_out,
                                void* workspace, void* stream) {
  PRL_REQUIRE(rows >= 0 && row_bytes >= 0, "prl_compact_rows: bad sizes");
  PRL_REQUIRE(workspace && count_out && (rows == 0 || (src && drop && dst)),
              "prl_compact_rows: null pointer");
  return run_ordered_scan(OpCompact{static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst),
                                    drop, row_bytes},
                          rows, workspace, count_out, as_stream(stream));
}

extern "C" int prl_mask_update(uint8_t* terminal, int64_t E, const uint8_t* dones, int64_t n,
                               void* workspace, void* stream) {
  PRL_REQUIRE(E >= 0 && n >= 0 && n <= E, "prl_mask_update: bad sizes");
  PRL_REQUIRE(workspace && (E == 0 || terminal) && (n == 0 || dones), "prl_mask_update: null pointer");
  if (E == 0 || n == 0) return PRL_OK;
  hipStream_t s = as_stream(stream);
  ScanWs ws = scan_ws_carve(workspace, E);
  int rc = run_ordered_scan(OpActive{terminal, ws.idx}, E, workspace, nullptr, s);
  if (rc) return rc;
  hipLaunchKernelGGL(mask_update_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, terminal,
                     ws.idx, ws.count, dones, n);
  PRL_LAUNCH_CHECK("mask_update");
  return PRL_OK;
}

extern "C" int prl_flatten_env_major(int64_t E, int32_t t_max, int32_t D, int32_t Adim,
                                     const int64_t* offsets, int64_t N, const float* traj_obs,
                                     const float* traj_act, const float* traj_rew,
                                     const uint8_t* traj_done, float* S, float* A, float* R,
                                     float* Dn, void* stream) {
  PRL_REQUIRE(E >= 0 && N >= 0 && D > 0 && Adim > 0 && t_max > 0, "prl_flatten_env_major: bad sizes");
  if (N == 0) return PRL_OK;
  PRL_REQUIRE(offsets && traj_obs && traj_act && traj_rew && traj_done && S && A && R && Dn,
              "prl_flatten_env_major: null pointer");
  PRL_REQUIRE(D != 4 || (aligned16(traj_obs) && aligned16(S)),
              "prl_flatten_env_major: obs buffers must be 16-B aligned");
  FlattenArgs a{E, D, Adim, offsets, N, traj_obs, traj_act, traj_rew, traj_done, S, A, R, Dn};
  hipStream_t s = as_stream(stream);
  if (D <= 32) {
    hipLaunchKernelGGL(flatten_rows_kernel, dim3((unsigned)cdiv(N, 256)), dim3(256), 0, s, a);
  } else {
    if ((D & 3) == 0 && aligned16(traj_obs) && aligned16(S))
      hipLaunchKernelGGL(flatten_wide_kernel<true>, dim3((unsigned)cdiv(N, 4)), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(flatten_wide_kernel<false>, dim3((unsigned)cdiv(N, 4)), dim3(256), 0, s, a);
  }
  PRL_LAUNCH_CHECK("flatten_env_major");
  return PRL_OK;
}
