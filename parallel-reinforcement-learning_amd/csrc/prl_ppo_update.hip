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
// Decomposition (G workgroups of 256 threads, one per CU, co-resident: occupancy-checked plain launch):
//   phase A  workgroup g takes rows [g*R, (g+1)*R) of the step's minibatch in 16-row tiles;
//            forward + backward run out of LDS with the CURRENT parameters in LDS (every
//            workgroup holds a full, bit-identical copy), accumulating this workgroup's partial
//            gradient (and the loss partials) in LDS, then publishes it write-through (sc1
//            16-B stores) to part[g] and bumps counter A;
//   phase B  when all G partials are in, workgroup g sums its 1/G slice of the gradient over the
//            G partials in workgroup order (deterministic), publishes the slice (sc1) and bumps
//            counter B;
//   phase C  when all slices are in, EVERY workgroup reads the whole reduced gradient (sc1
//            loads), forms its squared norm in one fixed order and the clip coefficient, and
//            applies AdamW to its own copy of the parameters (LDS) and moments (registers) —
//            identical inputs, identical code, so every copy stays bit-identical and no
//            parameter broadcast (third hand-off) is needed.
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
#include <vector>

#include <dlfcn.h>
#include <string.h>
#include <stdlib.h>
#include <rccl/rccl.h>

namespace prl {

constexpr int UPD_THREADS = 256;
constexpr int UPD_HDR = 128;      // LDS header floats: broadcast words, timers (u64 at +16 / +64)
constexpr int UPD_H = 64;         // hidden width
constexpr int UPD_HS = 68;        // LDS row stride of [*][64] arrays
constexpr int UPD_MAXH = 3;       // heads
constexpr int UPD_MAXD = 64;      // max observation dim on the fused path
constexpr int UPD_MAXA = 8;       // max action dim on the fused path
constexpr int UPD_MAX_RANKS = 8;   // data-parallel ranks of one persistent launch (one node)
constexpr unsigned UPD_SPIN_LIMIT = 1u << 22;  // ~0.1-0.3 s of s_sleep polls: never expected
// the cross-RANK wait of the data-parallel launch (upd_dp_union_slice) also absorbs the skew
// between the ranks' launches and each poll is a system-scope load (a peer GPU's memory over
// xGMI): its own, much longer default limit, set per process by prl_dp_set_spin_limit (tests
// lower it to provoke the timeout path)
constexpr unsigned UPD_DP_SPIN_LIMIT = 1u << 24;

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

// LDS image + flat offsets of the reference's parameter tensors, torch parameters() order.
// constexpr: the specialised kernels fold the whole layout into immediates.
__host__ __device__ constexpr void upd_add(UpdTensor& t, int& flat, int& lds, int rows, int cols,
                                           int stride) {
  t.flat = flat;
  t.lds = lds;
  t.rows = rows;
  t.cols = cols;
  t.stride = stride;
  flat += rows * cols;
  lds += (rows * stride + 3) & ~3;
}
__host__ __device__ constexpr bool upd_layout(int D, int A, int discrete, UpdNet& n) {
  if (D < 1 || D > UPD_MAXD || A < 1 || A > UPD_MAXA) return false;
  n = UpdNet{};
  n.D = D;
  n.A = A;
  n.discrete = discrete ? 1 : 0;
  n.nh = discrete ? 2 : 3;
  int flat = 0, lds = 0;
  upd_add(n.w0, flat, lds, UPD_H, D, D | 1);
  upd_add(n.g0, flat, lds, 1, UPD_H, UPD_H);
  upd_add(n.b0, flat, lds, 1, UPD_H, UPD_H);
  int col = 0;
  for (int h = 0; h < n.nh; ++h) {
    const int out = (h == n.nh - 1) ? 1 : A;
    n.out[h] = out;
    n.ocol[h] = col;
    col += out;
    upd_add(n.w1[h], flat, lds, UPD_H, UPD_H, UPD_HS);
    upd_add(n.g1[h], flat, lds, 1, UPD_H, UPD_H);
    upd_add(n.b1[h], flat, lds, 1, UPD_H, UPD_H);
    upd_add(n.w2[h], flat, lds, out, UPD_H, UPD_HS);
    upd_add(n.b2[h], flat, lds, 1, out, out);
  }
  n.nout = col;
  if (n.nout > 16) return false;   // one 16-row output tile (UPD_MAXO)
  n.P = flat;
  n.Lp = lds;
  return true;
}
__host__ __device__ constexpr UpdNet upd_make(int D, int A, int discrete) {
  UpdNet n{};
  upd_layout(D, A, discrete, n);
  return n;
}

struct UpdArgs {
  UpdNet net;
  const float* S;
  const float* act;
  const float* old_logp;
  const float* adv;
  const float* ret;
  int64_t N;
  int mb, nb, total_steps, G, R;
  int Gt;           // tile groups (= G, or G / replicas in the latency form's replicated tiles)
  int Gs;           // head-split form: phase-B slice owners = the G tile workgroups + Gs - G helpers
  float clip, vf_coef, ent_coef, lr;
  double beta1, beta2;   // AdamW betas as the caller's doubles: 1 - beta2 from a float32 beta2 is 1.3e-5 off
  float eps, wd, max_norm;
  float* params;
  float* exp_avg;
  float* exp_avg_sq;
  float* adam_step;
  float* loss_out;
  float* part;      // [G][Qtot * 4]
  float* part2;     // head-split form: role 1's trunk + loss-partial quads [Gt][QT + 1][4]
  int spl_fill;     // head-split form's phase B: threads per quad (PRL_UPD_SPL_FILL, A/B)
  int spl_direct;   // head-split form: dW1 stored from registers into the partial (PRL_UPD_SPL_DIRECT)
  int spl_poll;     // head-split form: counter waits with four polls in flight (PRL_UPD_SPL_POLL)
  int spl_pk;       // head-split form: AdamW two elements per packed-f32 instruction (PRL_UPD_SPL_PK)
  int spl_pieces;   // head-split form: the clip norm from per-chunk pieces (PRL_UPD_SPL_PIECES)
  int spl_tw4;      // head-split form: 4 x a trunk / loss quad's weight in phase B's slicing (PRL_UPD_SPL_TW4)
  float* red;       // [Qtot * 4]
  float* sq;        // [NW G] per-wave squared-norm pieces of the slices
  unsigned* ctr;    // [0] arrivals A, [1] arrivals B, [2] abort, [3] status (zeroed per launch),
                    // [4] sticky timeout flag (never zeroed by a launch)
  unsigned long long* prof;  // [8] workgroup 0's time per phase (100 MHz ticks, summed over steps)
  unsigned grad_target;      // ppo_grad_kernel: arrivals on ctr[0] that end its hand-off
  int profile;               // 1: workgroup 0 records its phase / tile-stage times (PRL_UPD_PROFILE)
  // data-parallel persistent launch (prl_ppo_update_dpx; world == 1: the single-GPU engine)
  int world, rank;
  const float* inv_count;    // [nb] 1 / rows of union minibatch j over all ranks (null: 1 / B)
  unsigned long long dp_seq0;   // exchange sequence number of this launch's first step
  unsigned dp_spin_limit;       // polls of the cross-rank wait before it gives up
  int dp_fine;                  // some rank's slice buffer is fine-grained: fence the flag
  float* xbuf[UPD_MAX_RANKS];             // rank r's [2][Qtot * 4] slice buffers (peer mappings)
  unsigned long long* xflag[UPD_MAX_RANKS];   // rank r's [G] per-workgroup step flags
  float* xbuf_self;                       // == xbuf[rank] (no dynamic kernarg indexing)
  unsigned long long* xflag_self;         // == xflag[rank]
  // push form of the cross-rank exchange (dp_push, head-split kernel): every rank's buffer also
  // holds receive slices [2 parity][UPD_MAX_RANKS][Qtot][4] f32 at float offset xpush_off and
  // receive flags [UPD_MAX_RANKS][xpush_gmax] u64 at u64 offset xpush_flags_off
  int dp_push;
  size_t xpush_off, xpush_flags_off;
  int xpush_gmax;
  float *tp_m0, *tp_v0, *tp_m1, *tp_v1;   // the throughput form's moment buffers (image layout)
};

// ---- sc1 (write-through / L1-bypassing) accessors -------------------------------------------
typedef unsigned v4u __attribute__((ext_vector_type(4)));

// The resource is built from a WAVE-UNIFORM base (a kernel argument); the per-lane part of the
// address goes in the byte offset.  (A per-lane base forces a 64-iteration waterfall loop.)
__device__ inline __amdgpu_buffer_rsrc_t upd_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
// cache policy of the 16-B buffer accesses: sc1 = device scope (the hand-offs inside one GPU);
// sc0 sc1 = system scope (the data-parallel slices other ranks' kernels read through IPC maps)
constexpr int UPD_AUX_SC1 = 16, UPD_AUX_SYS = 17;
template <int AUX>
__device__ inline float4 ld4_aux(__amdgpu_buffer_rsrc_t rs, size_t float_off) {
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(float_off * 4), 0, AUX);
  return float4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                __uint_as_float(v.w)};
}
template <int AUX>
__device__ inline void st4_aux(__amdgpu_buffer_rsrc_t rs, size_t float_off, float4 x) {
  v4u v;
  v.x = __float_as_uint(x.x);
  v.y = __float_as_uint(x.y);
  v.z = __float_as_uint(x.z);
  v.w = __float_as_uint(x.w);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, (unsigned)(float_off * 4), 0, AUX);
}
__device__ inline float4 ld4_sc1(__amdgpu_buffer_rsrc_t rs, size_t float_off) {
  return ld4_aux<UPD_AUX_SC1>(rs, float_off);
}
// the same with the per-lane part in the VGPR offset and a wave-uniform part in the SGPR offset
// (one address register for a whole strided sweep: nothing per load for the compiler to spill)
__device__ inline float4 ld4_sc1_so(__amdgpu_buffer_rsrc_t rs, unsigned voff_bytes, unsigned soff_bytes) {
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff_bytes, soff_bytes, UPD_AUX_SC1);
  return float4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                __uint_as_float(v.w)};
}
__device__ inline void st4_sc1(__amdgpu_buffer_rsrc_t rs, size_t float_off, float4 x) {
  st4_aux<UPD_AUX_SC1>(rs, float_off, x);
}
// Hand-off words (counters, status, flags) are addressed through the GLOBAL address space:
// without it, kernels whose pointers pass through private memory (the runtime-layout kernel)
// lowered them to flat_ atomics / loads, which the guide's hand-off table does not cover
// (tests/test_host_cpu.py::test_handoff_isa checks the built code object).
template <class T>
__device__ inline __attribute__((address_space(1))) T* upd_g(T* p) {
  return (__attribute__((address_space(1))) T*)(p);
}
__device__ inline float ld_sc1f(const float* p) {
  return __uint_as_float(__hip_atomic_load(upd_g(reinterpret_cast<const unsigned*>(p)), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}
__device__ inline void st_sc1f(float* p, float x) {
  __hip_atomic_store(upd_g(reinterpret_cast<unsigned*>(p)), __float_as_uint(x), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned ld_sc1u(const unsigned* p) {
  return __hip_atomic_load(upd_g(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 8-way sharded arrival counters (shard k at word 32 (1 + k) of its block, one 128-B line each):
// an arrival adds to shard g & 7, so at most G / 8 atomics meet on one line; a whole wave polls,
// lanes 0..7 one shard each, and the DPP sum over the 8 lanes is the arrival count.
#ifndef PRL_UPD_SHARDS
#define PRL_UPD_SHARDS 8   // (8 or 16; -DPRL_UPD_SHARDS=16 builds the 16-line form for A/Bs)
#endif
constexpr int UPD_SHARDS = PRL_UPD_SHARDS;
static_assert(UPD_SHARDS == 8 || UPD_SHARDS == 16, "8 or 16 counter shards");
constexpr int UPD_CTR_A = 32;                              // first shard word of counter A
constexpr int UPD_CTR_B = UPD_CTR_A + 32 * UPD_SHARDS;     // ... of counter B
constexpr int UPD_CTR_C = UPD_CTR_B + 32 * UPD_SHARDS;     // ... of counter C (split form, OWN)
constexpr int UPD_CTR_WORDS = UPD_CTR_C + 32 * UPD_SHARDS;
__device__ inline void upd_arrive(unsigned* ctr, int base, int g) {
  __hip_atomic_fetch_add(upd_g(ctr + base + 32 * (g & (UPD_SHARDS - 1))), 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned upd_isum8(unsigned v) {   // (lanes 0 .. UPD_SHARDS - 1 into lane 0)
  v += (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  v += (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  v += (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
  if constexpr (UPD_SHARDS == 16) v += (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);
  return v;
}
// one whole wave: wait until the shards of counter `base` sum to >= target; false on timeout /
// abort (same abort / status / sticky words as upd_wait).  Lane 8 loads the abort word in the
// same round as lanes 0-7 load the shards: one memory round trip per poll, not two in series.
template <int SL = 1>   // s_sleep between polls (64 x SL cycles)
__device__ inline bool upd_wait_sharded(unsigned* ctr, int base, unsigned target) {
  const int l = threadIdx.x & 63;
  for (unsigned spins = 0;; ++spins) {
    const unsigned v = l < UPD_SHARDS ? ld_sc1u(ctr + base + 32 * l)
                                      : (l == UPD_SHARDS ? ld_sc1u(ctr + 2) : 0u);
    const unsigned tot = (unsigned)__builtin_amdgcn_readlane((int)upd_isum8(l < UPD_SHARDS ? v : 0u), 0);
    if (tot >= target) return true;
    if ((unsigned)__builtin_amdgcn_readlane((int)v, UPD_SHARDS) != 0u) return false;
    if (spins > UPD_SPIN_LIMIT) {
      if (l == 0) {
        __hip_atomic_store(upd_g(ctr + 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(upd_g(ctr + 3), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_or(upd_g(ctr + 4), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sticky
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(SL);
  }
}

// upd_wait_sharded with FOUR polls in flight: a poll is re-issued as soon as the oldest one is
// checked, so a counter reaching its target is seen about a quarter of a poll round trip after
// it lands instead of up to a whole one (every check waits only for its own load: the compiler's
// counted vmcnt).  Same words, same abort / timeout handling.
__device__ inline unsigned upd_poll8(unsigned* ctr, int base, int l) {
  return l < UPD_SHARDS ? ld_sc1u(ctr + base + 32 * l) : (l == UPD_SHARDS ? ld_sc1u(ctr + 2) : 0u);
}
__device__ inline int upd_poll_check(unsigned v, int l, unsigned target) {
  const unsigned tot = (unsigned)__builtin_amdgcn_readlane((int)upd_isum8(l < UPD_SHARDS ? v : 0u), 0);
  if (tot >= target) return 1;
  if ((unsigned)__builtin_amdgcn_readlane((int)v, UPD_SHARDS) != 0u) return -1;
  return 0;
}
__device__ inline bool upd_wait_sharded_pipe(unsigned* ctr, int base, unsigned target) {
  const int l = threadIdx.x & 63;
  unsigned v0 = upd_poll8(ctr, base, l);
  __builtin_amdgcn_s_sleep(1);
  unsigned v1 = upd_poll8(ctr, base, l);
  __builtin_amdgcn_s_sleep(1);
  unsigned v2 = upd_poll8(ctr, base, l);
  __builtin_amdgcn_s_sleep(1);
  unsigned v3 = upd_poll8(ctr, base, l);
  for (unsigned spins = 0;; spins += 4) {
    int c = upd_poll_check(v0, l, target);
    if (c) return c > 0;
    v0 = upd_poll8(ctr, base, l);
    c = upd_poll_check(v1, l, target);
    if (c) return c > 0;
    v1 = upd_poll8(ctr, base, l);
    c = upd_poll_check(v2, l, target);
    if (c) return c > 0;
    v2 = upd_poll8(ctr, base, l);
    c = upd_poll_check(v3, l, target);
    if (c) return c > 0;
    v3 = upd_poll8(ctr, base, l);
    if (spins > UPD_SPIN_LIMIT) {
      if (l == 0) {
        __hip_atomic_store(upd_g(ctr + 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(upd_g(ctr + 3), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_or(upd_g(ctr + 4), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sticky
      }
      return false;
    }
  }
}

// one lane: wait until *c >= target (or abort); false on timeout / abort (both words loaded in
// one round)
__device__ inline bool upd_wait(unsigned* ctr, int which, unsigned target) {
  for (unsigned spins = 0;; ++spins) {
    const unsigned v = ld_sc1u(ctr + which), ab = ld_sc1u(ctr + 2);
    if (v >= target) return true;
    if (ab != 0u) return false;
    if (spins > UPD_SPIN_LIMIT) {
      __hip_atomic_store(upd_g(ctr + 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(upd_g(ctr + 3), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_or(upd_g(ctr + 4), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sticky
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Hardware transcendentals (v_exp_f32 / v_log_f32 / v_rcp_f32 / v_rsq_f32, ~1 ulp) for the
// engine's per-row and per-channel math: the forward's log-probs stay within float32 rounding of
// float64 (tests/test_engine_gpu.py checks them), and evaluate/update share these helpers, so the
// first minibatch's ratio is still exactly 1.
__device__ inline float upd_exp(float x) { return __expf(x); }
__device__ inline float upd_log(float x) { return __logf(x); }
// log of a clamped probability (x in [FLT_EPSILON, 1 - FLT_EPSILON], or NaN): no denormal / inf
// cases, so v_log_f32 (log2) times ln 2 alone — __logf's lowering adds a denormal rescale and an
// extra-precision ln 2 split around it, ~9 dependent instructions on the actor's loss chain
__device__ inline float upd_log_unit(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }
__device__ inline float upd_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ inline float upd_sigmoid(float y) { return upd_rcp(1.0f + upd_exp(-y)); }

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
#pragma unroll
  for (int h = 0; h < UPD_MAXH; ++h)   // compile-time h: no dynamic indexing of the kernarg
    if (h < n.nh && (upd_in(n.w1[h], k, f) || upd_in(n.g1[h], k, f) || upd_in(n.b1[h], k, f) ||
                     upd_in(n.w2[h], k, f) || upd_in(n.b2[h], k, f)))
      return f;
  return -1;
}

// ---- per-tile LDS scratch (floats, carved after the parameter / gradient images) -------------
// One tile = 16 rows.  Wave w (of 4) owns channel block w (channels 16w .. 16w+15) of every
// 64-wide layer; activations stay in MFMA C fragments (lane (x = l & 15, q = l >> 4), register i
// holds [row x][channel 16 b + 4 q + i]), and the only LDS traffic is the transposes the weight
// gradients need (they contract over rows) plus the output-layer partials.
constexpr int UPD_RT = 16;        // rows per tile
constexpr int UPD_ZS = 80;        // row stride of the [16 rows][64 ch] tiles (80 = 16 mod 64)
constexpr int UPD_RIN = 12;       // row-input record: act[8], old_logp, adv, ret, pad
constexpr int UPD_MAXO = 16;      // outputs of all heads together (one 16-row MFMA tile)

__host__ __device__ inline int upd_xs(int D) { return D <= 16 ? 16 : UPD_ZS; }
// transpose slots per wave: one per head for the two-head (discrete) nets, so both heads'
// backward chains interleave; the three-head (continuous) nets share one slot (LDS is short)
__host__ __device__ constexpr int upd_ts(const UpdNet& n) { return n.discrete ? 2 : 1; }
__host__ __device__ inline int upd_scratch_floats(int D, int NW, int TS) {
  return UPD_RT * upd_xs(D)          // Xs  [16][XS]       tile inputs (rows x features)
         + NW * UPD_RT * 16          // Op  [NW][16][16]   output-layer partial per wave
         + NW * UPD_RT * 16          // Os  [NW][16][16]   assembled outputs per wave
         + NW * UPD_RT * 16          // dOs [NW][16][16]   d loss / d outputs per wave
         + UPD_RT * UPD_RIN          // Rin [16][12]       row inputs
         + 2 * UPD_RT * UPD_ZS       // Fs  [2][16][80]    trunk output (double-buffered by tile)
         + UPD_MAXH * UPD_RT * UPD_ZS  // Zs [h][16][80]   head dZ
         + NW * TS * UPD_RT * 16     // Ts  [NW][TS][16][16] per-wave transpose slots (G_h; dH0 in 0)
         + 16;
}
struct UpdScr {
  float *Xs, *Op, *Os, *dOs, *Rin, *Fs, *Zs, *Ts;
  float* Fs2;   // the other trunk-output buffer: consecutive tiles of a step alternate (a tile's
                // forward writes Fs before any barrier, while a slower wave may still read the
                // previous tile's after that tile's barrier #2)
  int XS;
};
// the scratch view of the step's tile number c (odd tiles use the second trunk-output buffer)
__device__ inline UpdScr upd_scr_tile(const UpdScr& s, int c) {
  UpdScr r = s;
  if (c & 1) r.Fs = s.Fs2;
  return r;
}
__device__ inline UpdScr upd_scr(float* p, int D, int NW) {
  UpdScr s;
  s.XS = upd_xs(D);
  s.Xs = p; p += UPD_RT * s.XS;
  s.Op = p; p += NW * UPD_RT * 16;
  s.Os = p; p += NW * UPD_RT * 16;
  s.dOs = p; p += NW * UPD_RT * 16;
  s.Rin = p; p += UPD_RT * UPD_RIN;
  s.Fs = p; p += UPD_RT * UPD_ZS;
  s.Fs2 = p; p += UPD_RT * UPD_ZS;
  s.Zs = p; p += UPD_MAXH * UPD_RT * UPD_ZS;
  s.Ts = p;
  return s;
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
// KD: 1 discrete / 0 continuous / -1 runtime, 2 / 3 the 8-wave discrete / continuous forms of
// the persistent kernel (upd_nw);  KA: action dim (0 = runtime).  Specialised kernels keep the
// per-row code (executed by 16 lanes, but fetched every step) small.
constexpr bool upd_kd_discrete(int KD) { return KD == 1 || KD == 2; }
template <int KD, int KA, class OT>
__device__ inline void upd_row_dist(const UpdNet& n, const OT& O, const float* act, UpdDist& d) {
  const int A = KA > 0 ? KA : n.A;
  const bool discrete = KD >= 0 ? upd_kd_discrete(KD) : (n.discrete != 0);
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
      d.p[k] = k < A ? upd_exp(O[k] - mx) : 0.f;
      s += d.p[k];
    }
    const float rs = upd_rcp(s);
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      d.p[k] = k < A ? d.p[k] * rs : 0.f;
      d.S2 += d.p[k];
    }
    const float rS2 = upd_rcp(d.S2);
    d.ai = (int)act[0];
    const bool bad = d.ai < 0 || d.ai >= A;   // torch's gather would raise: poison instead
    float la = 0.f;
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      d.q[k] = d.p[k] * rS2;
      if (k < A) {
        // torch's clamp(probs, eps, 1 - eps), NaN propagated; branch-free (a select per bound, the
        // log always evaluated: no per-branch constant folding into divergent code)
        const float qk = d.q[k];
        const float c = qk != qk ? qk : fminf(fmaxf(qk, FLT_EPSILON), 1.0f - FLT_EPSILON);
        const float l = upd_log_unit(c);
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
        const float sd = upd_log(1.0f + upd_exp(lsc));   // softplus, beta 1 (lsc <= 2 < 20)
        const float dd = act[k] - mu;
        const float lsd = upd_log(sd);
        d.logp += -(dd * dd) * upd_rcp(2.0f * (sd * sd)) - lsd - half_log_2pi;
        d.H += 0.5f + half_log_2pi + lsd;
      }
    }
  }
}

// Per-row loss (surrogate, prl_loss.hip semantics) and the gradient w.r.t. the head outputs
// dO[0 .. nout) (dO[nout .. 16) = 0).  lp = {-min(s1, s2), SmoothL1, H}.  O / dO: LDS rows (the
// runtime-layout kernel) or register arrays (the specialised kernels: indices fold to constants).
// PART 1: the critic's dO and lp[1] only; 2: the actor's dO, lp[0] and lp[2] only (the same
// arithmetic for what is computed; the rest stays 0).
template <int KD, int KA, int PART = 0, class OT, class DT>
__device__ inline void upd_row_loss(const UpdNet& n, const OT& O, const float* rin, float invB,
                                    float clip, float vf_coef, DT& dO, float (&lp)[3]) {
  const int A = KA > 0 ? KA : n.A;
  const bool discrete = KD >= 0 ? upd_kd_discrete(KD) : (n.discrete != 0);
  const int vcol = discrete ? A : 2 * A;      // critic output column
#pragma unroll
  for (int j = 0; j < UPD_MAXO; ++j) dO[j] = 0.f;
  if constexpr (PART != 2) {
    const float V = O[vcol];
    const float x = V - rin[10];
    const float ax = fabsf(x);
    const float sl = ax < 1.0f ? 0.5f * ax * ax : ax - 0.5f;
    const float gx = ax < 1.0f ? x : (x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f));
    dO[vcol] = vf_coef * invB * gx;
    lp[1] = sl;
  }
  if constexpr (PART == 1) return;
  UpdDist dist;
  upd_row_dist<KD, KA, OT>(n, O, rin, dist);
  const float logp = dist.logp, H = dist.H, S2 = dist.S2, qa = dist.qa;
  const int ai = dist.ai;
  const float* p = dist.p;
  // surrogate
  const float diff = logp - rin[8];
  const float cl = diff < -20.0f ? -20.0f : (diff > 20.0f ? 20.0f : diff);
  const float ratio = upd_exp(cl);
  const float adv = rin[9];
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
  lp[0] = -m;
  lp[2] = H;
  // d logp / d head outputs
  if (discrete) {
    const float mk = (qa >= FLT_EPSILON && qa <= 1.0f - FLT_EPSILON) ? 1.0f : 0.0f;
    const float gq = (logp != logp) ? logp : dlogp * mk;
    float dp[UPD_MAXA];
    float dot = 0.f;
    const float rqa = upd_rcp(qa), rS2 = upd_rcp(S2);
#pragma unroll
    for (int k = 0; k < UPD_MAXA; ++k) {
      dp[k] = k < A ? gq * (((k == ai) ? rqa : 0.0f) - 1.0f) * rS2 : 0.f;
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
        const float sd = upd_log(1.0f + upd_exp(lsc));
        const float d = rin[k] - mu;
        const float var = sd * sd;
        const float rvar = upd_rcp(var), rsd = upd_rcp(sd);
        dO[k] = dlogp * (d * rvar);
        const float dsd = dlogp * ((d * d) * (rvar * rsd) - rsd);
        const float pass = (lsr >= -2.0f && lsr <= 2.0f) ? 1.0f : 0.0f;
        dO[A + k] = dsd * upd_sigmoid(lsc) * pass;
      }
    }
  }
}

// Cross-lane moves by DPP (no LDS round trip, unlike __shfl*, which lowers to ds_bpermute):
// quad_perm [1,0,3,2] = xor 1, [2,3,0,1] = xor 2, row_half_mirror (lane i <-> 7 - i), row_mirror
// (lane i <-> 15 - i).  Butterflies of commutative adds: every lane ends with the same bits.
template <int CTRL>
__device__ inline float upd_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ inline float upd_xor1(float v) { return upd_dpp<0xB1>(v); }
__device__ inline float upd_xor2(float v) { return upd_dpp<0x4E>(v); }
// sum over the 16 lanes of a DPP row (= the 16 rows of a tile, for one channel quad q)
__device__ inline float upd_rsum16(float v) {
  v += upd_xor1(v);
  v += upd_xor2(v);
  v += upd_dpp<0x141>(v);
  v += upd_dpp<0x140>(v);
  return v;
}
// v + (v of the partner lane l ^ 16: the other 4 channels of the lane's GroupNorm group), by
// v_permlane16_swap (VALU, no LDS round trip): with both operands = v it returns {v of the even
// row of each row pair, v of the odd row}, so r[0] + r[1] has the same bits in both rows.
__device__ inline float upd_pair_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

typedef float upd_v4 __attribute__((ext_vector_type(4)));
typedef float upd_f2 __attribute__((ext_vector_type(2)));
__device__ inline upd_f2 upd_pkfma(upd_f2 a, upd_f2 b, upd_f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ inline upd_v4 upd_mma(float a, float b, upd_v4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ inline upd_v4 upd_ld4(const float* p) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  return upd_v4{v.x, v.y, v.z, v.w};
}
__device__ inline void upd_st4(float* p, upd_v4 v) {
  *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
}
// intra-wave LDS hand-off between lanes (LDS ops of one wave complete in order)
__device__ inline void upd_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// GroupNorm(8 groups of 8) + SiLU forward on a C fragment: the lane's 4 channels + the partner
// lane's 4 form the group.  Returns xhat, rstd and the block output.
__device__ inline void upd_gn_fwd_frag(upd_v4 z, upd_v4 gw, upd_v4 gb, upd_v4& xh, float& rstd,
                                       upd_v4& y) {
  const float s4 = (z[0] + z[1]) + (z[2] + z[3]);
  const float mean = upd_pair_sum(s4) * 0.125f;
  upd_v4 d;
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = z[i] - mean;
  const float q4 = (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
  rstd = __builtin_amdgcn_rsqf(upd_pair_sum(q4) * 0.125f + 1e-5f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xh[i] = d[i] * rstd;
    const float u = xh[i] * gw[i] + gb[i];
    y[i] = u * upd_sigmoid(u);
  }
}
// backward of the above: go = d(block output); returns dX, dy = d(pre-SiLU) (for dγ, dβ)
__device__ inline upd_v4 upd_gn_bwd_frag(upd_v4 go, upd_v4 xh, upd_v4 gw, upd_v4 gb, float rstd,
                                         upd_v4& dy) {
  upd_v4 dxh;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float u = xh[i] * gw[i] + gb[i];
    const float sg = upd_sigmoid(u);
    dy[i] = go[i] * (sg * (1.0f + u * (1.0f - sg)));
    dxh[i] = dy[i] * gw[i];
  }
  const float a4 = (dxh[0] + dxh[1]) + (dxh[2] + dxh[3]);
  const float b4 = (dxh[0] * xh[0] + dxh[1] * xh[1]) + (dxh[2] * xh[2] + dxh[3] * xh[3]);
  const float m1 = upd_pair_sum(a4) * 0.125f;
  const float m2 = upd_pair_sum(b4) * 0.125f;
  upd_v4 dx;
#pragma unroll
  for (int i = 0; i < 4; ++i) dx[i] = rstd * (dxh[i] - m1 - xh[i] * m2);
  return dx;
}

// image offset of output j's bias (head chosen by compile-time h: no dynamic kernarg indexing)
__device__ inline int upd_bias_of(const UpdNet& n, int j) {
  int off = 0;
#pragma unroll
  for (int h = 0; h < UPD_MAXH; ++h)
    if (h < n.nh && j >= n.ocol[h] && j < n.ocol[h] + n.out[h]) off = n.b2[h].lds + (j - n.ocol[h]);
  return off;
}

template <int KD>
__device__ inline int upd_nh(const UpdNet& n) { return KD < 0 ? n.nh : (upd_kd_discrete(KD) ? 2 : 3); }

// Forward state of one tile kept for the backward (wave w's channel block, lane's row x).
// KSM = compile-time bound on the input k-steps ceil(D / 4) (4 for the specialised kernels);
// HPW = heads per wave (all heads with 4 waves; one head per wave group with 8 waves).
template <int KSM, int HPW>
struct UpdFwd {
  upd_v4 Fw;                     // trunk output, block b
  upd_v4 xh0;                    // trunk xhat (block b)
  float r0;                      // trunk rstd (block b)
  upd_v4 xh[HPW], G[HPW];        // head xhat / output (block b) of the wave's heads
  float rh[HPW];
};
template <int KA>
constexpr int upd_ksm() { return KA > 0 ? 4 : 16; }
// Waves per workgroup.  KD = 2 is the persistent engine's two-head discrete specialisation
// (CartPole, used by prl_ppo_update / _dpx): 8 waves, wave w = (head group w >> 2, channel block
// w & 3) — two waves per SIMD hide each other's MFMA / LDS latency and every per-wave chain is
// half as long (round 3, tools/engine_profile.py: 15.65 -> 15.02 us per step at mb 512,
// 140.1 -> 120.2 us at mb 65,536; the moments then take 5 quads per thread).  KD = 1 (the same
// net; the stepped and evaluate kernels), the three-head nets (Pendulum) and the generic kernel
// run 4 waves (wave w = channel block w, all heads) to stay inside the LDS.
template <int KD, int KA>
constexpr int upd_nw() { return ((KD == 2 && KA == 2) || KD == 3) ? 8 : 4; }
// heads per wave: with 8 waves group 0 takes heads 0 (and 2), group 1 head 1
template <int KD, int KA>
constexpr int upd_hpw() { return upd_nw<KD, KA>() == 8 ? (upd_kd_discrete(KD) ? 1 : 2) : UPD_MAXH; }
// global head of the wave's local head slot hs
template <int NW>
__device__ inline int upd_head(int hs, int hg) { return NW == 8 ? hg + 2 * hs : hs; }
// image offsets / output columns of head h (h wave-uniform, possibly runtime): selected over
// compile-time indices, so the kernarg struct is never indexed dynamically (that would copy it
// to scratch)
struct UpdHead {
  int w1, g1, b1, w2, oc, no;
};
// Branch-free: head 0's value plus the steps to heads 1 and 2 times (h >= 1), (h >= 2).  (A
// select chain let the compiler turn a runtime h — the 8-wave kernels' head group — into a
// lookup table in private memory, i.e. scratch loads on every use.)
__device__ inline UpdHead upd_head_info(const UpdNet& n, int h) {
  if (n.nh == 2) {   // (the two-head nets: one select, as the register budget of their 8-wave kernel has it)
    return h == 1 ? UpdHead{n.w1[1].lds, n.g1[1].lds, n.b1[1].lds, n.w2[1].lds, n.ocol[1], n.out[1]}
                  : UpdHead{n.w1[0].lds, n.g1[0].lds, n.b1[0].lds, n.w2[0].lds, n.ocol[0], n.out[0]};
  }
  const int s1 = h >= 1 ? 1 : 0, s2 = h >= 2 ? 1 : 0;
  auto pick = [&](int v0, int v1, int v2) { return v0 + s1 * (v1 - v0) + s2 * (v2 - v1); };
  static_assert(UPD_MAXH == 3, "upd_head_info picks among three heads");
  return UpdHead{pick(n.w1[0].lds, n.w1[1].lds, n.w1[2].lds), pick(n.g1[0].lds, n.g1[1].lds, n.g1[2].lds),
                 pick(n.b1[0].lds, n.b1[1].lds, n.b1[2].lds), pick(n.w2[0].lds, n.w2[1].lds, n.w2[2].lds),
                 pick(n.ocol[0], n.ocol[1], n.ocol[2]), pick(n.out[0], n.out[1], n.out[2])};
}

// A tile's global inputs, loaded into registers ahead of the tile (prefetch): the B fragments
// of the observations X[row x][4 s + q] and one word of the row-input record (thread t < 192:
// row t / 12, field t % 12 = act[0..7], old_logp, adv, ret, pad).  Every slot is ONE load from a
// selected address (a valid dummy for an empty slot) with its validity in `ok` (bit s: xin[s],
// bit 31: rin); upd_in_real zeroes the empty ones.  The persistent kernel's prefetch applies it
// only when the tile starts: with the zeroing in divergent branches around the loads, the
// compiler joined the paths with copies that waited for the loads at once — right before the
// step's arrival at counter A, which put a global load's latency on every step's critical path.
template <int KSM>
struct UpdIn {
  float xin[KSM];
  float rin;
  unsigned ok;
};
template <int KSM>
__device__ inline UpdIn<KSM> upd_in_real(const UpdIn<KSM>& in) {
  UpdIn<KSM> o;
#pragma unroll
  for (int s = 0; s < KSM; ++s) o.xin[s] = (in.ok >> s) & 1u ? in.xin[s] : 0.0f;
  o.rin = (in.ok >> 31) & 1u ? in.rin : 0.0f;
  o.ok = in.ok;
  return o;
}
template <int KD, int KA, bool RAW = false>
__device__ inline void upd_tile_load(const UpdNet& n, const float* Sg, const float* actg,
                                     const float* oldg, const float* advg, const float* retg,
                                     int64_t row0, int rc, UpdIn<upd_ksm<KA>()>& in) {
  constexpr int KSM = upd_ksm<KA>();
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4;
  const int D = n.D, KS = (D + 3) >> 2;
  const bool rowok = x < rc;
  unsigned ok = 0u;
#pragma unroll
  for (int s = 0; s < KSM; ++s) {
    const int d = 4 * s + q;
    const bool v = s < KS && rowok && d < D;
    in.xin[s] = *(v ? Sg + (row0 + x) * D + d : Sg);
    ok |= v ? 1u << s : 0u;
  }
  const float* src = nullptr;
  if (t < UPD_RT * UPD_RIN) {
    const int r = t / UPD_RIN, k = t % UPD_RIN;
    const int Aw = n.discrete ? 1 : n.A;
    if (r < rc) {
      if (k < UPD_MAXA) src = k < Aw ? actg + (row0 + r) * Aw + k : nullptr;
      else if (k == 8 && oldg) src = oldg + row0 + r;
      else if (k == 9 && advg) src = advg + row0 + r;
      else if (k == 10 && retg) src = retg + row0 + r;
    }
  }
  in.rin = *(src ? src : Sg);
  ok |= src ? 1u << 31 : 0u;
  in.ok = ok;
  if constexpr (!RAW) in = upd_in_real(in);
}

// Forward of one tile (rows row0 .. row0 + rc - 1, rc <= 16) up to the output-layer partials:
// every wave runs the trunk for all 64 channels (it is the B operand of every head block), then
// its heads' block b; the output layer's K = 64 sum is split over the waves (partial per wave
// in Op[w]).  Also stages the row inputs into Rin.  No barrier inside; the caller's barrier
// publishes Op / Rin.
template <int KD, int KA>
__device__ inline void upd_tile_fwd(const UpdNet& n, const float* W, const UpdScr& sc,
                                    const UpdIn<upd_ksm<KA>()>& in,
                                    UpdFwd<upd_ksm<KA>(), upd_hpw<KD, KA>()>& f) {
  constexpr int KSM = upd_ksm<KA>(), NW = upd_nw<KD, KA>(), HPW = upd_hpw<KD, KA>();
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4, w = t >> 6;
  const int b = w & 3, hg = w >> 2;
  const int D = n.D, KS = (D + 3) >> 2;
  const int nh = upd_nh<KD>(n);
  // trunk: H0^T block b = W0[16b .. 16b+15][:] X^T  (A: W0 rows, B: inputs), then GN + SiLU —
  // this wave's block only; the four blocks meet in Fs (rows x channels) behind a barrier, and
  // every wave reads all of them back as the heads' B operand (one 16-B read per block)
  upd_v4 F[4];
  {
    upd_v4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* wr = W + n.w0.lds + (16 * b + x) * n.w0.stride;
#pragma unroll
    for (int s = 0; s < KSM; ++s) {
      if (s < KS) {
        const int d = 4 * s + q;
        acc = upd_mma(d < D ? wr[d] : 0.0f, in.xin[s], acc);
      }
    }
    upd_gn_fwd_frag(acc, upd_ld4(W + n.g0.lds + 16 * b + 4 * q), upd_ld4(W + n.b0.lds + 16 * b + 4 * q),
                    f.xh0, f.r0, f.Fw);
    if (hg == 0) upd_st4(sc.Fs + x * UPD_ZS + 16 * b + 4 * q, f.Fw);
  }
  __syncthreads();   // #0: Fs
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) F[bb] = upd_ld4(sc.Fs + x * UPD_ZS + 16 * bb + 4 * q);
  // heads: Z_h^T block b = W1_h[16b ..][:] F^T; K order per step (bb, i): lane q <-> input
  // channel 16 bb + 4 q + i, so F's C fragments are the B operand as they stand
  upd_v4 z[HPW];
#pragma unroll
  for (int hs = 0; hs < HPW; ++hs) z[hs] = upd_v4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) {
#pragma unroll
    for (int hs = 0; hs < HPW; ++hs) {
      const int h = upd_head<NW>(hs, hg);
      if (h < nh) {
        const UpdHead hi = upd_head_info(n, h);
        const upd_v4 wa = upd_ld4(W + hi.w1 + (16 * b + x) * UPD_HS + 16 * bb + 4 * q);
        z[hs] = upd_mma(wa[0], F[bb][0], z[hs]);
        z[hs] = upd_mma(wa[1], F[bb][1], z[hs]);
        z[hs] = upd_mma(wa[2], F[bb][2], z[hs]);
        z[hs] = upd_mma(wa[3], F[bb][3], z[hs]);
      }
    }
  }
  // head GN + SiLU, then the output layer's partial over this block's 16 channels:
  // O^T[j][row] += W2[j][16b + 4q + i] G^T (A row m = output j, head h's rows at ocol[h])
  upd_v4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int hs = 0; hs < HPW; ++hs) {
    const int h = upd_head<NW>(hs, hg);
    if (h < nh) {
      const UpdHead hi = upd_head_info(n, h);
      upd_gn_fwd_frag(z[hs], upd_ld4(W + hi.g1 + 16 * b + 4 * q),
                      upd_ld4(W + hi.b1 + 16 * b + 4 * q), f.xh[hs], f.rh[hs], f.G[hs]);
      const int oc = hi.oc, no = hi.no;
      const bool mine = x >= oc && x < oc + no;
      const upd_v4 wv = mine ? upd_ld4(W + hi.w2 + (x - oc) * UPD_HS + 16 * b + 4 * q)
                             : upd_v4{0.f, 0.f, 0.f, 0.f};
      o = upd_mma(wv[0], f.G[hs][0], o);
      o = upd_mma(wv[1], f.G[hs][1], o);
      o = upd_mma(wv[2], f.G[hs][2], o);
      o = upd_mma(wv[3], f.G[hs][3], o);
    }
  }
  upd_st4(sc.Op + (w * 16 + x) * 16 + 4 * q, o);   // [w][row x][j = 4q + i]
  if (t < UPD_RT * UPD_RIN) sc.Rin[t] = in.rin;
}

// After the barrier that publishes Op: lanes q == 0 of every wave assemble row x's outputs
// (the NW partials in wave order, then the bias) into Os[w][x][*]; returns the pointer.  Every
// caller reads a row only from the lane that wrote it, so no wave sync follows.  A head's
// output gets exact zeros from the other head group's waves, so 4 and 8 waves give equal bits.
template <int NW>
__device__ inline const float* upd_tile_outputs(const UpdNet& n, const float* W, const UpdScr& sc) {
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4, w = t >> 6;
  float* Orow = sc.Os + (w * 16 + x) * 16;
  if (q == 0) {
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      if (4 * j4 >= n.nout) break;
      upd_v4 v = upd_ld4(sc.Op + (0 * 16 + x) * 16 + 4 * j4);
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) {
        const upd_v4 p = upd_ld4(sc.Op + (ww * 16 + x) * 16 + 4 * j4);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += p[e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = 4 * j4 + e;
        if (j < n.nout) v[e] += W[upd_bias_of(n, j)];
      }
      upd_st4(Orow + 4 * j4, v);
    }
  }
  return Orow;
}
// The same into registers (lanes q == 0; entries past nout undefined): the specialised kernels'
// loss then reads its outputs without an LDS round trip.
template <int NW>
__device__ inline void upd_tile_outputs_reg(const UpdNet& n, const float* W, const UpdScr& sc,
                                            float (&O)[UPD_MAXO]) {
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4;
  if (q == 0) {
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      if (4 * j4 < n.nout) {
        // every wave's partial and the biases read first, all in flight together (one LDS round
        // trip on the loss's critical path: the scheduler otherwise chained them one by one under
        // the kernel's register pressure), then summed in wave order
        upd_v4 pv[NW];
        float bz[4];
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) pv[ww] = upd_ld4(sc.Op + (ww * 16 + x) * 16 + 4 * j4);
#pragma unroll
        for (int e = 0; e < 4; ++e) bz[e] = 4 * j4 + e < n.nout ? W[upd_bias_of(n, 4 * j4 + e)] : 0.f;
        __builtin_amdgcn_sched_barrier(0);
        upd_v4 v = pv[0];
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) {
          const upd_v4 p = pv[ww];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += p[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = 4 * j4 + e;
          O[j] = j < n.nout ? v[e] + bz[e] : 0.f;
        }
      }
    }
  }
}
// The row's loss into its dO row of LDS (only the first nout entries are ever read: dW2, dG and
// the output biases index outputs < nout), 16-B stores; rows past rc get zeros.
// The 8-wave two-head kernels (CartPole; upd_loss_split) compute per head group only what the
// group's head reads: group 0 the actor's dO (the ratio / clip / entropy chain), group 1 the
// critic's — the two waves of a SIMD no longer both issue the whole chain.  Group 0 also leaves
// its lp[0], lp[2] at columns 12, 13 of its dO rows for wave NW - 1's loss sums.
template <int NW, int KD, int KA>
constexpr bool upd_loss_split() { return NW == 8 && KA > 0 && KD >= 0 && upd_kd_discrete(KD); }
// The 8-wave three-head kernels (Pendulum): both groups need the dlogp chain (group 1 runs the
// log-std head), so group 0 alone runs the whole loss and group 1 reads group 0's dO rows
// (wave w & 3's) behind one workgroup barrier instead of issuing the same chain beside it;
// lp[0..2] ride in columns 12-14 of those rows for wave NW - 1's loss sums.
template <int NW, int KD, int KA>
constexpr bool upd_loss_handoff() { return NW == 8 && KA > 0 && KD >= 0 && !upd_kd_discrete(KD); }
template <int NW, int KD, int KA>
__device__ inline void upd_tile_loss(const UpdNet& n, const float* W, const UpdScr& sc, int rc,
                                     float invB, const UpdArgs& args, float (&lp)[3]) {
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4, w = t >> 6;
  float* dOrow = sc.dOs + (w * 16 + x) * 16;
  if constexpr (KA > 0) {
    constexpr bool SPLIT = upd_loss_split<NW, KD, KA>();
    constexpr bool HANDOFF = upd_loss_handoff<NW, KD, KA>();
    static_assert(!SPLIT || KA + 1 <= 12, "the split loss keeps columns 12, 13 of a dO row free");
    static_assert(!HANDOFF || 2 * KA + 1 <= 12, "the loss hand-off keeps columns 12-14 of a dO row free");
    if (HANDOFF && (w >> 2) == 1) return;
    float O[UPD_MAXO], dO[UPD_MAXO];
    upd_tile_outputs_reg<NW>(n, W, sc, O);
    if (q == 0) {
      if (x < rc) {
        if (SPLIT && (w >> 2) == 1)
          upd_row_loss<KD, KA, 1>(n, O, sc.Rin + x * UPD_RIN, invB, args.clip, args.vf_coef, dO, lp);
        else if (SPLIT)
          upd_row_loss<KD, KA, 2>(n, O, sc.Rin + x * UPD_RIN, invB, args.clip, args.vf_coef, dO, lp);
        else
          upd_row_loss<KD, KA>(n, O, sc.Rin + x * UPD_RIN, invB, args.clip, args.vf_coef, dO, lp);
      } else {
#pragma unroll
        for (int j = 0; j < UPD_MAXO; ++j) dO[j] = 0.f;
      }
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4)
        if (4 * j4 < n.nout) upd_st4(dOrow + 4 * j4, upd_v4{dO[4 * j4], dO[4 * j4 + 1], dO[4 * j4 + 2], dO[4 * j4 + 3]});
      if (SPLIT && (w >> 2) == 0) upd_st4(dOrow + 12, upd_v4{lp[0], lp[2], 0.f, 0.f});
      if (HANDOFF) upd_st4(dOrow + 12, upd_v4{lp[0], lp[1], lp[2], 0.f});
    }
  } else {
    const float* Orow = upd_tile_outputs<NW>(n, W, sc);
    if (q == 0) {
      if (x < rc) {
        upd_row_loss<KD, KA>(n, Orow, sc.Rin + x * UPD_RIN, invB, args.clip, args.vf_coef, dOrow, lp);
      } else {
#pragma unroll
        for (int j = 0; j < UPD_MAXO; ++j) dOrow[j] = 0.f;
      }
    }
  }
}

// gradient-image update: the step's first tile stores, later tiles accumulate (first is
// wave-uniform; every image entry has one owning lane, so the step needs no zeroing pass)
__device__ inline void upd_gadd(float* p, float v, bool first) {
  if (first) *p = v;   // first is a compile-time constant at every call site (upd_tile<.., FIRST>)
  else *p += v;
}
// sum over the tile's rows (DPP row) of a per-lane channel quad; lanes x == 0 add it to g[0..3]
__device__ inline void upd_colsum_add(upd_v4 v, float* g, bool owner, bool first) {
  upd_v4 s;
#pragma unroll
  for (int i = 0; i < 4; ++i) s[i] = upd_rsum16(v[i]);
  if (owner) {
#pragma unroll
    for (int i = 0; i < 4; ++i) upd_gadd(g + i, s[i], first);
  }
}

// The throughput form (TP, many tiles per workgroup and step): the step's gradient accumulates in
// REGISTERS of its owning lane — the same entries, tile order and per-tile sums as the LDS image
// above (so the same bits), without the image's load + store per entry and tile — and is stored
// straight from the registers into the workgroup's partial at the end of phase A.  With 8 waves
// the two head groups own disjoint parts (group 1: dW1 of both heads; group 0: the trunk), so
// they share the registers u[].
template <int NW, int HPW, int KSM, int NH>
struct UpdGrad {
  static constexpr int NE = (KSM + 3) / 4;                   // dW0 column blocks
  static constexpr int NU = NW == 8 ? (4 * NH > NE ? 4 * NH : NE) : 4 * UPD_MAXH + NE;
  // GroupNorm column sums, packed: after the DPP row sum all 16 lanes of a row hold the same
  // value, so lane x keeps value v = 16 r + x of cs[r] — v = 8 hs + i: the weight (i < 4) /
  // bias (i >= 4) sums of head slot hs, v = 8 HPW + i: the trunk's — one or two registers
  // instead of 4 per sum quad
  static constexpr int NV = 8 * HPW + 8, NCS = (NV + 15) / 16;
  upd_v4 w2[HPW];                     // dW2 of head slot hs: [out 4q+i][16b+x]
  float cs[NCS];
  upd_v4 u[NU];
  float bias;                         // wave NW-1, lane l < nout: output bias l
  float loss[3];                      // wave NW-1 (every lane the same sum; lane 0 publishes)
  __device__ upd_v4& w1(int h, int bb) { return u[4 * h + bb]; }   // dW1_h [16b+4q+i][16bb+x]
  __device__ upd_v4& w0(int e) { return u[(NW == 8 ? 0 : 4 * UPD_MAXH) + e]; }
  // add a row sum s (the same in every lane of the row) into packed value v (compile-time)
  __device__ void csadd(int v, float s, int x) { cs[v >> 4] += ((v & 15) == x) ? s : 0.f; }
  __device__ void zero() {
#pragma unroll
    for (int k = 0; k < HPW; ++k) w2[k] = upd_v4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NCS; ++k) cs[k] = 0.f;
#pragma unroll
    for (int k = 0; k < NU; ++k) u[k] = upd_v4{0.f, 0.f, 0.f, 0.f};
    bias = 0.f;
    loss[0] = loss[1] = loss[2] = 0.f;
  }
};
template <int KD, int KA>
using UpdGradOf = UpdGrad<upd_nw<KD, KA>(), upd_hpw<KD, KA>(), upd_ksm<KA>(),
                          KD < 0 ? UPD_MAXH : (upd_kd_discrete(KD) ? 2 : 3)>;
// sums over the tile's rows of a channel quad, added into packed values v0 .. v0 + 3
template <class GR>
__device__ inline void upd_colsum_acc(upd_v4 v, GR& gr, int v0) {
  const int x = threadIdx.x & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i) gr.csadd(v0 + i, upd_rsum16(v[i]), x);
}
// largest head output count (the dW2 rows any lane can hold)
__device__ inline int upd_nomax(const UpdNet& n) {
  const int a = n.out[0] > n.out[1] ? n.out[0] : n.out[1];
  return (n.nh > 2 && n.out[2] > a) ? n.out[2] : a;
}
// 4-B write-through store of image entry k of a partial (buffer resource at the partial's base)
__device__ inline void st1_sc1(__amdgpu_buffer_rsrc_t rs, int k, float x) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), rs, (unsigned)k * 4u, 0, UPD_AUX_SC1);
}

// One tile of the update: forward, loss, backward; the tile's gradient is added into the LDS
// gradient image Ga (every image entry has exactly one owning lane, so no atomics).  Two
// workgroup barriers per tile.  RG: into the register gradient gr instead (Ga unused).
template <int KD, int KA, bool FIRST, bool RG = false>
__device__ void upd_tile(const UpdNet& n, const UpdArgs& args, const float* W, float* Ga,
                         const UpdScr& sc, const UpdIn<upd_ksm<KA>()>& in, int rc, float invB,
                         unsigned long long* tm, UpdGradOf<KD, KA>& gr) {
  constexpr int KSM = upd_ksm<KA>(), NW = upd_nw<KD, KA>(), HPW = upd_hpw<KD, KA>();
  constexpr bool first = FIRST;
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4, w = t >> 6;
  const int b = w & 3, hg = w >> 2;
  const int D = n.D, KS = (D + 3) >> 2;
  const int nh = upd_nh<KD>(n);
  // the marks wait for their s_memrealtime (and the LDS queue): off unless profiling, since every
  // hand-off waits for workgroup 0 too
  const bool timer = args.profile && blockIdx.x == 0 && t == 0;
  unsigned long long tl = timer ? __builtin_amdgcn_s_memrealtime() : 0ull;
#define UPD_CMARK(i)                                                   \
  if (timer) {                                                         \
    const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();  \
    tm[i] += now_ - tl;                                                \
    tl = now_;                                                         \
  }
  UpdFwd<KSM, HPW> f;
  upd_tile_fwd<KD, KA>(n, W, sc, in, f);
  UPD_CMARK(0)
  __syncthreads();   // #1: Op, Rin
  UPD_CMARK(1)
  // ---- loss of row x (lanes q == 0 of every wave, redundantly: each wave needs dO)
  constexpr bool HANDOFF = upd_loss_handoff<NW, KD, KA>();
  const float* dOw = sc.dOs + (HANDOFF ? (w & 3) : w) * 16 * 16;   // [row][j] of this wave (hand-off: its group-0 partner's)
  float lp[3] = {0.f, 0.f, 0.f};
  upd_tile_loss<NW, KD, KA>(n, W, sc, rc, invB, args, lp);
  if constexpr (HANDOFF) __syncthreads();
  else upd_wave_sync();
  UPD_CMARK(2)
  // this wave's [16 rows][16 ch] transpose slots (upd_ts): with one per head, every head stores
  // its G first, then ONE wave sync, so the heads' backward chains below are independent and
  // interleave; with one shared slot each head waits for the previous head's reads
  const int TS = upd_ts(n);
  float* Tw = sc.Ts + w * TS * UPD_RT * 16;
#pragma unroll
  for (int hs = 0; hs < HPW; ++hs)
    if (hs < TS && upd_head<NW>(hs, hg) < nh) upd_st4(Tw + hs * UPD_RT * 16 + x * 16 + 4 * q, f.G[hs]);
  upd_wave_sync();
#pragma unroll
  for (int hs = 0; hs < HPW; ++hs) {
    const int h = upd_head<NW>(hs, hg);
    if (h < nh) {
      const UpdHead hi = upd_head_info(n, h);
      const int oc = hi.oc, no = hi.no;
      const int slot = TS == 1 ? 0 : hs;
      if (hs >= TS) {   // the shared slot is free once the previous head has read it
        upd_wave_sync();
        upd_st4(Tw + x * 16 + 4 * q, f.G[hs]);
        upd_wave_sync();
      }
      const float* Th = Tw + slot * UPD_RT * 16;
      // dW2_h[j][16b + x] += sum_rows dO[row][oc + j] G_h[row][ch]  (G_h transposed via Th)
      upd_v4 acc = {0.f, 0.f, 0.f, 0.f};
      float oa[4], tb[4];   // (every operand read first, in flight together)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        oa[s] = x < no ? dOw[(4 * s + q) * 16 + oc + x] : 0.0f;
        tb[s] = Th[(4 * s + q) * 16 + x];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = upd_mma(oa[s], tb[s], acc);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (RG) {
          if (i < upd_nomax(n)) gr.w2[hs][i] += acc[i];
        } else if (4 * q + i < no) upd_gadd(Ga + hi.w2 + (4 * q + i) * UPD_HS + 16 * b + x, acc[i], first);
      }
      // dG_h^T block b = W2_h^T dO_h^T (K = the head's outputs), GroupNorm + SiLU backward
      upd_v4 dg = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < UPD_MAXA / 4; ++s) {
        if (4 * s < no) {
          const int j = 4 * s + q;
          const float a = j < no ? W[hi.w2 + j * UPD_HS + 16 * b + x] : 0.0f;
          const float bb = j < no ? dOw[x * 16 + oc + j] : 0.0f;
          dg = upd_mma(a, bb, dg);
        }
      }
      const upd_v4 gw = upd_ld4(W + hi.g1 + 16 * b + 4 * q);
      upd_v4 dy;
      const upd_v4 dz = upd_gn_bwd_frag(dg, f.xh[hs], gw, upd_ld4(W + hi.b1 + 16 * b + 4 * q),
                                        f.rh[hs], dy);
      upd_st4(sc.Zs + h * UPD_RT * UPD_ZS + x * UPD_ZS + 16 * b + 4 * q, dz);
      upd_v4 dyx;
#pragma unroll
      for (int i = 0; i < 4; ++i) dyx[i] = dy[i] * f.xh[hs][i];
      if constexpr (RG) {
        upd_colsum_acc(dyx, gr, 8 * hs);
        upd_colsum_acc(dy, gr, 8 * hs + 4);
      } else {
        upd_colsum_add(dyx, Ga + hi.g1 + 16 * b + 4 * q, x == 0, first);
        upd_colsum_add(dy, Ga + hi.b1 + 16 * b + 4 * q, x == 0, first);
      }
    }
  }
  // inputs, rows x channels, for the weight gradients (the trunk output is in Fs already)
#pragma unroll
  for (int s = 0; s < KSM; ++s)
    if (s < KS && (s % NW) == w) sc.Xs[x * sc.XS + 4 * s + q] = in.xin[s];
  UPD_CMARK(3)
  __syncthreads();   // #2: Zs, Fs, Xs
  UPD_CMARK(4)
  // After the barrier, with 8 waves: group 1 takes the head weight gradients (dW1), group 0 the
  // trunk (dF, GroupNorm backward, dW0); with 4 waves each wave does both for its block.
  if (NW == 4 || hg == 1) {
    // ---- dW1_h[16b + 4q + i][16bb + x] += sum_rows dZ_h[row][out] F[row][in]  (K = rows)
#pragma unroll
    for (int h = 0; h < UPD_MAXH; ++h) {
      if (h < nh) {
        const float* Zh = sc.Zs + h * UPD_RT * UPD_ZS;
        // KD = 3 (8-wave three-head net; no LDS form to match bits with): the MFMAs accumulate
        // straight into the register gradient — 16 registers fewer at the kernel's peak
        constexpr bool CHAIN = RG && KD == 3;
        upd_v4 acc[4];
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) acc[bb] = CHAIN ? gr.w1(h, bb) : upd_v4{0.f, 0.f, 0.f, 0.f};
        float za[4], fb[4][4];   // (every operand read first, in flight together)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          za[s] = Zh[(4 * s + q) * UPD_ZS + 16 * b + x];
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) fb[s][bb] = sc.Fs[(4 * s + q) * UPD_ZS + 16 * bb + x];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) acc[bb] = upd_mma(za[s], fb[s][bb], acc[bb]);
        }
        if constexpr (CHAIN) {
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) gr.w1(h, bb) = acc[bb];
        } else if constexpr (RG) {
#pragma unroll
          for (int bb = 0; bb < 4; ++bb)
#pragma unroll
            for (int i = 0; i < 4; ++i) gr.w1(h, bb)[i] += acc[bb][i];
        } else {
          float* gw1 = Ga + n.w1[h].lds + (16 * b + 4 * q) * UPD_HS + x;
#pragma unroll
          for (int bb = 0; bb < 4; ++bb)
#pragma unroll
            for (int i = 0; i < 4; ++i) upd_gadd(gw1 + i * UPD_HS + 16 * bb, acc[bb][i], first);
        }
      }
    }
  }
  UPD_CMARK(5)
  if (NW == 4 || hg == 0) {
    // ---- dF^T block b = sum_h W1_h^T dZ_h^T (K = 64 head channels, permuted so that the A
    //      reads are conflict-free: step s, lane q <-> channel 16 (s & 3) + 4 q + (s >> 2))
    upd_v4 dF;
    {
      upd_v4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < UPD_MAXH; ++h) {
        if (h < nh) {
          const float* Zh = sc.Zs + h * UPD_RT * UPD_ZS + x * UPD_ZS;
          const float* Wh = W + n.w1[h].lds + 16 * b + x;
          // the B operands of a lane's 16 steps are 4 runs of 4 consecutive channels: four
          // 16-B reads up front (same steps, same order)
          upd_v4 zb[4];
#pragma unroll
          for (int sg = 0; sg < 4; ++sg) zb[sg] = upd_ld4(Zh + 16 * sg + 4 * q);
          float wa[16];   // (the A operands read first, in flight together with zb)
#pragma unroll
          for (int s = 0; s < 16; ++s) wa[s] = Wh[(16 * (s & 3) + 4 * q + (s >> 2)) * UPD_HS];
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            if (s & 1) d1 = upd_mma(wa[s], zb[s & 3][s >> 2], d1);
            else d0 = upd_mma(wa[s], zb[s & 3][s >> 2], d0);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) dF[i] = d0[i] + d1[i];
    }
    // trunk GroupNorm + SiLU backward -> dH0 (block b), its weight / bias gradients
    upd_v4 dy0;
    const upd_v4 dH0 = upd_gn_bwd_frag(dF, f.xh0, upd_ld4(W + n.g0.lds + 16 * b + 4 * q),
                                       upd_ld4(W + n.b0.lds + 16 * b + 4 * q), f.r0, dy0);
    {
      upd_v4 dyx;
#pragma unroll
      for (int i = 0; i < 4; ++i) dyx[i] = dy0[i] * f.xh0[i];
      if constexpr (RG) {
        upd_colsum_acc(dyx, gr, 8 * HPW);
        upd_colsum_acc(dy0, gr, 8 * HPW + 4);
      } else {
        upd_colsum_add(dyx, Ga + n.g0.lds + 16 * b + 4 * q, x == 0, first);
        upd_colsum_add(dy0, Ga + n.b0.lds + 16 * b + 4 * q, x == 0, first);
      }
    }
    UPD_CMARK(6)
    // ---- dW0[16b + 4q + i][16e + x] += sum_rows dH0[row][ch] X[row][d]  (dH0 transposed via Tw)
    upd_st4(Tw + x * 16 + 4 * q, dH0);
    upd_wave_sync();
#pragma unroll
    for (int e = 0; e < (KSM + 3) / 4; ++e) {
      if (16 * e < D) {
        upd_v4 acc = {0.f, 0.f, 0.f, 0.f};
        const int d = 16 * e + x;
        float ta[4], xb[4];   // (operands read first, in flight together)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          ta[s] = Tw[(4 * s + q) * 16 + x];
          xb[s] = d < D ? sc.Xs[(4 * s + q) * sc.XS + d] : 0.0f;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = upd_mma(ta[s], xb[s], acc);
        if constexpr (RG) {
#pragma unroll
          for (int i = 0; i < 4; ++i) gr.w0(e)[i] += acc[i];
        } else if (d < D) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            upd_gadd(Ga + n.w0.lds + (16 * b + 4 * q + i) * n.w0.stride + d, acc[i], first);
        }
      }
    }
  }
  // ---- output biases and loss partials (one wave: the last one).  Split loss: the actor's
  //      columns and lp[0], lp[2] come from wave 3's dO rows (written before barrier #2; wave 3
  //      rewrites them only after the next tile's barrier #1)
  if (w == NW - 1) {
    constexpr bool SPLIT = upd_loss_split<NW, KD, KA>();
    const int tl_ = l;
    if (tl_ < n.nout) {   // f64 sum: the softmax outputs' dO cancel across rows
      const float* dOb = (SPLIT && tl_ < n.out[0]) ? sc.dOs + 3 * 16 * 16 : dOw;
      double acc = 0.0;
#pragma unroll
      for (int r = 0; r < UPD_RT; ++r) acc += (double)dOb[r * 16 + tl_];
      if constexpr (RG) gr.bias += (float)acc;
      else upd_gadd(Ga + upd_bias_of(n, tl_), (float)acc, first);
    }
    if constexpr (SPLIT) {
      const float* a = sc.dOs + (3 * 16 + x) * 16 + 12;
      lp[0] = q == 0 ? a[0] : 0.f;
      lp[2] = q == 0 ? a[1] : 0.f;
    }
    if constexpr (HANDOFF) {
      const float* a = sc.dOs + (3 * 16 + x) * 16 + 12;
      lp[0] = q == 0 ? a[0] : 0.f;
      lp[1] = q == 0 ? a[1] : 0.f;
      lp[2] = q == 0 ? a[2] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float s = upd_rsum16(lp[k]);
      if constexpr (RG) gr.loss[k] += s;
      else if (tl_ == 0) upd_gadd(Ga + n.Lp + k, s, first);
    }
  }
  // (the next tile rewrites Tw only after its barrier #0)
  UPD_CMARK(7)
#undef UPD_CMARK
}

// TP: store this lane's register gradient into the workgroup's partial (rs = its base), at the
// image entries the LDS form would have written (the others were zeroed at launch start).
// Lanes x of one register i store 16 consecutive words.
template <int KD, int KA>
__device__ inline void upd_grad_publish(const UpdNet& n, UpdGradOf<KD, KA>& gr,
                                        __amdgpu_buffer_rsrc_t rs) {
  constexpr int KSM = upd_ksm<KA>(), NW = upd_nw<KD, KA>(), HPW = upd_hpw<KD, KA>();
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4, w = t >> 6;
  const int b = w & 3, hg = w >> 2;
  const int D = n.D;
  const int nh = upd_nh<KD>(n);
#pragma unroll
  for (int hs = 0; hs < HPW; ++hs) {
    const int h = upd_head<NW>(hs, hg);
    if (h < nh) {
      const UpdHead hi = upd_head_info(n, h);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < upd_nomax(n) && 4 * q + i < hi.no) st1_sc1(rs, hi.w2 + (4 * q + i) * UPD_HS + 16 * b + x, gr.w2[hs][i]);
    }
  }
  // packed column sums: lane x of register r holds value v = 16 r + x
  using GR = UpdGradOf<KD, KA>;
#pragma unroll
  for (int r = 0; r < GR::NCS; ++r) {
    const int v = 16 * r + x;
    if (v < 8 * HPW) {
      const int h = upd_head<NW>(v >> 3, hg), j = v & 7;
      if (h < nh) {
        const UpdHead hi = upd_head_info(n, h);
        st1_sc1(rs, (j < 4 ? hi.g1 : hi.b1) + 16 * b + 4 * q + (j & 3), gr.cs[r]);
      }
    } else if (v < GR::NV && (NW == 4 || hg == 0)) {
      const int j = v - 8 * HPW;
      st1_sc1(rs, (j < 4 ? n.g0.lds : n.b0.lds) + 16 * b + 4 * q + (j & 3), gr.cs[r]);
    }
  }
  if (NW == 4 || hg == 1) {
#pragma unroll
    for (int h = 0; h < UPD_MAXH; ++h) {
      if (h < nh) {
        const int base = n.w1[h].lds + (16 * b + 4 * q) * UPD_HS + x;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
          for (int i = 0; i < 4; ++i) st1_sc1(rs, base + i * UPD_HS + 16 * bb, gr.w1(h, bb)[i]);
      }
    }
  }
  if (NW == 4 || hg == 0) {
#pragma unroll
    for (int e = 0; e < (KSM + 3) / 4; ++e) {
      const int d = 16 * e + x;
      if (16 * e < D && d < D) {
#pragma unroll
        for (int i = 0; i < 4; ++i) st1_sc1(rs, n.w0.lds + (16 * b + 4 * q + i) * n.w0.stride + d, gr.w0(e)[i]);
      }
    }
  }
  if (w == NW - 1) {
    if (l < n.nout) st1_sc1(rs, upd_bias_of(n, l), gr.bias);
    if (l == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) st1_sc1(rs, n.Lp + k, gr.loss[k]);
    }
  }
}

__device__ inline float f4get(const float4& v, int e) {
  return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}
__device__ inline void f4set(float4& v, int e, float x) {
  if (e == 0) v.x = x; else if (e == 1) v.y = x; else if (e == 2) v.z = x; else v.w = x;
}

// sum of quad q over partials gg = first, first + stride, ... < G (in that order), loads issued
// in batches of NB so their latencies overlap (NB = 8 for the 8-wave kernel: its 256 registers
// per lane cannot hold 16 quads in flight without spilling around the phase)
template <int NB = 16>
__device__ inline void upd_sum_partials(__amdgpu_buffer_rsrc_t rs_part, int Qtot, int q, int first,
                                        int stride, int G, double& ax, double& ay, double& az,
                                        double& aw) {
  for (int g0 = first; g0 < G; g0 += NB * stride) {
    float4 v[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int gg = g0 + u * stride;
      if (gg < G) v[u] = ld4_sc1(rs_part, ((size_t)gg * Qtot + q) * 4);
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      if (g0 + u * stride < G) {
        ax += v[u].x; ay += v[u].y; az += v[u].z; aw += v[u].w;
      }
    }
  }
}

// ---- AdamW pieces shared by ppo_adam_kernel and the folded prologue of ppo_grad_kernel: one
// arithmetic, so the folded and the separate AdamW give the same bits.
struct AdamConst {
  float step_size, inv_bc2_sqrt, decay, omb1, omb2, beta2, eps;
};
__device__ __forceinline__ AdamConst adam_const(double tstep, float lr, double beta1, double beta2,
                                                float eps, float wd) {
  const double bc1 = 1.0 - pow((double)beta1, tstep);
  const double bc2 = 1.0 - pow((double)beta2, tstep);
  AdamConst c;
  c.step_size = (float)((double)lr / bc1);
  c.inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
  c.decay = (float)(1.0 - (double)lr * (double)wd);
  c.omb1 = (float)(1.0 - (double)beta1);
  c.omb2 = (float)(1.0 - (double)beta2);
  c.beta2 = (float)beta2;
  c.eps = eps;
  return c;
}
__device__ __forceinline__ float adam_sq4(float4 r) { return r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w; }
// clip coefficient from this thread's partial sum of squares; 256 threads, 4 wave partials in
// s_part (LDS), summed in wave order (every workgroup forms the same value)
__device__ __forceinline__ float adam_clip(float acc, float max_norm, float* s_part) {
  const int t = threadIdx.x;
  acc = wave_sum(acc);
  if ((t & 63) == 0) s_part[t >> 6] = acc;
  __syncthreads();
  float tot = 0.f;
  for (int w = 0; w < UPD_THREADS / 64; ++w) tot += s_part[w];
  const float coef = max_norm / (sqrtf(tot) + 1e-6f);
  return coef < 1.0f ? coef : 1.0f;
}
__device__ __forceinline__ void adam_quad(const AdamConst& c, float clipc, float4 g4, float4& m4,
                                          float4& v4, float4& pw) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float gr = f4get(g4, e) * clipc;
    float m = f4get(m4, e), v = f4get(v4, e), p = f4get(pw, e);
    p = p * c.decay;
    m = m + c.omb1 * (gr - m);
    v = v * c.beta2 + c.omb2 * gr * gr;
    const float denom = __builtin_amdgcn_sqrtf(v) * c.inv_bc2_sqrt + c.eps;
    float rq = __builtin_amdgcn_rcpf(denom);
    rq = rq * (2.0f - denom * rq);
    p = p - c.step_size * (m * rq);
    f4set(m4, e, m);
    f4set(v4, e, v);
    f4set(pw, e, p);
  }
}
__device__ __forceinline__ float adam_loss(const float* grad, int Lp, float inv_count, float vf_coef,
                                           float ent_coef) {
  const float4 lp = *reinterpret_cast<const float4*>(grad + Lp);
  return lp.x * inv_count + vf_coef * (lp.y * inv_count) - ent_coef * (lp.z * inv_count);
}

// Diagnostic sub-phase marks (PRL_UPD_PROFILE=1, workgroup 0, thread 0): time since the
// current phase began (pts[7]) added into acc[i]; off (null) in normal runs.
struct UpdSub {
  unsigned long long* acc;
  const unsigned long long* ref;
  __device__ inline void mark(int i) const {
    if (acc && threadIdx.x == 0) acc[i] += __builtin_amdgcn_s_memrealtime() - *ref;
  }
};

// Phase B: workgroup g sums its slice [qlo, qhi) of the G slices of the gradient quads over the
// Gp partials in workgroup order (deterministic) with float64 accumulators (the partials of the
// output biases cancel across workgroups), publishes the slice (sc1) and returns this thread's
// share of the slice's sum of squares (parameter quads only).  Uses scratch as [spl][nq] double4.
// (Gp < G: the latency form's replicated tiles, one partial per tile group; see ppo_update_body.)
__device__ inline float upd_slice_reduce(__amdgpu_buffer_rsrc_t rs_part, __amdgpu_buffer_rsrc_t rs_red,
                                         int Qtot, int Qp, int g, int G, float* scratch, int NT,
                                         int aux = UPD_AUX_SC1, UpdSub sub = UpdSub{nullptr, nullptr},
                                         int Gp = -1) {
  if (Gp < 0) Gp = G;
  const int t = threadIdx.x;
  const int qlo = (int)((int64_t)Qtot * g / G), qhi = (int)((int64_t)Qtot * (g + 1) / G);
  const int nq = qhi - qlo;
  float ssq = 0.f;
  auto fin = [&](int qi, double ax, double ay, double az, double aw) {
    const float4 r = float4{(float)ax, (float)ay, (float)az, (float)aw};
    if (aux == UPD_AUX_SYS) st4_aux<UPD_AUX_SYS>(rs_red, (size_t)(qlo + qi) * 4, r);
    else st4_aux<UPD_AUX_SC1>(rs_red, (size_t)(qlo + qi) * 4, r);
    if (qlo + qi < Qp) ssq += r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w;
  };
  if (nq > NT / 2) {
    // wide slices (few workgroups): each thread owns whole quads, partials summed in order
    for (int qi = t; qi < nq; qi += NT) {
      double ax = 0.0, ay = 0.0, az = 0.0, aw = 0.0;
      if (NT > 256) upd_sum_partials<8>(rs_part, Qtot, qlo + qi, 0, 1, Gp, ax, ay, az, aw);
      else upd_sum_partials<16>(rs_part, Qtot, qlo + qi, 0, 1, Gp, ax, ay, az, aw);
      fin(qi, ax, ay, az, aw);
    }
  } else if (nq > 0) {
    // narrow slices: split the G partials of each quad over spl threads, combine in LDS
    int spl = 1;
    while (spl * 2 * nq <= NT && spl * 2 <= Gp) spl *= 2;
    double* red = reinterpret_cast<double*>(scratch);   // [spl][nq][4]
    if (t < spl * nq) {
      const int qi = t % nq, sub_ = t / nq;
      double ax = 0.0, ay = 0.0, az = 0.0, aw = 0.0;
      if (NT > 256) upd_sum_partials<8>(rs_part, Qtot, qlo + qi, sub_, spl, Gp, ax, ay, az, aw);
      else upd_sum_partials<16>(rs_part, Qtot, qlo + qi, sub_, spl, Gp, ax, ay, az, aw);
      double* o = red + 4 * (sub_ * nq + qi);
      o[0] = ax; o[1] = ay; o[2] = az; o[3] = aw;
    }
    sub.mark(0);   // thread 0's partial loads landed and summed
    __syncthreads();
    if (t < nq) {
      double ax = red[4 * t], ay = red[4 * t + 1], az = red[4 * t + 2], aw = red[4 * t + 3];
      for (int k = 1; k < spl; ++k) {
        const double* o = red + 4 * (k * nq + t);
        ax += o[0]; ay += o[1]; az += o[2]; aw += o[3];
      }
      fin(t, ax, ay, az, aw);
    }
  }
  return ssq;
}

// Data-parallel ranks (world > 1, one persistent launch per rank): this workgroup's slice of the
// step's gradient summed over ranks.  Workgroup g of every rank has just written its rank-local
// slice into its own xbuf[par] (system-scope stores, drained); it raises its flag to the step's
// exchange sequence number + 1 (the caller continues the sequence from launch to launch, so the
// flags only grow and are never reset), waits until workgroup
// g of every rank has, then sums the world slices in rank order (float32, as the stepped path's
// all-reduce) into red, where phase C reads the reduced gradient.  xbuf is double-buffered by
// step parity: a rank rewrites xbuf[par] two steps later, by which time every rank has raised
// the flag of the step in between, i.e. has finished reading this one.
// Ordering: the flag store and the polls are RELAXED system-scope atomics on purpose.  The slice
// stores before it are system-scope (sc0 sc1: written through to memory) and drained by the
// caller's s_waitcnt vmcnt(0) before this store issues; the slice loads after the poll are
// system-scope too (they miss every cache), and the __syncthreads below orders them after the
// poll.  A formal system-scope release / acquire would add buffer_wbl2 / buffer_inv of the whole
// L2 per workgroup per step, writing back or dropping the minibatch rows every workgroup keeps
// in L2, for ordering the encodings already give.  That argument holds for the uncached
// allocation only; when any rank's buffer is fine-grained (prl_dp_xbuf_alloc's fallback,
// args.dp_fine) the flag store follows a system-scope release and the slice loads a system-scope
// acquire.

// The head-split form's clip-norm pieces (prl_ppo_split.h, spl_piece): chunks of 4 reduced-gradient
// quads, piece = ((q0^2 + q1^2) + (q2^2 + q3^2)) of ((x^2 + y^2) + (z^2 + w^2)), formed here for the
// data-parallel union slices exactly as the single-GPU slice owners form them.
__device__ inline float upd_sq4(float4 r) { return (r.x * r.x + r.y * r.y) + (r.z * r.z + r.w * r.w); }
__device__ inline void upd_piece(float* pieces, float sqv, int q, bool valid) {
  sqv += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(sqv), 0xB1, 0xF, 0xF, false));
  sqv += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(sqv), 0x4E, 0xF, 0xF, false));
  if (valid && (q & 3) == 0) st_sc1f(pieces + q / 4, sqv);
}

__device__ bool upd_dp_union_slice(const UpdArgs& args, __amdgpu_buffer_rsrc_t rs_red, int Qtot,
                                   int g, int G, unsigned long long gstep, int par, int* s_abort,
                                   int qlo_in = -1, int qhi_in = -1, float* pieces = nullptr) {
  const int t = threadIdx.x, NT = blockDim.x;
  const unsigned long long want = gstep + 1ull;
  if (t == 0) {
    if (args.dp_fine) {
      // fine-grained slice buffers (prl_dp_xbuf_alloc's fallback) may be cached: a system-scope
      // release makes this workgroup's drained slice stores visible before its flag (the asm
      // wait keeps the compiler from dropping the release's wait, MI355X_MICROARCH.md)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_store(upd_g(args.xflag_self + g), want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (t < 64) {
    unsigned long long* fl = args.xflag[0];   // lane r polls rank r (selected, not indexed)
#pragma unroll
    for (int r = 1; r < UPD_MAX_RANKS; ++r)
      if (t == r) fl = args.xflag[r];
    bool ok = true;
    for (unsigned spins = 0;; ++spins) {
      // lanes < world poll the ranks' flags, lane 63 the abort word, in one round
      const bool ready = t >= args.world ||
                         __hip_atomic_load(upd_g(fl + g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= want;
      const unsigned ab = t == 63 ? ld_sc1u(args.ctr + 2) : 0u;
      if (__ballot(!ready) == 0ull) break;
      if ((unsigned)__builtin_amdgcn_readlane((int)ab, 63) != 0u) { ok = false; break; }
      if (spins > args.dp_spin_limit) {
        if (t == 0) {
          __hip_atomic_store(upd_g(args.ctr + 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(upd_g(args.ctr + 3), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_or(upd_g(args.ctr + 4), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (t == 0) *s_abort = ok ? 0 : 1;
    if (args.dp_fine && ok) {
      // ... and a system-scope acquire after the matched poll, before any slice load (the
      // workgroup barrier below holds the other waves until it has completed)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (*s_abort) return false;
  // this workgroup's slice: phase B's (uniform, or the split form's load-balanced one)
  const int qlo = qlo_in >= 0 ? qlo_in : (int)((int64_t)Qtot * g / G);
  const int qhi = qhi_in >= 0 ? qhi_in : (int)((int64_t)Qtot * (g + 1) / G);
  const size_t base = (size_t)par * Qtot * 4;
  // (uniform trip count: the split form's norm pieces, spl_piece, need every lane)
  for (int q0 = qlo; q0 < qhi; q0 += NT) {
    const int q = q0 + t;
    float sqv = 0.f;
    if (q < qhi) {
      float4 acc = ld4_aux<UPD_AUX_SYS>(upd_rsrc(args.xbuf[0] + base), (size_t)q * 4);
#pragma unroll
      for (int r = 1; r < UPD_MAX_RANKS; ++r) {
        if (r < args.world) {
          const float4 x = ld4_aux<UPD_AUX_SYS>(upd_rsrc(args.xbuf[r] + base), (size_t)q * 4);
          acc.x += x.x;
          acc.y += x.y;
          acc.z += x.z;
          acc.w += x.w;
        }
      }
      st4_sc1(rs_red, (size_t)q * 4, acc);
      sqv = q < Qtot - 1 ? upd_sq4(acc) : 0.f;
    }
    if (pieces) upd_piece(pieces, sqv, q, q < qhi && q < Qtot - 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  return true;
}

// The PUSH form of the cross-rank step (dp_push; the head-split kernel's data-parallel form):
// phase B has already stored this workgroup's slice into EVERY rank's receive slot
// [par][this rank] (system-scope stores, drained by the caller); one lane now raises this
// workgroup's flag in every rank's receive flags [this rank][g] (remote writes are posted: one
// one-way trip over xGMI instead of the pull form's remote poll + remote slice read), then a wave
// polls its OWN buffer's flags [r][g] for every rank r (local loads) and the slices are summed
// from local memory in rank order into red.  Ordering as the pull form: system-scope stores
// drained before the flag store, system-scope loads after the matched poll, a system-scope
// release / acquire around them when any buffer is fine-grained.  Reuse of a receive slot: rank
// r rewrites [par][r] two steps later, after every rank raised the flag of the step between,
// i.e. finished reading this one.
__device__ bool upd_dp_union_slice_push(const UpdArgs& args, __amdgpu_buffer_rsrc_t rs_red, int Qtot,
                                        int g, unsigned long long gstep, int par, int* s_abort,
                                        int qlo, int qhi, float* pieces = nullptr) {
  const int t = threadIdx.x, NT = blockDim.x;
  const unsigned long long want = gstep + 1ull;
  if (t == 0) {
    if (args.dp_fine) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int r = 0; r < UPD_MAX_RANKS; ++r) {
      if (r < args.world) {
        unsigned long long* fl = reinterpret_cast<unsigned long long*>(args.xbuf[r]) + args.xpush_flags_off +
                                 (size_t)args.rank * args.xpush_gmax + g;
        __hip_atomic_store(upd_g(fl), want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  if (t < 64) {
    const unsigned long long* fl = reinterpret_cast<const unsigned long long*>(args.xbuf_self) +
                                   args.xpush_flags_off + (size_t)(t < UPD_MAX_RANKS ? t : 0) * args.xpush_gmax + g;
    bool ok = true;
    for (unsigned spins = 0;; ++spins) {
      const bool ready = t >= args.world ||
                         __hip_atomic_load(upd_g(fl), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= want;
      const unsigned ab = t == 63 ? ld_sc1u(args.ctr + 2) : 0u;
      if (__ballot(!ready) == 0ull) break;
      if ((unsigned)__builtin_amdgcn_readlane((int)ab, 63) != 0u) { ok = false; break; }
      if (spins > args.dp_spin_limit) {
        if (t == 0) {
          __hip_atomic_store(upd_g(args.ctr + 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(upd_g(args.ctr + 3), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_or(upd_g(args.ctr + 4), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (t == 0) *s_abort = ok ? 0 : 1;
    if (args.dp_fine && ok) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (*s_abort) return false;
  const __amdgpu_buffer_rsrc_t rs_rx = upd_rsrc(args.xbuf_self + args.xpush_off +
                                                (size_t)par * UPD_MAX_RANKS * Qtot * 4);
  for (int q0 = qlo; q0 < qhi; q0 += NT) {
    const int q = q0 + t;
    float sqv = 0.f;
    if (q < qhi) {
      float4 acc = ld4_aux<UPD_AUX_SYS>(rs_rx, (size_t)q * 4);
#pragma unroll
      for (int r = 1; r < UPD_MAX_RANKS; ++r) {
        if (r < args.world) {
          const float4 x = ld4_aux<UPD_AUX_SYS>(rs_rx, ((size_t)r * Qtot + q) * 4);
          acc.x += x.x;
          acc.y += x.y;
          acc.z += x.z;
          acc.w += x.w;
        }
      }
      st4_sc1(rs_red, (size_t)q * 4, acc);
      sqv = q < Qtot - 1 ? upd_sq4(acc) : 0.f;
    }
    if (pieces) upd_piece(pieces, sqv, q, q < qhi && q < Qtot - 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  return true;
}

// NQ = parameter quads per thread (ceil(Lp / 4 / 256)): AdamW's moments live in registers.
// DP: the data-parallel form (prl_ppo_update_dpx): union-minibatch row weights and the
// cross-rank slice sum; a separate instantiation, so the single-GPU kernel carries none of it.
// TP: the throughput form for many tiles per workgroup and step (upd_tp_host): the gradient in
// registers (UpdGrad, no LDS image) and the moments streamed from device memory in phase C
// instead of held in registers — the owner of each slice writes its new moments to the other of
// two buffers (the step's source for the next step) — so the tiles run with ~110 more registers
// and without the image's LDS traffic.  Needs >= 2 steps (upd_run).  TPM: 1 = the throughput form.
template <int NQ, int KD, int KA, bool DP, int TPM = 0>
__device__ __forceinline__ void ppo_update_body(const UpdNet& n, const UpdArgs& args) {
  constexpr int NW = upd_nw<KD, KA>(), NT = 64 * NW;
  constexpr bool TP = TPM > 0;
  extern __shared__ __align__(16) float upd_lds[];
  const int t = threadIdx.x, g = blockIdx.x, G = args.G;
  // Replicated tiles (latency form, single GPU, PRL_UPD_REPL): workgroups g, g + Gt, g + 2 Gt, ...
  // run the SAME rows (tile group gt = g % Gt: same inputs, same code, the same partial gradient
  // bits) and each publishes only its 1/X share of that partial, so the publish moves 1/X of the
  // bytes per workgroup and phase B's G slices are X times narrower; every workgroup then takes
  // the whole reduced gradient in phase C as before.  Gt == G: no replication.
  const int Gt = (TP || DP) ? G : args.Gt;
  const int gt = (TP || DP) ? g : g % Gt;
  const int Lp = n.Lp;
  const int Qp = Lp / 4;            // parameter quads
  const int Qtot = Qp + 1;          // + one quad of loss partials
  float* hdr = upd_lds;             // [64] broadcast words + chunk stage timers
  // LDS: header | tile scratch | parameter image W | gradient image Ga (not TP).  The scratch
  // sits below 64 KB so every scratch address folds into the ds instructions' 16-bit offset field
  // (no base registers kept live across the step loop)
  float* scratch = upd_lds + UPD_HDR;                                   // tile activations
  const int scr_floats = (upd_scratch_floats(n.D, NW, upd_ts(n)) + 3) & ~3;
  float* W = scratch + scr_floats;                                       // [Lp]
  float* Ga = W + Lp;                                                    // [Lp + 4]
  const UpdScr sc = upd_scr(scratch, n.D, NW);
  int* s_abort = reinterpret_cast<int*>(hdr + 8);
  float* s_adam = hdr + 10;         // [2] this step's AdamW step size, 1 / sqrt(bc2)

  // ---- load the parameter image into LDS and this thread's moment quads (q = t + NT i) into
  //      registers: args.params / exp_avg / exp_avg_sq are IMAGES here (prl_ppo_update converts
  //      the flat torch vectors around the launch), so no layout arithmetic stays live in SGPRs
  constexpr int NQR = TP ? 1 : NQ;
  float4 mreg[NQR], vreg[NQR];
  for (int q = t; q < Qp; q += NT)
    *reinterpret_cast<float4*>(W + 4 * q) = *reinterpret_cast<const float4*>(args.params + 4 * q);
  if constexpr (!TP) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int q = t + i * NT;
      mreg[i] = q < Qp ? *reinterpret_cast<const float4*>(args.exp_avg + 4 * q) : float4{0.f, 0.f, 0.f, 0.f};
      vreg[i] = q < Qp ? *reinterpret_cast<const float4*>(args.exp_avg_sq + 4 * q) : float4{0.f, 0.f, 0.f, 0.f};
    }
  } else {
    // the register gradient covers only real entries: the rest of this workgroup's partial
    // (padding) is zeroed here once, drained before the first publish
    const __amdgpu_buffer_rsrc_t rs_mypart = upd_rsrc(args.part + (size_t)g * Qtot * 4);
    for (int q = t; q < Qtot; q += NT) st4_sc1(rs_mypart, (size_t)q * 4, float4{0.f, 0.f, 0.f, 0.f});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  const float step0 = args.adam_step[0];
  if (t < 24) reinterpret_cast<unsigned long long*>(hdr + 16)[t] = 0ull;
  __syncthreads();
  if constexpr (!TP) {
    for (int k = t; k < Lp + 4; k += NT) Ga[k] = 0.0f;   // padding stays 0 for good
    __syncthreads();
  }

  const int R = args.R;
  float loss_last = 0.f;
  // phase timers of workgroup 0 live in LDS (hdr + 64: pt[7], tp, rt0, ck0), not in SGPRs:
  // the step loop is short of scalar registers
  unsigned long long* const pts = reinterpret_cast<unsigned long long*>(hdr + 64);
  if (g == 0 && t == 0) {
    for (int i = 0; i < 7; ++i) pts[i] = 0ull;
    pts[7] = __builtin_amdgcn_s_memrealtime();
    pts[8] = pts[7];
    pts[9] = __builtin_amdgcn_s_memtime();
  }
  const UpdSub subm{(args.profile && g == 0) ? reinterpret_cast<unsigned long long*>(hdr + 16) + 8
                                              : nullptr, pts + 7};
  auto mark = [&](int i) {
    if (args.profile && g == 0 && t == 0) {
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      pts[i] += now - pts[7];
      pts[7] = now;
    }
  };
  UpdIn<upd_ksm<KA>()> nin[1];   // inputs of the next tile to run (prefetched)
  // load the tile at row0 (rows_left rows of this workgroup's share from there on)
  auto load_next = [&](int64_t row0, int rows_left) {
    upd_tile_load<KD, KA, true>(n, args.S, args.act, args.old_logp, args.adv, args.ret, row0,
                                std::min(UPD_RT, rows_left), nin[0]);
  };
  unsigned long long* const tm = reinterpret_cast<unsigned long long*>(hdr + 16);
  // step s's first tile: its rows of minibatch s % nb (0 rows: every slot a dummy load)
  auto first_row = [&](int s) { return (int64_t)(s % args.nb) * args.mb + (int64_t)gt * R; };
  auto first_rows = [&](int s) {
    const int64_t fmb0 = (int64_t)(s % args.nb) * args.mb;
    const int fB = (int)std::min<int64_t>(args.mb, args.N - fmb0);
    return args.profile == 2 ? 0 : std::max(0, std::min(R, fB - gt * R));
  };
  auto load_first = [&](int s) { load_next(first_row(s), first_rows(s)); };
  // Every prefetch is unconditional (clamped arguments instead of branches around it): a load
  // under a branch made the compiler join nin's paths with copies that waited for the loads on
  // the spot.
  load_first(0);
  for (int s = 0; s < args.total_steps; ++s) {
    const int j = s % args.nb;
    const int64_t mb0 = (int64_t)j * args.mb;
    const int B = (int)std::min<int64_t>(args.mb, args.N - mb0);
    const float invB = DP ? args.inv_count[j] : 1.0f / (float)B;
    // profile mode 2 (PRL_UPD_PROFILE=2, diagnostics only): no rows, i.e. the exchange alone
    const int myrows = args.profile == 2 ? 0 : std::max(0, std::min(R, B - gt * R));
    const int64_t myrow0 = mb0 + (int64_t)gt * R;
    // ---- phase A: partial gradient of this workgroup's rows ------------------------------------
    UpdGradOf<KD, KA> gr;
    if constexpr (TP) gr.zero();
    if (!TP && myrows == 0) {   // no rows this step: publish zeros
      for (int k = t; k < Lp + 4; k += NT) Ga[k] = 0.0f;
    }
    for (int c0 = 0; c0 < myrows; c0 += UPD_RT) {
      const UpdIn<upd_ksm<KA>()> cur = upd_in_real(nin[0]);
      // prefetch the next tile to run: this step's next one, else the next step's first (runs
      // under this tile and the step's hand-offs)
      const bool more = c0 + UPD_RT < myrows;
      if constexpr (TP) {   // many tiles per step: the next step's first after the publish
        if (more) load_next(myrow0 + c0 + UPD_RT, myrows - c0 - UPD_RT);
      } else {
        load_next(more ? myrow0 + c0 + UPD_RT : first_row(s + 1),
                  more ? myrows - c0 - UPD_RT : first_rows(s + 1));
      }
      if constexpr (TP)
        upd_tile<KD, KA, false, true>(n, args, W, Ga, upd_scr_tile(sc, c0 / UPD_RT), cur, std::min(UPD_RT, myrows - c0),
                                      invB, tm, gr);
      else if (c0 == 0)
        upd_tile<KD, KA, true>(n, args, W, Ga, upd_scr_tile(sc, c0 / UPD_RT), cur, std::min(UPD_RT, myrows - c0), invB,
                               tm, gr);
      else
        upd_tile<KD, KA, false>(n, args, W, Ga, upd_scr_tile(sc, c0 / UPD_RT), cur, std::min(UPD_RT, myrows - c0), invB,
                                tm, gr);
    }
    if constexpr (!TP) __syncthreads();
    mark(0);   // phase A compute
    const __amdgpu_buffer_rsrc_t rs_part = upd_rsrc(args.part), rs_red = upd_rsrc(args.red);
    if constexpr (TP) {
      upd_grad_publish<KD, KA>(n, gr, upd_rsrc(args.part + (size_t)g * Qtot * 4));
    } else {
      // replica g / Gt of tile group gt publishes quads [qa, qb) of the group's partial
      const int rep = g / Gt, X = G / Gt;
      const int qa = (int)((int64_t)Qtot * rep / X), qb = (int)((int64_t)Qtot * (rep + 1) / X);
      for (int q = qa + t; q < qb; q += NT)
        st4_sc1(rs_part, ((size_t)gt * Qtot + q) * 4, *reinterpret_cast<const float4*>(Ga + 4 * q));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    mark(1);   // publish partials
    // the latency form prefetched the next step's first tile at its tile's start (no tile ran:
    // here); the throughput form here, under the waits (at the last tile's start its loads
    // were still in flight at the publish drain: +0.7-0.9 us per step at mb 65,536)
    if (TP || myrows == 0) load_first(s + 1);
    if (t < 64) {
      if (t == 0) upd_arrive(args.ctr, UPD_CTR_A, g);
      const bool ok = upd_wait_sharded(args.ctr, UPD_CTR_A, (unsigned)G * (unsigned)(s + 1));
      if (t == 0) *s_abort = ok ? 0 : 1;
    } else if (t == 64) {
      // this step's AdamW bias corrections (float64 pow, as torch's AdamW) on the second wave,
      // which only waits at the barrier: off the polling wave's path (for the last workgroup
      // to arrive the poll ends at once, and its phase B gates every other workgroup)
      const double tstep = (double)step0 + (double)(s + 1);
      const double bc1 = 1.0 - pow((double)args.beta1, tstep);
      const double bc2 = 1.0 - pow((double)args.beta2, tstep);
      s_adam[0] = (float)((double)args.lr / bc1);   // step size
      s_adam[1] = (float)(1.0 / sqrt(bc2));         // 1 / sqrt(bias correction 2)
    }
    __syncthreads();
    if (*s_abort) return;
    mark(2);   // wait A
    // ---- phase B: reduce this workgroup's slice over the G partials --------------------------
    {
      constexpr bool dp = DP;
      const unsigned long long gstep = args.dp_seq0 + (unsigned long long)s;
      const int par = (int)(gstep & 1ull);
      (void)upd_slice_reduce(rs_part, dp ? upd_rsrc(args.xbuf_self + (size_t)par * Qtot * 4) : rs_red,
                             Qtot, Qp, g, G, scratch, NT, dp ? UPD_AUX_SYS : UPD_AUX_SC1, subm, Gt);
      subm.mark(1);   // slice combined, its stores issued
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (dp && !upd_dp_union_slice(args, rs_red, Qtot, g, G, gstep, par, s_abort)) return;
      mark(3);   // slice reduce
      if (t < 64) {
        if (t == 0) upd_arrive(args.ctr, UPD_CTR_B, g);
        const bool ok = upd_wait_sharded(args.ctr, UPD_CTR_B, (unsigned)G * (unsigned)(s + 1));
        if (t == 0) *s_abort = ok ? 0 : 1;
      }
      __syncthreads();
      if (*s_abort) return;
      mark(4);   // wait B
    }
    // ---- phase C: clip_grad_norm_(2.0) + AdamW on every workgroup's own copy ------------------
    // this thread's gradient quads: every load issued at once under a wave-uniform condition (a
    // per-lane `q < Qp` guard put the last quads under divergent exec masks, and with 8 waves the
    // compiler then drained each of them to a spill slot before issuing the next: three round
    // trips instead of one).  Lanes past Qp read the workspace that follows `red` (its loss quad,
    // then `part`): garbage, masked below.
    float4 gq[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i)
      if (i * NT < Qp) gq[i] = ld4_sc1_so(rs_red, 16u * (unsigned)t, 16u * (unsigned)(i * NT));
    // TP: this step's moments (written by the slice owners last step; the launch's images at
    // step 0), loaded with the gradient; the new ones go to the other buffer (the images at the
    // last step: every workgroup read them at step 0 only, before the barriers since)
    constexpr int NQM = TP ? NQ : 1;
    float4 mq[NQM], vq[NQM];
    const bool lastst = s + 1 == args.total_steps;
    const float* msrc = s == 0 ? args.exp_avg : ((s & 1) ? args.tp_m1 : args.tp_m0);
    const float* vsrc = s == 0 ? args.exp_avg_sq : ((s & 1) ? args.tp_v1 : args.tp_v0);
    float* mdst = lastst ? args.exp_avg : ((s & 1) ? args.tp_m0 : args.tp_m1);
    float* vdst = lastst ? args.exp_avg_sq : ((s & 1) ? args.tp_v0 : args.tp_v1);
    if constexpr (TP) {
      const __amdgpu_buffer_rsrc_t rm = upd_rsrc(msrc), rv = upd_rsrc(vsrc);
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        if (i * NT < Qp) {
          mq[i] = ld4_sc1_so(rm, 16u * (unsigned)t, 16u * (unsigned)(i * NT));
          vq[i] = ld4_sc1_so(rv, 16u * (unsigned)t, 16u * (unsigned)(i * NT));
        }
      }
    }
    // 8 waves (two per SIMD, 256 registers each): park the quads in the gradient image, free
    // since the publish, so they do not stay live across the norm into AdamW
    constexpr bool PARK = NW == 8 && !TP;
    float* const park = Ga;
    float clipc;
    {
      // clip_grad_norm_'s norm from the reduced gradient this workgroup just loaded: per thread
      // its quads in order, a fixed DPP tree per wave, the NW wave sums in wave order (LDS) — the
      // same data, order and code in every workgroup, so every copy forms the same coefficient.
      // (Round 1 summed per-slice pieces published by the slice owners instead: those 4-B words,
      // eight workgroups' to a 128-B line, were read stale on some runs — a wrong clip
      // coefficient, run-to-run differences; tools/exp/engine_determinism4.py.)
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        if (i * NT < Qp && t + i * NT < Qp) {
          acc += (gq[i].x * gq[i].x + gq[i].y * gq[i].y) + (gq[i].z * gq[i].z + gq[i].w * gq[i].w);
          if (PARK) *reinterpret_cast<float4*>(park + 4 * (t + i * NT)) = gq[i];
        }
      }
      subm.mark(2);   // thread 0's gradient quads landed
      acc = wave_sum_f32_to63(acc);
      float* s_nrm = hdr + 96;  // [NW <= 16] (hdr + 8 / + 10 hold s_abort / s_adam)
      if ((t & 63) == 63) s_nrm[t >> 6] = acc;
      __syncthreads();
      float tot = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) tot += s_nrm[w];
      const float coef = args.max_norm / (sqrtf(tot) + 1e-6f);
      clipc = coef < 1.0f ? coef : 1.0f;
      // profile: steps whose clip_grad_norm_ scaled the gradient (prof[28])
      if (args.profile && g == 0 && t == 0 && coef < 1.0f) tm[20] += 1ull;
      if (g == 0 && t == 0 && s + 1 == args.total_steps) {
        const float4 lp = ld4_sc1(rs_red, (size_t)Qp * 4);
        loss_last = lp.x * invB + args.vf_coef * (lp.y * invB) - args.ent_coef * (lp.z * invB);
      }
    }
    mark(5);   // norm + loss
    {
      const float step_size = s_adam[0];
      const float inv_bc2_sqrt = s_adam[1];   // scalar divide -> one multiply
      const float decay = (float)(1.0 - (double)args.lr * (double)args.wd);
      const float b2 = (float)args.beta2;
      const float omb1 = (float)(1.0 - (double)args.beta1), omb2 = (float)(1.0 - (double)args.beta2);
      constexpr int BATCH = NQ;
#pragma unroll
      for (int i0 = 0; i0 < NQ; i0 += BATCH) {
#pragma unroll
        for (int b = 0; b < BATCH; ++b) {
          const int i = i0 + b;
          const int q = t + i * NT;
          if (i < NQ && q < Qp) {
            float4 pw = *reinterpret_cast<float4*>(W + 4 * q);
            float4 m4, v4;
            if constexpr (TP) {
              m4 = mq[i];
              v4 = vq[i];
            } else {
              m4 = mreg[i];
              v4 = vreg[i];
            }
            const float4 g4 = PARK ? *reinterpret_cast<const float4*>(park + 4 * q) : gq[i];
            // torch AdamW (decoupled decay; lerp for m; addcmul for v) with fused multiply-adds.
            // 8 waves: two elements per packed-f32 instruction (v_pk_mul / v_pk_fma: the same
            // operations per element, so the same bits as the scalar form; sqrt / rcp scalar):
            // CartPole mb 512 AdamW 1.32 -> 1.23 us; the 4-wave Pendulum kernel (14 quads per
            // thread) measured slower packed (2.03 -> 2.36 us) and keeps the scalar form
            if constexpr (NW == 4) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float gr = f4get(g4, e) * clipc;
                float m = f4get(m4, e), v = f4get(v4, e), p = f4get(pw, e);
                p = p * decay;
                m = fmaf(omb1, gr - m, m);
                v = fmaf(omb2 * gr, gr, v * b2);
                const float denom = fmaf(__builtin_amdgcn_sqrtf(v), inv_bc2_sqrt, args.eps);
                float rq = __builtin_amdgcn_rcpf(denom);
                rq = fmaf(rq, fmaf(-denom, rq, 1.0f), rq);   // one Newton step: ~0.5 ulp
                p = fmaf(-step_size, m * rq, p);
                f4set(m4, e, m);
                f4set(v4, e, v);
                f4set(pw, e, p);
              }
            } else {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
              const upd_f2 gr = upd_f2{f4get(g4, 2 * hh), f4get(g4, 2 * hh + 1)} * clipc;
              upd_f2 m = upd_f2{f4get(m4, 2 * hh), f4get(m4, 2 * hh + 1)};
              upd_f2 v = upd_f2{f4get(v4, 2 * hh), f4get(v4, 2 * hh + 1)};
              upd_f2 p = upd_f2{f4get(pw, 2 * hh), f4get(pw, 2 * hh + 1)};
              p = p * decay;
              m = upd_pkfma(upd_f2{omb1, omb1}, gr - m, m);
              v = upd_pkfma((upd_f2)(omb2 * gr), gr, v * b2);
              const upd_f2 sq{__builtin_amdgcn_sqrtf(v.x), __builtin_amdgcn_sqrtf(v.y)};
              const upd_f2 denom = upd_pkfma(sq, upd_f2{inv_bc2_sqrt, inv_bc2_sqrt}, upd_f2{args.eps, args.eps});
              upd_f2 rq{__builtin_amdgcn_rcpf(denom.x), __builtin_amdgcn_rcpf(denom.y)};
              rq = upd_pkfma(rq, upd_pkfma(-denom, rq, upd_f2{1.0f, 1.0f}), rq);   // one Newton step: ~0.5 ulp
              p = upd_pkfma(upd_f2{-step_size, -step_size}, m * rq, p);
              f4set(m4, 2 * hh, m.x);
              f4set(m4, 2 * hh + 1, m.y);
              f4set(v4, 2 * hh, v.x);
              f4set(v4, 2 * hh + 1, v.y);
              f4set(pw, 2 * hh, p.x);
              f4set(pw, 2 * hh + 1, p.y);
            }
            }
            if constexpr (TP) {
              if (q >= (int)((int64_t)Qtot * g / G) && q < (int)((int64_t)Qtot * (g + 1) / G)) {   // my slice
                st4_sc1(upd_rsrc(mdst), (size_t)q * 4, m4);
                st4_sc1(upd_rsrc(vdst), (size_t)q * 4, v4);
              }
            } else {
              mreg[i] = m4;
              vreg[i] = v4;
            }
            *reinterpret_cast<float4*>(W + 4 * q) = pw;
          }
        }
      }
    }
    __syncthreads();
    mark(6);   // AdamW
  }
  // ---- write back (workgroup 0): parameter / moment images, step count, last loss -----------
  if (g == 0) {
    for (int q = t; q < Qp; q += NT)
      *reinterpret_cast<float4*>(args.params + 4 * q) = *reinterpret_cast<const float4*>(W + 4 * q);
    if constexpr (!TP) {   // (TP: the slice owners stored them at the last step)
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int q = t + i * NT;
        if (q < Qp) {
          *reinterpret_cast<float4*>(args.exp_avg + 4 * q) = mreg[i];
          *reinterpret_cast<float4*>(args.exp_avg_sq + 4 * q) = vreg[i];
        }
      }
    }
    if (t == 0) {
      for (int i = 0; i < 7; ++i) args.prof[i] = pts[i];
      args.prof[7] = (unsigned long long)args.total_steps;
      args.prof[30] = __builtin_amdgcn_s_memrealtime() - pts[8];
      args.prof[31] = __builtin_amdgcn_s_memtime() - pts[9];
      for (int i = 0; i < 22; ++i) args.prof[8 + i] = reinterpret_cast<unsigned long long*>(hdr + 16)[i];
      args.adam_step[0] = step0 + (float)args.total_steps;
      if (args.loss_out) args.loss_out[0] = loss_last;
    }
  }
}

// KDIM > 0: the observation dim is a compile-time constant and the whole parameter layout folds
// into immediates (the specialised shapes); KDIM = 0: runtime layout from the kernel argument.
template <int NQ, int KD, int KA, int KDIM, bool DP = false, int TPM = 0>
__global__ __launch_bounds__((64 * upd_nw<KD, KA>()), 1) void ppo_update_kernel(UpdArgs args) {
  if constexpr (KDIM > 0) {
    constexpr UpdNet N = upd_make(KDIM, KA, upd_kd_discrete(KD) ? 1 : 0);
    ppo_update_body<NQ, KD, KA, DP, TPM>(N, args);
  } else {
    ppo_update_body<NQ, KD, KA, DP, TPM>(args.net, args);
  }
}

// ActorCritic.get_evaluate over N rows (PPO.learn's policy_old pass, PPO.py:127-154):
// log_prob, state value and (optionally) entropy per row, with exactly the update kernel's
// forward arithmetic, so the first minibatch of learn() sees ratio == 1 exactly, as in the
// reference.  Workgroups stride over 8-row chunks; parameters are staged once into LDS.
template <int KD, int KA>
__device__ __forceinline__ void ppo_evaluate_body(const UpdNet& n, const UpdArgs& args, float* logp_out,
                                                  float* V_out, float* H_out) {
  constexpr int NW = upd_nw<KD, KA>(), NT = 64 * NW;
  extern __shared__ __align__(16) float upd_lds[];
  const int t = threadIdx.x, l = t & 63, x = l & 15, q = l >> 4, w = t >> 6;
  float* scratch = upd_lds + UPD_HDR;
  float* W = scratch + ((upd_scratch_floats(n.D, NW, upd_ts(n)) + 3) & ~3);
  const UpdScr sc = upd_scr(scratch, n.D, NW);
  for (int k = t; k < n.Lp; k += NT) {
    const int f = upd_flat_of(n, k);
    W[k] = f >= 0 ? args.params[f] : 0.0f;
  }
  __syncthreads();
  const int64_t ntiles = (args.N + UPD_RT - 1) / UPD_RT;
  for (int64_t c = blockIdx.x; c < ntiles; c += gridDim.x) {
    const int64_t row0 = c * UPD_RT;
    const int rc = (int)std::min<int64_t>(UPD_RT, args.N - row0);
    UpdIn<upd_ksm<KA>()> in;
    upd_tile_load<KD, KA>(n, args.S, args.act, nullptr, nullptr, nullptr, row0, rc, in);
    UpdFwd<upd_ksm<KA>(), upd_hpw<KD, KA>()> f;
    upd_tile_fwd<KD, KA>(n, W, sc, in, f);
    __syncthreads();
    if (w == 0) {
      const float* Orow = upd_tile_outputs<NW>(n, W, sc);
      if (q == 0 && x < rc) {
        UpdDist d;
        upd_row_dist<KD, KA>(n, Orow, sc.Rin + x * UPD_RIN, d);
        logp_out[row0 + x] = d.logp;
        V_out[row0 + x] = Orow[n.discrete ? n.A : 2 * n.A];   // critic output column
        if (H_out) H_out[row0 + x] = d.H;
      }
    }
    __syncthreads();
  }
}

template <int KD, int KA, int KDIM>
__global__ __launch_bounds__((64 * upd_nw<KD, KA>()), 1) void ppo_evaluate_kernel(UpdArgs args, float* logp_out,
                                                                              float* V_out, float* H_out) {
  if constexpr (KDIM > 0) {
    constexpr UpdNet N = upd_make(KDIM, KA, upd_kd_discrete(KD) ? 1 : 0);
    ppo_evaluate_body<KD, KA>(N, args, logp_out, V_out, H_out);
  } else {
    ppo_evaluate_body<KD, KA>(args.net, args, logp_out, V_out, H_out);
  }
}

// The previous optimizer step's clip + AdamW folded into the next gradient launch (stepped mode):
// every workgroup applies it to ALL parameters of its LDS copy (identical inputs and code, so the
// copies agree), and workgroup g also writes quads [g Qp / G, (g+1) Qp / G) of the new parameter /
// moment images.  in != out (other workgroups are still reading `in`), grad_prev != this launch's
// grad_out: the caller double-buffers both.  grad_prev == nullptr: no prologue (first step).
struct UpdFold {
  const float* grad_prev;             // all-reduced gradient image (+ loss quad) of the previous step
  const float *p_in, *m_in, *v_in;    // state before that step's AdamW
  float *p_out, *m_out, *v_out;       // state after it
  double tstep;                       // that step's AdamW step number (1-based)
  float lr;
  double beta1, beta2;
  float eps, wd, max_norm, inv_count, vf_coef, ent_coef;
  float* loss_out;                    // that step's loss (workgroup 0), may be null
};

// NI > 0: Qp <= 256 NI known at compile time, every load issued before the norm (one round trip);
// NI == 0: runtime layout, norm loop then update loop.  Same summation order as ppo_adam_kernel.
template <int NI>
__device__ __forceinline__ void upd_fold_adam(const UpdFold& f, int Lp, float* W, float* s_part) {
  const int t = threadIdx.x, g = blockIdx.x, G = gridDim.x, Qp = Lp / 4;
  const int qlo = (int)((int64_t)g * Qp / G), qhi = (int)((int64_t)(g + 1) * Qp / G);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (NI > 0) {
    float4 gq[NI], mq[NI], vq[NI], pq[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = t + i * UPD_THREADS;
      const bool in = q < Qp;
      gq[i] = in ? *reinterpret_cast<const float4*>(f.grad_prev + 4 * q) : z4;
      mq[i] = in ? *reinterpret_cast<const float4*>(f.m_in + 4 * q) : z4;
      vq[i] = in ? *reinterpret_cast<const float4*>(f.v_in + 4 * q) : z4;
      pq[i] = in ? *reinterpret_cast<const float4*>(f.p_in + 4 * q) : z4;
    }
    const AdamConst c = adam_const(f.tstep, f.lr, f.beta1, f.beta2, f.eps, f.wd);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) acc += adam_sq4(gq[i]);
    const float clipc = adam_clip(acc, f.max_norm, s_part);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = t + i * UPD_THREADS;
      if (q < Qp) {
        adam_quad(c, clipc, gq[i], mq[i], vq[i], pq[i]);
        *reinterpret_cast<float4*>(W + 4 * q) = pq[i];
        if (q >= qlo && q < qhi) {
          *reinterpret_cast<float4*>(f.p_out + 4 * q) = pq[i];
          *reinterpret_cast<float4*>(f.m_out + 4 * q) = mq[i];
          *reinterpret_cast<float4*>(f.v_out + 4 * q) = vq[i];
        }
      }
    }
  } else {
    float acc = 0.f;
    for (int q = t; q < Qp; q += UPD_THREADS) acc += adam_sq4(*reinterpret_cast<const float4*>(f.grad_prev + 4 * q));
    const AdamConst c = adam_const(f.tstep, f.lr, f.beta1, f.beta2, f.eps, f.wd);
    const float clipc = adam_clip(acc, f.max_norm, s_part);
    for (int q = t; q < Qp; q += UPD_THREADS) {
      const float4 g4 = *reinterpret_cast<const float4*>(f.grad_prev + 4 * q);
      float4 m4 = *reinterpret_cast<const float4*>(f.m_in + 4 * q);
      float4 v4 = *reinterpret_cast<const float4*>(f.v_in + 4 * q);
      float4 pw = *reinterpret_cast<const float4*>(f.p_in + 4 * q);
      adam_quad(c, clipc, g4, m4, v4, pw);
      *reinterpret_cast<float4*>(W + 4 * q) = pw;
      if (q >= qlo && q < qhi) {
        *reinterpret_cast<float4*>(f.p_out + 4 * q) = pw;
        *reinterpret_cast<float4*>(f.m_out + 4 * q) = m4;
        *reinterpret_cast<float4*>(f.v_out + 4 * q) = v4;
      }
    }
  }
  if (g == 0 && t == 0 && f.loss_out)
    f.loss_out[0] = adam_loss(f.grad_prev, Lp, f.inv_count, f.vf_coef, f.ent_coef);
}

// ---- stepped mode (world_size > 1): one optimizer step = grad kernel -> RCCL all-reduce of the
// flat gradient (caller) -> AdamW kernel.  Parameters and moments live in HBM in the LDS-image
// layout between launches ("images"); prl_ppo_image converts to / from torch's flat vectors.

// Phase A + B of one step for this rank's rows [row0, row0 + B_local) of global minibatch j:
// partial gradients per workgroup, then the in-GPU reduction into grad_out[Lp + 4] (the last
// quad: loss partials {sum -min(s1,s2), sum SmoothL1, sum H}).  inv_count = 1 / (rows of the
// union minibatch over all ranks), so the all-reduced sum is the union's gradient.
template <int KD, int KA, int NI>
__device__ __forceinline__ void ppo_grad_body(const UpdNet& n, const UpdArgs& args, const float* img,
                                              float* grad_out, int64_t row0, int B_local,
                                              float inv_count, const UpdFold& fold) {
  constexpr int NW = upd_nw<KD, KA>(), NT = 64 * NW;
  extern __shared__ __align__(16) float upd_lds[];
  const int t = threadIdx.x, g = blockIdx.x, G = args.G;
  const int Lp = n.Lp, Qp = Lp / 4, Qtot = Qp + 1;
  float* hdr = upd_lds;
  float* scratch = upd_lds + UPD_HDR;
  float* W = scratch + ((upd_scratch_floats(n.D, NW, upd_ts(n)) + 3) & ~3);
  float* Ga = W + Lp;
  const UpdScr sc = upd_scr(scratch, n.D, NW);
  float* s_ssq = hdr + 4;
  int* s_abort = reinterpret_cast<int*>(hdr + 8);
  unsigned long long* tm = reinterpret_cast<unsigned long long*>(hdr + 16);
  static_assert(NT == UPD_THREADS, "the folded AdamW assumes 256-thread workgroups");
  if (fold.grad_prev) {                // previous step's AdamW, then this step's gradient
    upd_fold_adam<NI>(fold, Lp, W, scratch);
  } else {
    for (int q = t; q < Qp; q += NT)   // written by the previous launch: plain loads
      *reinterpret_cast<float4*>(W + 4 * q) = *reinterpret_cast<const float4*>(img + 4 * q);
  }
  for (int k = t; k < Lp + 4; k += NT) Ga[k] = 0.0f;
  if (t < 24) tm[t] = 0ull;
  __syncthreads();
  const int R = args.R;
  const int myrows = std::max(0, std::min(R, B_local - g * R));
  for (int c0 = 0; c0 < myrows; c0 += UPD_RT) {
    const int rc = std::min(UPD_RT, myrows - c0);
    UpdIn<upd_ksm<KA>()> in;
    upd_tile_load<KD, KA>(n, args.S, args.act, args.old_logp, args.adv, args.ret,
                          row0 + (int64_t)g * R + c0, rc, in);
    UpdGradOf<KD, KA> unused;   // (the LDS form: never touched)
    if (c0 == 0) upd_tile<KD, KA, true>(n, args, W, Ga, upd_scr_tile(sc, c0 / UPD_RT), in, rc, inv_count, tm, unused);
    else upd_tile<KD, KA, false>(n, args, W, Ga, upd_scr_tile(sc, c0 / UPD_RT), in, rc, inv_count, tm, unused);
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs_part = upd_rsrc(args.part), rs_red = upd_rsrc(grad_out);
  for (int q = t; q < Qtot; q += NT)
    st4_sc1(rs_part, ((size_t)g * Qtot + q) * 4, *reinterpret_cast<const float4*>(Ga + 4 * q));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __hip_atomic_fetch_add(upd_g(args.ctr + 0), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_abort = upd_wait(args.ctr, 0, args.grad_target) ? 0 : 1;
  }
  __syncthreads();
  if (*s_abort) return;
  upd_slice_reduce(rs_part, rs_red, Qtot, Qp, g, G, scratch, NT);
  (void)s_ssq;
}

template <int KD, int KA, int KDIM>
__global__ __launch_bounds__((64 * upd_nw<KD, KA>()), 1) void ppo_grad_kernel(UpdArgs args, const float* img,
                                                                float* grad_out, int64_t row0,
                                                                int B_local, float inv_count,
                                                                UpdFold fold) {
  if constexpr (KDIM > 0) {
    constexpr UpdNet N = upd_make(KDIM, KA, upd_kd_discrete(KD) ? 1 : 0);
    constexpr int NI = (N.Lp / 4 + UPD_THREADS - 1) / UPD_THREADS;
    ppo_grad_body<KD, KA, NI>(N, args, img, grad_out, row0, B_local, inv_count, fold);
  } else {
    ppo_grad_body<KD, KA, 0>(args.net, args, img, grad_out, row0, B_local, inv_count, fold);
  }
}

// clip_grad_norm_(max_norm) + AdamW on the images, one parameter quad per thread.  Every
// workgroup forms the same norm (same order), so no hand-off is needed.  Latency-bound (a few
// KB per workgroup): every load — the whole gradient for the norm AND this thread's own
// gradient / moment / parameter quads — is issued at entry, so the kernel pays ONE memory
// round trip; the bias corrections are formed while those loads are in flight.
constexpr int ADAM_PF = 24;   // gradient quads per thread held in registers (Qp <= 6144)
__global__ __launch_bounds__(UPD_THREADS) void ppo_adam_kernel(int Lp, float* img_p, float* img_m,
                                                             float* img_v, const float* grad,
                                                             double tstep, float lr, double beta1,
                                                             double beta2, float eps, float wd,
                                                             float max_norm, float inv_count,
                                                             float vf_coef, float ent_coef,
                                                             float* loss_out) {
  __shared__ float s_part[UPD_THREADS / 64];
  const int t = threadIdx.x, Qp = Lp / 4;
  const int q = blockIdx.x * UPD_THREADS + t;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 g4 = z4, m4 = z4, v4 = z4, pw = z4;
  if (q < Qp) {
    g4 = *reinterpret_cast<const float4*>(grad + 4 * q);
    m4 = *reinterpret_cast<const float4*>(img_m + 4 * q);
    v4 = *reinterpret_cast<const float4*>(img_v + 4 * q);
    pw = *reinterpret_cast<const float4*>(img_p + 4 * q);
  }
  float4 pre[ADAM_PF];
#pragma unroll
  for (int i = 0; i < ADAM_PF; ++i) {
    const int qq = t + i * UPD_THREADS;
    pre[i] = qq < Qp ? *reinterpret_cast<const float4*>(grad + 4 * qq) : z4;
  }
  const AdamConst c = adam_const(tstep, lr, beta1, beta2, eps, wd);
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < ADAM_PF; ++i) acc += adam_sq4(pre[i]);
  for (int qq = t + ADAM_PF * UPD_THREADS; qq < Qp; qq += UPD_THREADS)  // beyond the registers
    acc += adam_sq4(*reinterpret_cast<const float4*>(grad + 4 * qq));
  const float clipc = adam_clip(acc, max_norm, s_part);
  if (q < Qp) {
    adam_quad(c, clipc, g4, m4, v4, pw);
    *reinterpret_cast<float4*>(img_m + 4 * q) = m4;
    *reinterpret_cast<float4*>(img_v + 4 * q) = v4;
    *reinterpret_cast<float4*>(img_p + 4 * q) = pw;
  }
  if (blockIdx.x == 0 && t == 0 && loss_out) loss_out[0] = adam_loss(grad, Lp, inv_count, vf_coef, ent_coef);
}

#include "prl_ppo_split.h"

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

// waves per workgroup of the kernels chosen for this shape (upd_nw<KD, KA>() on the device)
bool upd_force_generic();
// PRL_UPD_WAVES=4 keeps the persistent CartPole engine at 4 waves (A/B, diagnostics)
bool upd_waves8_enabled() {
  static const int v = [] {
    const char* e = getenv("PRL_UPD_WAVES");
    return (e && e[0] == '4') ? 0 : 1;
  }();
  return v != 0;
}
bool upd_is_cartpole(const UpdNet& n) { return n.discrete && n.A == 2 && n.D == 4; }
// waves of the kernel that runs this shape: the persistent kernels (update, data-parallel
// update) or the others (evaluate, stepped gradient, AdamW)
int upd_nw_host(const UpdNet& n, bool persistent) {
  return (persistent && upd_is_cartpole(n) && !upd_force_generic() && upd_waves8_enabled()) ? 8 : 4;
}
int upd_nt(const UpdNet& n, bool persistent = false) { return 64 * upd_nw_host(n, persistent); }
int upd_nq(const UpdNet& n) { return (int)cdiv(n.Lp / 4, upd_nt(n, true)); }
// Specialisations for the configs' shapes (CartPole: discrete, A = 2; Pendulum: continuous,
// A = 1); every other shape runs the generic (runtime head configuration) kernel.
// PRL_UPD_PROFILE=1: the engine records workgroup 0's per-phase times (FusedUpdate.profile)
int upd_profile_enabled() {
  const char* e = getenv("PRL_UPD_PROFILE");
  return e && e[0] == '1' ? 1 : (e && e[0] == '2' ? 2 : 0);
}
// PRL_UPD_GENERIC=1 routes every shape through the runtime-layout kernels (testing)
bool upd_force_generic() {
  const char* e = getenv("PRL_UPD_GENERIC");
  return e && e[0] == '1';
}
// PRL_UPD_TP / prl_ppo_update_set_tp: 0 never, 1 whenever allowed, 2 (default) auto (>= 2
// tiles per workgroup and step)
int g_tp_mode = [] {
  const char* e = getenv("PRL_UPD_TP");
  return (e && e[0] == '0') ? 0 : ((e && e[0] == '1') ? 1 : 2);
}();
int upd_tp_mode() { return g_tp_mode; }
// the throughput form (ppo_update_body<.., TP>) for this launch: rows per workgroup and step R,
// total steps (the streamed moments need >= 2), single-GPU only
bool upd_tp_host(int R, int total_steps, bool dp) {
  const int m = upd_tp_mode();
  if (dp || total_steps < 2 || m == 0) return false;
  return m == 1 || R >= 2 * UPD_RT;
}
const void* upd_kernel_for(const UpdNet& n, bool dp = false) {
  if (dp) {
    const int nq = upd_nq(n);
    if (upd_force_generic()) return nq <= 20 ? reinterpret_cast<const void*>(ppo_update_kernel<20, -1, 0, 0, true>) : nullptr;
    if (upd_is_cartpole(n) && nq <= 5) return reinterpret_cast<const void*>(ppo_update_kernel<5, 2, 2, 4, true>);
    if (upd_is_cartpole(n) && nq <= 10) return reinterpret_cast<const void*>(ppo_update_kernel<10, 1, 2, 4, true>);
    if (!n.discrete && n.A == 1 && n.D == 3 && nq <= 14) return reinterpret_cast<const void*>(ppo_update_kernel<14, 0, 1, 3, true>);
    if (nq <= 20) return reinterpret_cast<const void*>(ppo_update_kernel<20, -1, 0, 0, true>);
    return nullptr;
  }
  const int nq = upd_nq(n);
  if (upd_force_generic()) return nq <= 20 ? reinterpret_cast<const void*>(ppo_update_kernel<20, -1, 0, 0>) : nullptr;
  if (upd_is_cartpole(n) && nq <= 5) return reinterpret_cast<const void*>(ppo_update_kernel<5, 2, 2, 4>);
  if (upd_is_cartpole(n) && nq <= 10) return reinterpret_cast<const void*>(ppo_update_kernel<10, 1, 2, 4>);
  if (!n.discrete && n.A == 1 && n.D == 3 && nq <= 14) return reinterpret_cast<const void*>(ppo_update_kernel<14, 0, 1, 3>);
  if (nq <= 20) return reinterpret_cast<const void*>(ppo_update_kernel<20, -1, 0, 0>);
  return nullptr;
}
// The throughput form's kernel for this shape: the 8-wave head-split kernels for CartPole and
// Pendulum (PRL_UPD_WAVES=4: the 4-wave ones); none for other shapes (null: the latency form).
struct UpdPlan {
  const void* kern;
  int nw, tiles;
};
UpdPlan upd_tp_plan(const UpdNet& n) {
  const int qp = n.Lp / 4;
  if (!upd_force_generic()) {
    if (upd_is_cartpole(n) && upd_waves8_enabled() && cdiv(qp, 512) <= 5)
      return {reinterpret_cast<const void*>(ppo_update_kernel<5, 2, 2, 4, false, 1>), 8, 1};
    if (upd_is_cartpole(n) && cdiv(qp, 256) <= 10)
      return {reinterpret_cast<const void*>(ppo_update_kernel<10, 1, 2, 4, false, 1>), 4, 1};
    const bool pend = !n.discrete && n.A == 1 && n.D == 3;
    if (pend && upd_waves8_enabled() && cdiv(qp, 512) <= 7)
      return {reinterpret_cast<const void*>(ppo_update_kernel<7, 3, 1, 3, false, 1>), 8, 1};
    if (pend && cdiv(qp, 256) <= 14)
      return {reinterpret_cast<const void*>(ppo_update_kernel<14, 0, 1, 3, false, 1>), 4, 1};
  }
  return {nullptr, 4, 1};   // (the runtime-layout kernel spills more in this form: latency form)
}
size_t upd_lds_bytes_plan(const UpdNet& n, int nw, bool tp, int tiles) {
  return sizeof(float) * (size_t)(UPD_HDR + (tp ? n.Lp : 2 * n.Lp + 4) +
                                  tiles * ((upd_scratch_floats(n.D, nw, upd_ts(n)) + 3) & ~3));
}
const void* upd_grad_kernel_for(const UpdNet& n) {
  if (upd_force_generic()) return reinterpret_cast<const void*>(ppo_grad_kernel<-1, 0, 0>);
  if (n.discrete && n.A == 2 && n.D == 4) return reinterpret_cast<const void*>(ppo_grad_kernel<1, 2, 4>);
  if (!n.discrete && n.A == 1 && n.D == 3) return reinterpret_cast<const void*>(ppo_grad_kernel<0, 1, 3>);
  return reinterpret_cast<const void*>(ppo_grad_kernel<-1, 0, 0>);
}
const void* upd_eval_kernel_for(const UpdNet& n) {
  if (upd_force_generic()) return reinterpret_cast<const void*>(ppo_evaluate_kernel<-1, 0, 0>);
  if (n.discrete && n.A == 2 && n.D == 4) return reinterpret_cast<const void*>(ppo_evaluate_kernel<1, 2, 4>);
  if (!n.discrete && n.A == 1 && n.D == 3) return reinterpret_cast<const void*>(ppo_evaluate_kernel<0, 1, 3>);
  return reinterpret_cast<const void*>(ppo_evaluate_kernel<-1, 0, 0>);
}

int upd_grid(int64_t mb) { return (int)std::min<int64_t>(256, cdiv(mb, UPD_RT)); }
// Replicas per tile group of the latency form (ppo_update_body: workgroups g, g + Gt, ... run the
// same rows and split the publish): PRL_UPD_REPL (default 2: mb 512 13.84 vs 14.03 us per step,
// same-box A/B; 4 and 8 slower, their waits grow), capped so that all Gt x X
// workgroups fit one per CU.
int g_repl = [] {
  const char* e = getenv("PRL_UPD_REPL");
  const int v = e ? atoi(e) : 2;
  return v >= 1 ? v : 1;
}();
// The head-split latency form (prl_ppo_split.h) for the two-head discrete nets of the CartPole
// shape: PRL_UPD_SPLIT / prl_ppo_update_set_split (1 = on, the default; 0 = the 8-wave kernel).
int g_split = [] {
  const char* e = getenv("PRL_UPD_SPLIT");
  return (e && e[0] == '0') ? 0 : 1;
}();
// Quads per thread of the split kernel's phase-C sweep that are instantiated (4 / 8 waves)
constexpr int SPL_NQC = 10, SPL_NQC8 = 5;
// PRL_UPD_SPL_WAVES=8: the split kernel's 8-wave form (waves 4-7 in the exchange phases only)
int upd_split_waves() {
  const char* e = getenv("PRL_UPD_SPL_WAVES");
  return (e && e[0] == '8') ? 8 : 4;
}
// The split form's slice-owner variant (prl_ppo_split.h, OWN): one rank, PRL_UPD_SPL_OWN=1
// (opt-in: it wins only where clip_grad_norm_ rarely scales a step — 11.84 vs 12.58 us per step
// on the fixed synthetic 2^20 memory — while C2's training clips every step, where each clipped
// step's redo + extra hand-off makes it 14.1 vs 12.8 us; tools/clip_stats.py), and every slice
// narrow (2 nq <= NT: one owned quad per thread; mb >= 256 at the CartPole shape), with the
// slices cut as spl_slice_start cuts them.
int g_last_own = 0;
bool upd_split_own(const UpdNet& n, int G, int NT) {
  const char* e = getenv("PRL_UPD_SPL_OWN");
  if (!(e && e[0] == '1')) return false;
  const int Qp = n.Lp / 4, QT = n.w1[0].lds / 4;
  for (int g = 0; g < G; ++g)   // (the default trunk weight: the owner form ignores PRL_UPD_SPL_TW4)
    if (2 * (spl_slice_start(g + 1, G, Qp, QT) - spl_slice_start(g, G, Qp, QT)) > NT) return false;
  return true;
}
// Phase-B helper workgroups of the single-GPU split form (spl_helper): PRL_UPD_SPL_HELP = their
// number, at most the CUs the G tile workgroups leave free (capped at 256 owners).  Default 0:
// measured slower (mb 512, same box: 12.74 us per step without helpers, 13.77 with 64, 14.88
// with 192) — their polls of counter A during the tiles and of B during the slice loads slow
// both hand-offs (wait A 1.40 -> 2.31 us, slice reduce 2.08 -> 2.71) more than the smaller
// slices save.
int upd_split_helpers(int G) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const int room = std::max(0, std::min(cus, 256) - G);
  const char* e = getenv("PRL_UPD_SPL_HELP");
  return e ? std::min(room, std::max(0, atoi(e))) : 0;
}
bool upd_split_host(const UpdNet& n, int Gt, int R, bool tp) {
  if (tp || !g_split || upd_force_generic() || !upd_is_cartpole(n) || R != UPD_RT) return false;
  if (cdiv(n.Lp / 4, 64 * upd_split_waves()) > (upd_split_waves() == 8 ? SPL_NQC8 : SPL_NQC)) return false;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  return 2 * Gt <= cus;
}
int upd_repl(int Gt) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 1;
  int x = g_repl;
  while (x > 1 && Gt * x > cus) --x;
  return x;
}

// The persistent kernels need all G workgroups resident at once (they hand data to each other).
// A plain launch gives the same residency as a cooperative one (MI355X_MICROARCH.md,
// coop-launch); what the cooperative API adds is this check, ~15-19 us of host time per launch,
// and, under rocprofv3's kernel tracing, a SIGSEGV inside exit() at process teardown (round 1's
// profiled bench; tools/teardown_probe.sh isolates it to the cooperative launch).  So: check the
// occupancy ourselves, then launch plainly.
hipError_t upd_launch_resident(const void* kern, int G, int threads, size_t lds, void** kargs,
                               hipStream_t st) {
  int per_cu = 0, dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds);
  if (e != hipSuccess) return e;
  if ((int64_t)per_cu * cus < G) return hipErrorCooperativeLaunchTooLarge;
  return hipLaunchKernel(kern, dim3(G), dim3(threads), kargs, lds, st);
}

size_t upd_lds_bytes(const UpdNet& n, bool persistent, bool tp = false) {
  return sizeof(float) * (size_t)(UPD_HDR + (tp ? n.Lp : 2 * n.Lp + 4) +
                                  ((upd_scratch_floats(n.D, upd_nw_host(n, persistent), upd_ts(n)) + 3) & ~3));
}

struct UpdWs {
  unsigned* ctr;
  unsigned long long* prof;
  float* sq;
  float* red;
  float* part;
  float* img;   // [3][Lp + 4]: parameter, exp_avg, exp_avg_sq images of the persistent launch
  float* mv;    // [4][Lp + 4]: the throughput form's moment buffers m0, v0, m1, v1
  float* part2; // [Gt][QT + 1][4]: the head-split form's role-1 trunk (+ loss) partials
};

// workspace: ctr[UPD_CTR_WORDS] (words 0-3 and the shards zeroed per launch, word 4 sticky) |
// prof[32] + arrival stamps[2][256] | sq[NW G] | red[2][Qtot*4] | part[G][Qtot*4] | img[3][Qtot*4] |
// mv[4][Qtot*4] | part2[G][(QT+1)*4] | slack
// (phase C's sweeps read up to one thread block of quads past an image: the slack keeps the
// last one inside the allocation)
size_t upd_ws_carve(const UpdNet& n, int G, char* base, UpdWs* ws) {
  const size_t Qtot = (size_t)n.Lp / 4 + 1;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
  const size_t o_ctr = take(4 * UPD_CTR_WORDS), o_prof = take(256 + 2 * 256 * 8), o_sq = take(2048 * 4), o_red = take(2 * Qtot * 16),
               o_part = take((size_t)G * Qtot * 16), o_img = take((size_t)3 * Qtot * 16),
               o_mv = take((size_t)4 * Qtot * 16),
               o_part2 = take((size_t)G * ((size_t)n.w1[0].lds / 4 + 1) * 16);
  (void)take(512 * 16);
  if (ws) {
    ws->ctr = reinterpret_cast<unsigned*>(base + o_ctr);
    ws->prof = reinterpret_cast<unsigned long long*>(base + o_prof);
    ws->sq = reinterpret_cast<float*>(base + o_sq);
    ws->red = reinterpret_cast<float*>(base + o_red);
    ws->part = reinterpret_cast<float*>(base + o_part);
    ws->img = reinterpret_cast<float*>(base + o_img);
    ws->mv = reinterpret_cast<float*>(base + o_mv);
    ws->part2 = reinterpret_cast<float*>(base + o_part2);
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
  return (upd_lds_bytes(n, true) <= 160 * 1024 && upd_kernel_for(n)) ? PRL_OK : PRL_ERR_ARG;
}

namespace {
// the data-parallel part of a persistent launch (prl_ppo_update_dpx)
struct UpdDp {
  int world, rank, nb;
  const float* inv_count;
  void* const* xbufs;
  int64_t seq0;
  int fine;
};
// the slice buffers [2][Qtot * 4] f32, then the per-workgroup step flags [2 G] u64 (pull form);
// then the push form's receive slices [2][UPD_MAX_RANKS][Qtot * 4] f32 and receive flags
// [UPD_MAX_RANKS][2 G] u64 (G = upd_grid(mini_batch); two workgroups per tile group at most)
size_t upd_xbuf_flags_off(const UpdNet& n) { return (((size_t)n.Lp / 4 + 1) * 32 + 255) & ~(size_t)255; }
size_t upd_xbuf_push_off(const UpdNet& n, int mb) {
  return (upd_xbuf_flags_off(n) + 2 * (size_t)upd_grid(mb) * 8 + 255) & ~(size_t)255;
}
size_t upd_xbuf_push_flags_off(const UpdNet& n, int mb) {
  return upd_xbuf_push_off(n, mb) + (size_t)2 * UPD_MAX_RANKS * ((size_t)n.Lp / 4 + 1) * 16;
}
size_t upd_xbuf_bytes(const UpdNet& n, int mb) {
  return upd_xbuf_push_flags_off(n, mb) + (size_t)UPD_MAX_RANKS * 2 * upd_grid(mb) * 8;
}
unsigned g_dp_spin_limit = UPD_DP_SPIN_LIMIT;
int32_t g_last_plan[8] = {-1, -1, -1, -1, -1, -1, -1, -1};   // prl_ppo_update_last_plan

int upd_run(float* params, float* exp_avg, float* exp_avg_sq, float* adam_step, int32_t D,
            int32_t A, int32_t discrete, const float* S, const float* actions,
            const float* old_logp, const float* adv, const float* ret, int64_t N,
            int32_t mini_batch, int32_t k_epochs, float clip, float vf_coef, float ent_coef,
            float lr, double beta1, double beta2, float eps, float weight_decay, float max_norm,
            float* loss_out, void* workspace, int64_t workspace_bytes, void* stream,
            const UpdDp* dp) {
  UpdArgs args{};
  PRL_REQUIRE(upd_layout(D, A, discrete, args.net), "prl_ppo_update: D=%d A=%d not supported", D, A);
  PRL_REQUIRE(N > 0 && mini_batch > 0 && k_epochs >= 0, "prl_ppo_update: bad sizes");
  PRL_REQUIRE(params && exp_avg && exp_avg_sq && adam_step && S && actions && old_logp && adv && ret &&
                  workspace, "prl_ppo_update: null pointer");
  const int Gt = upd_grid(mini_batch);   // tile groups (one partial each)
  UpdWs ws;
  const size_t need = upd_ws_carve(args.net, Gt, reinterpret_cast<char*>(workspace), &ws);
  PRL_REQUIRE((size_t)workspace_bytes >= need, "prl_ppo_update: workspace %lld < %zu bytes",
              (long long)workspace_bytes, need);
  const int64_t nb = dp ? (int64_t)dp->nb : cdiv(N, (int64_t)mini_batch);
  PRL_REQUIRE(nb >= cdiv(N, (int64_t)mini_batch), "prl_ppo_update_dpx: nb < this rank's minibatches");
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
  args.Gt = Gt;
  args.R = (int)cdiv(cdiv((int64_t)mini_batch, (int64_t)Gt), (int64_t)UPD_RT) * UPD_RT;
  args.clip = clip;
  args.vf_coef = vf_coef;
  args.ent_coef = ent_coef;
  args.lr = lr;
  args.beta1 = beta1;
  args.beta2 = beta2;
  args.eps = eps;
  args.wd = weight_decay;
  args.max_norm = max_norm;
  const size_t L4 = (size_t)args.net.Lp + 4;
  float* img_p = ws.img;
  float* img_m = ws.img + L4;
  float* img_v = ws.img + 2 * L4;
  args.params = img_p;
  args.exp_avg = img_m;
  args.exp_avg_sq = img_v;
  args.adam_step = adam_step;
  args.loss_out = loss_out;
  args.part = ws.part;
  args.red = ws.red;
  args.sq = ws.sq;
  args.ctr = ws.ctr;
  args.prof = ws.prof;
  args.profile = upd_profile_enabled();
  args.world = 1;
  if (dp) {
    PRL_REQUIRE(dp->world >= 1 && dp->world <= UPD_MAX_RANKS && dp->rank >= 0 && dp->rank < dp->world,
                "prl_ppo_update_dpx: world %d / rank %d (at most %d ranks)", dp->world, dp->rank,
                UPD_MAX_RANKS);
    PRL_REQUIRE(dp->inv_count && dp->xbufs, "prl_ppo_update_dpx: null pointer");
    args.world = dp->world;
    args.rank = dp->rank;
    args.inv_count = dp->inv_count;
    args.dp_seq0 = (unsigned long long)dp->seq0;
    args.dp_spin_limit = g_dp_spin_limit;
    args.dp_fine = (dp->fine & 1) ? 1 : 0;
    args.dp_push = (dp->fine & 2) ? 1 : 0;
    args.xpush_off = upd_xbuf_push_off(args.net, mini_batch) / 4;
    args.xpush_flags_off = upd_xbuf_push_flags_off(args.net, mini_batch) / 8;
    args.xpush_gmax = 2 * upd_grid(mini_batch);
    const size_t fo = upd_xbuf_flags_off(args.net);
    for (int r = 0; r < dp->world; ++r) {
      PRL_REQUIRE(dp->xbufs[r], "prl_ppo_update_dpx: null slice buffer of rank %d", r);
      args.xbuf[r] = reinterpret_cast<float*>(dp->xbufs[r]);
      args.xflag[r] = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(dp->xbufs[r]) + fo);
    }
    args.xbuf_self = args.xbuf[dp->rank];
    args.xflag_self = args.xflag[dp->rank];
  }
  args.part2 = ws.part2;
  {
    const char* e = getenv("PRL_UPD_SPL_FILL");   // default 1 (mb 512: 13.58 vs 14.07 us per step)
    args.spl_fill = (e && e[0] == '0') ? 0 : 1;
    const char* d = getenv("PRL_UPD_SPL_DIRECT");
    args.spl_direct = (d && d[0] == '1') ? 1 : 0;
    const char* pp = getenv("PRL_UPD_SPL_POLL");
    args.spl_poll = pp ? std::max(0, std::min(4, atoi(pp))) : 0;
    const char* pk = getenv("PRL_UPD_SPL_PK");
    args.spl_pk = (pk && pk[0] == '1') ? 1 : 0;
    const char* tw = getenv("PRL_UPD_SPL_TW4");
    args.spl_tw4 = tw ? std::max(4, std::min(16, atoi(tw))) : 8;
    const char* pc = getenv("PRL_UPD_SPL_PIECES");
    args.spl_pieces = (pc && pc[0] == '0') ? 0 : 1;
  }
  args.tp_m0 = ws.mv;
  args.tp_v0 = ws.mv + L4;
  args.tp_m1 = ws.mv + 2 * L4;
  args.tp_v1 = ws.mv + 3 * L4;
  bool tp = upd_tp_host(args.R, args.total_steps, dp != nullptr);
  UpdPlan plan{upd_kernel_for(args.net, dp != nullptr), upd_nw_host(args.net, true), 1};
  if (tp) {
    const UpdPlan p2 = upd_tp_plan(args.net);
    if (p2.kern) plan = p2;
    else tp = false;
  }
  // data-parallel ranks: fine_grained bit 2 = the ranks voted for the 8-wave kernel
  // (prl_ppo_update_dp_split: the kernel form must not come from per-process state alone)
  const bool split = upd_split_host(args.net, Gt, args.R, tp) && !(dp && (dp->fine & 4));
  if (!split) args.dp_push = 0;   // the push form is the head-split kernel's (ranks decide alike)
  g_last_own = 0;
  if (split) {
    const int tw = upd_split_waves();
    const bool own = !dp && tw == 4 && upd_split_own(args.net, 2 * Gt, 64 * tw);
    const void* k = tw == 8 ? (dp ? reinterpret_cast<const void*>(ppo_update_split_kernel<SPL_NQC8, 2, 4, true, 8>)
                                  : reinterpret_cast<const void*>(ppo_update_split_kernel<SPL_NQC8, 2, 4, false, 8>))
                            : (dp ? reinterpret_cast<const void*>(ppo_update_split_kernel<SPL_NQC, 2, 4, true, 4>)
                                  : own ? reinterpret_cast<const void*>(ppo_update_split_kernel<SPL_NQC, 2, 4, false, 4, true>)
                                        : reinterpret_cast<const void*>(ppo_update_split_kernel<SPL_NQC, 2, 4, false, 4>));
    g_last_own = own ? 1 : 0;
    if (own) args.spl_tw4 = 8;   // upd_split_own checked the default slicing
    // the 4-wave workgroup-AdamW form updates by wave-block lists (prl_ppo_split.h, WB): its clip
    // norm always comes from the pieces (PRL_UPD_SPL_PIECES=0 applies to the other forms only)
    if (tw == 4 && !own) {
      args.spl_pieces = 1;
      PRL_REQUIRE(spl_wb_check(args.net), "prl_ppo_update: the wave-block AdamW lists do not cover the net");
    }
    plan = UpdPlan{k, tw, 1};
  }
  // replicated tiles: the latency form on one GPU only; the split form: two roles per tile group
  const int G = split ? 2 * Gt : ((tp || dp) ? Gt : Gt * upd_repl(Gt));
  args.G = G;
  // phase-B helpers of the single-GPU split form (prl_ppo_split.h, spl_helper)
  args.Gs = (split && !dp && !g_last_own) ? G + upd_split_helpers(G) : G;
  const size_t lds = upd_lds_bytes_plan(args.net, plan.nw, tp, plan.tiles);
  PRL_REQUIRE(lds <= 160 * 1024, "prl_ppo_update: %zu B of LDS needed", lds);
  hipStream_t st = as_stream(stream);
  const void* kern = plan.kern;
  PRL_REQUIRE(kern, "prl_ppo_update: %d parameter quads per thread not built", upd_nq(args.net));
  g_last_plan[0] = tp ? 1 : 0;
  g_last_plan[1] = plan.nw;
  g_last_plan[2] = G;
  g_last_plan[3] = args.R / UPD_RT;
  g_last_plan[4] = (!upd_force_generic() && (upd_is_cartpole(args.net) ||
                                             (!args.net.discrete && args.net.A == 1 && args.net.D == 3))) ? 1 : 0;
  g_last_plan[5] = G / Gt;
  g_last_plan[6] = split ? (g_last_own ? 2 : 1) : 0;
  g_last_plan[7] = args.Gs - G;
  PRL_HIP_TRY(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  PRL_HIP_TRY(hipMemsetAsync(ws.ctr, 0, 16, st));
  PRL_HIP_TRY(hipMemsetAsync(ws.ctr + UPD_CTR_A, 0, 4 * (UPD_CTR_WORDS - UPD_CTR_A), st));
  void* kargs[] = {&args};
  const unsigned img_grid = (unsigned)cdiv(args.net.Lp, UPD_THREADS);
  hipLaunchKernelGGL(ppo_image_kernel, dim3(img_grid), dim3(UPD_THREADS), 0, st, args.net, params,
                     exp_avg, exp_avg_sq, img_p, img_m, img_v, 1);
  PRL_LAUNCH_CHECK("ppo_image");
  PRL_HIP_TRY(upd_launch_resident(kern, args.Gs, 64 * plan.nw, lds, kargs, st));
  hipLaunchKernelGGL(ppo_image_kernel, dim3(img_grid), dim3(UPD_THREADS), 0, st, args.net, params,
                     exp_avg, exp_avg_sq, img_p, img_m, img_v, 0);
  PRL_LAUNCH_CHECK("ppo_image");
  return PRL_OK;
}
}  // namespace

extern "C" int prl_ppo_update(float* params, float* exp_avg, float* exp_avg_sq, float* adam_step,
                              int32_t D, int32_t A, int32_t discrete, const float* S,
                              const float* actions, const float* old_logp, const float* adv,
                              const float* ret, int64_t N, int32_t mini_batch, int32_t k_epochs,
                              float clip, float vf_coef, float ent_coef, float lr, double beta1,
                              double beta2, float eps, float weight_decay, float max_norm,
                              float* loss_out, void* workspace, int64_t workspace_bytes,
                              void* stream) {
  return upd_run(params, exp_avg, exp_avg_sq, adam_step, D, A, discrete, S, actions, old_logp,
                 adv, ret, N, mini_batch, k_epochs, clip, vf_coef, ent_coef, lr, beta1, beta2, eps,
                 weight_decay, max_norm, loss_out, workspace, workspace_bytes, stream, nullptr);
}

extern "C" int prl_ppo_update_dpx(float* params, float* exp_avg, float* exp_avg_sq,
                                  float* adam_step, int32_t D, int32_t A, int32_t discrete,
                                  const float* S, const float* actions, const float* old_logp,
                                  const float* adv, const float* ret, int64_t N,
                                  int32_t mini_batch, int32_t k_epochs, int32_t nb_union,
                                  const float* inv_count, float clip, float vf_coef,
                                  float ent_coef, float lr, double beta1, double beta2, float eps,
                                  float weight_decay, float max_norm, float* loss_out,
                                  int32_t world, int32_t rank, void* const* xbufs, int64_t seq0,
                                  int32_t fine_grained, void* workspace, int64_t workspace_bytes,
                                  void* stream) {
  PRL_REQUIRE(nb_union > 0 && seq0 >= 0, "prl_ppo_update_dpx: nb_union <= 0 or seq0 < 0");
  const UpdDp dp{world, rank, nb_union, inv_count, xbufs, seq0, fine_grained};
  return upd_run(params, exp_avg, exp_avg_sq, adam_step, D, A, discrete, S, actions, old_logp,
                 adv, ret, N, mini_batch, k_epochs, clip, vf_coef, ent_coef, lr, beta1, beta2, eps,
                 weight_decay, max_norm, loss_out, workspace, workspace_bytes, stream, &dp);
}

extern "C" int32_t prl_ppo_update_set_tp(int32_t mode) {
  const int prev = g_tp_mode;
  g_tp_mode = (mode >= 0 && mode <= 2) ? mode : 2;
  return prev;
}

extern "C" int32_t prl_ppo_update_set_repl(int32_t replicas) {
  const int prev = g_repl;
  g_repl = replicas >= 1 ? replicas : 1;
  return prev;
}

extern "C" int32_t prl_ppo_update_set_split(int32_t mode) {
  const int prev = g_split;
  g_split = mode ? 1 : 0;
  return prev;
}

extern "C" int32_t prl_ppo_update_dp_split(int32_t D, int32_t A, int32_t discrete, int32_t mini_batch) {
  UpdNet n;
  if (mini_batch <= 0 || !upd_layout(D, A, discrete, n)) return 0;
  const int Gt = upd_grid(mini_batch);   // as upd_run: tile groups, rows per workgroup and step
  const int R = (int)cdiv(cdiv((int64_t)mini_batch, (int64_t)Gt), (int64_t)UPD_RT) * UPD_RT;
  return upd_split_host(n, Gt, R, false) ? 1 : 0;   // (data-parallel launches never take tp)
}

extern "C" int32_t prl_ppo_update_wb_check(int32_t D, int32_t A, int32_t discrete) {
  UpdNet n;
  if (!upd_layout(D, A, discrete, n)) return 0;
  return spl_wb_check(n) ? 1 : 0;
}

extern "C" void prl_ppo_update_last_plan(int32_t out[8]) {
  for (int i = 0; i < 8; ++i) out[i] = g_last_plan[i];
}

extern "C" uint32_t prl_dp_set_spin_limit(uint32_t polls) {
  const uint32_t prev = g_dp_spin_limit;
  g_dp_spin_limit = polls ? polls : UPD_DP_SPIN_LIMIT;
  return prev;
}

extern "C" int64_t prl_dp_xbuf_bytes(int32_t D, int32_t A, int32_t discrete, int32_t mini_batch) {
  UpdNet net{};
  if (!upd_layout(D, A, discrete, net) || mini_batch <= 0) return -1;
  // pull flags for two workgroups per tile group (the head-split form) and the push form's region
  return (int64_t)upd_xbuf_bytes(net, mini_batch);
}

extern "C" int prl_dp_xbuf_alloc(int64_t bytes, int32_t* kind, void** out) {
  PRL_REQUIRE(bytes > 0 && out && kind && *kind >= 0 && *kind <= 2, "prl_dp_xbuf_alloc: bad arguments");
  // Its own allocation (shareable by IPC handle), UNCACHED: other GPUs read it over xGMI while
  // this GPU writes it, and coarse-grained memory is not coherent across devices inside a
  // kernel (RCCL keeps its cross-GPU flags and FIFOs in uncached / fine-grained memory too).
  // Fine-grained memory is the fallback (the kernel then fences the flags: dp_fine).
  void* p = nullptr;
  const int want = *kind;
  if (want != 2 && hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached) == hipSuccess) {
    *kind = 1;
  } else {
    (void)hipGetLastError();
    p = nullptr;
    PRL_REQUIRE(want != 1, "prl_dp_xbuf_alloc: no uncached memory");
    PRL_HIP_TRY(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocFinegrained));
    *kind = 2;
  }
  const hipError_t e = hipMemset(p, 0, (size_t)bytes);
  if (e != hipSuccess) {
    (void)hipFree(p);
    PRL_HIP_TRY(e);
  }
  *out = p;
  return PRL_OK;
}

extern "C" int prl_dp_xbuf_free(void* p) {
  if (p) PRL_HIP_TRY(hipFree(p));
  return PRL_OK;
}

extern "C" int prl_dp_ipc_handle(void* p, uint8_t* out, int64_t out_bytes) {
  PRL_REQUIRE(p && out && out_bytes >= (int64_t)sizeof(hipIpcMemHandle_t),
              "prl_dp_ipc_handle: need %zu bytes", sizeof(hipIpcMemHandle_t));
  hipIpcMemHandle_t h;
  PRL_HIP_TRY(hipIpcGetMemHandle(&h, p));
  memcpy(out, &h, sizeof(h));
  return PRL_OK;
}

extern "C" int prl_dp_ipc_open(const uint8_t* handle, int64_t bytes, void** out) {
  PRL_REQUIRE(handle && out && bytes >= (int64_t)sizeof(hipIpcMemHandle_t), "prl_dp_ipc_open: bad arguments");
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  PRL_HIP_TRY(hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess));
  return PRL_OK;
}

extern "C" int prl_dp_ipc_close(void* p) {
  if (p) PRL_HIP_TRY(hipIpcCloseMemHandle(p));
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
  const size_t lds = sizeof(float) * (size_t)(UPD_HDR + args.net.Lp + ((upd_scratch_floats(D, upd_nw_host(args.net, false), upd_ts(args.net)) + 3) & ~3));
  PRL_REQUIRE(lds <= 160 * 1024, "prl_ppo_evaluate: %zu B of LDS needed", lds);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(N, UPD_RT), 2 * 256);
  const void* kern = upd_eval_kernel_for(args.net);
  PRL_HIP_TRY(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  void* kargs[] = {&args, &logp, &V, &entropy};
  PRL_HIP_TRY(hipLaunchKernel(kern, dim3(grid), dim3(upd_nt(args.net)), kargs, lds, as_stream(stream)));
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
  args.Gt = G;
  args.R = (int)cdiv(cdiv((int64_t)mini_batch, (int64_t)G), (int64_t)UPD_RT) * UPD_RT;
  args.clip = clip;
  args.vf_coef = vf_coef;
  args.part = ws.part;
  args.ctr = ws.ctr;
  args.grad_target = (unsigned)G;
  args.profile = upd_profile_enabled();
  const size_t lds = upd_lds_bytes(args.net, false);
  hipStream_t st = as_stream(stream);
  const void* kern = upd_grad_kernel_for(args.net);
  PRL_HIP_TRY(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  PRL_HIP_TRY(hipMemsetAsync(ws.ctr, 0, 16, st));
  float inv = inv_count;
  int64_t r0 = row0;
  int bl = B_local;
  const float* img = img_params;
  UpdFold nofold{};
  void* kargs[] = {&args, &img, &grad_out, &r0, &bl, &inv, &nofold};
  // plain launch: G <= 256 workgroups of 1 per CU are co-resident in practice; the in-kernel
  // wait is bounded and reports a timeout through the status word like the persistent kernel
  PRL_HIP_TRY(hipLaunchKernel(kern, dim3(G), dim3(upd_nt(args.net)), kargs, lds, st));
  return PRL_OK;
}

extern "C" int prl_ppo_adam_step(float* img_params, float* img_m, float* img_v, int32_t D,
                                 int32_t A, int32_t discrete, const float* grad, int64_t step,
                                 float lr, double beta1, double beta2, float eps, float weight_decay,
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
// One folded stepped launch: the previous optimizer step's clip + AdamW (state in_* -> out_*,
// gradient grad_prev = its all-reduced gradient image) and then this rank's gradient of global
// minibatch j from the updated parameters, into grad_out.  in_* != out_* and grad_prev !=
// grad_out (the caller double-buffers).  grad_prev == NULL: no AdamW, parameters read from in_p.
extern "C" int prl_ppo_grad_fold_step(const float* in_p, const float* in_m, const float* in_v,
                                      float* out_p, float* out_m, float* out_v,
                                      const float* grad_prev, int64_t step_prev,
                                      float inv_count_prev, int32_t D, int32_t A, int32_t discrete,
                                      const float* S, const float* actions, const float* old_logp,
                                      const float* adv, const float* ret, int64_t N,
                                      int32_t mini_batch, int64_t minibatch_index, float inv_count,
                                      float clip, float vf_coef, float ent_coef, float lr,
                                      double beta1, double beta2, float eps, float weight_decay,
                                      float max_norm, float* loss_out, float* grad_out,
                                      void* workspace, int64_t workspace_bytes, void* stream) {
  UpdArgs args{};
  PRL_REQUIRE(upd_layout(D, A, discrete, args.net), "prl_ppo_grad_fold_step: D=%d A=%d not supported", D, A);
  PRL_REQUIRE(N >= 0 && mini_batch > 0 && minibatch_index >= 0, "prl_ppo_grad_fold_step: bad sizes");
  PRL_REQUIRE(in_p && grad_out && workspace, "prl_ppo_grad_fold_step: null pointer");
  PRL_REQUIRE(!grad_prev || (in_m && in_v && out_p && out_m && out_v && step_prev >= 1),
              "prl_ppo_grad_fold_step: AdamW operands missing");
  PRL_REQUIRE(grad_prev != grad_out && (!grad_prev || (out_p != in_p && out_m != in_m && out_v != in_v)),
              "prl_ppo_grad_fold_step: in/out buffers must differ");
  const int G = upd_grid(mini_batch);
  UpdWs ws;
  const size_t need = upd_ws_carve(args.net, G, reinterpret_cast<char*>(workspace), &ws);
  PRL_REQUIRE((size_t)workspace_bytes >= need, "prl_ppo_grad_fold_step: workspace too small");
  const int64_t row0 = minibatch_index * (int64_t)mini_batch;
  const int B_local = (int)std::max<int64_t>(0, std::min<int64_t>(mini_batch, N - row0));
  PRL_REQUIRE(B_local == 0 || (S && actions && old_logp && adv && ret), "prl_ppo_grad_fold_step: null input");
  args.S = S;
  args.act = actions;
  args.old_logp = old_logp;
  args.adv = adv;
  args.ret = ret;
  args.N = N;
  args.mb = mini_batch;
  args.G = G;
  args.Gt = G;
  args.R = (int)cdiv(cdiv((int64_t)mini_batch, (int64_t)G), (int64_t)UPD_RT) * UPD_RT;
  args.clip = clip;
  args.vf_coef = vf_coef;
  args.part = ws.part;
  args.ctr = ws.ctr;
  args.grad_target = (unsigned)G;
  args.profile = upd_profile_enabled();
  UpdFold f{grad_prev, in_p, in_m, in_v, out_p, out_m, out_v, (double)step_prev,
            lr, beta1, beta2, eps, weight_decay, max_norm, inv_count_prev, vf_coef, ent_coef,
            loss_out};
  const size_t lds = upd_lds_bytes(args.net, false);
  hipStream_t st = as_stream(stream);
  const void* kern = upd_grad_kernel_for(args.net);
  PRL_HIP_TRY(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  PRL_HIP_TRY(hipMemsetAsync(ws.ctr, 0, 16, st));
  float inv = inv_count;
  int64_t r0 = row0;
  int bl = B_local;
  const float* img = in_p;
  void* kargs[] = {&args, &img, &grad_out, &r0, &bl, &inv, &f};
  PRL_HIP_TRY(hipLaunchKernel(kern, dim3(G), dim3(upd_nt(args.net)), kargs, lds, st));
  return PRL_OK;
}

extern "C" int prl_ppo_update_status_ptr(void* workspace, uint32_t** status) {
  PRL_REQUIRE(workspace && status, "prl_ppo_update_status_ptr: null pointer");
  *status = reinterpret_cast<uint32_t*>(workspace) + 3;
  return PRL_OK;
}

// the engine's per-phase timing words (u64 [32], workgroup 0, see PPO/engine.py FusedUpdate.profile)
extern "C" int prl_ppo_update_profile_ptr(void* workspace, uint64_t** prof) {
  PRL_REQUIRE(workspace && prof, "prl_ppo_update_profile_ptr: null pointer");
  UpdWs ws;
  UpdNet n{};
  upd_ws_carve(n, 1, reinterpret_cast<char*>(workspace), &ws);
  *prof = reinterpret_cast<uint64_t*>(ws.prof);
  return PRL_OK;
}

// ---- data-parallel step loop without Python per step (world > 1) ----------------------------
// RCCL is resolved at run time from the library torch loaded (one RCCL per process); the
// communicator is this engine's own (unique id broadcast by the caller over torch.distributed).
namespace {
struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};
RcclApi g_rccl;
}  // namespace

extern "C" int prl_dp_rccl_open(const char* lib_path) {
  PRL_REQUIRE(lib_path, "prl_dp_rccl_open: null path");
  void* h = dlopen(lib_path, RTLD_NOW | RTLD_LOCAL);
  PRL_REQUIRE(h, "prl_dp_rccl_open: dlopen(%s) failed: %s", lib_path, dlerror());
  RcclApi api;
  api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
  api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
  api.all_reduce = reinterpret_cast<decltype(api.all_reduce)>(dlsym(h, "ncclAllReduce"));
  api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
  api.error_string = reinterpret_cast<decltype(api.error_string)>(dlsym(h, "ncclGetErrorString"));
  PRL_REQUIRE(api.get_unique_id && api.comm_init_rank && api.all_reduce && api.comm_destroy,
              "prl_dp_rccl_open: %s lacks the RCCL entry points", lib_path);
  g_rccl = api;
  return PRL_OK;
}

#define PRL_RCCL_TRY(call, what)                                                            \
  do {                                                                                      \
    const ncclResult_t r_ = (call);                                                         \
    PRL_REQUIRE(r_ == ncclSuccess, "%s: RCCL error %d (%s)", what, (int)r_,                 \
                g_rccl.error_string ? g_rccl.error_string(r_) : "?");                       \
  } while (0)

extern "C" int prl_dp_unique_id(uint8_t* id_out, int64_t id_bytes) {
  PRL_REQUIRE(g_rccl.get_unique_id, "prl_dp_unique_id: RCCL not opened (prl_dp_rccl_open)");
  PRL_REQUIRE(id_out && id_bytes == (int64_t)sizeof(ncclUniqueId), "prl_dp_unique_id: need %zu bytes",
              sizeof(ncclUniqueId));
  ncclUniqueId id;
  PRL_RCCL_TRY(g_rccl.get_unique_id(&id), "ncclGetUniqueId");
  memcpy(id_out, &id, sizeof(id));
  return PRL_OK;
}

extern "C" int prl_dp_comm_init(const uint8_t* id, int64_t id_bytes, int32_t nranks, int32_t rank,
                                void** comm) {
  PRL_REQUIRE(g_rccl.comm_init_rank, "prl_dp_comm_init: RCCL not opened (prl_dp_rccl_open)");
  PRL_REQUIRE(id && comm && id_bytes == (int64_t)sizeof(ncclUniqueId) && nranks >= 1 && rank >= 0 &&
                  rank < nranks, "prl_dp_comm_init: bad arguments");
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  PRL_RCCL_TRY(g_rccl.comm_init_rank(&c, nranks, uid, rank), "ncclCommInitRank");
  *comm = c;
  return PRL_OK;
}

extern "C" int prl_dp_comm_destroy(void* comm) {
  if (comm && g_rccl.comm_destroy) g_rccl.comm_destroy(reinterpret_cast<ncclComm_t>(comm));
  return PRL_OK;
}

// The whole k_epochs x nb loop of the stepped engine enqueued from C: per optimizer step the
// gradient kernel (this rank's slice of union minibatch j, scaled 1 / counts[j]), ncclAllReduce
// of the flat gradient image on `stream`, the AdamW kernel; asynchronous, no host sync.  The
// gradient kernel's hand-off counter is zeroed once and its target advances per launch (no
// memset node per step).  Semantics = FusedUpdate.run_stepped's Python loop, bit for bit.
extern "C" int prl_ppo_update_dp(float* img_params, float* img_m, float* img_v, int32_t D, int32_t A,
                                 int32_t discrete, const float* S, const float* actions,
                                 const float* old_logp, const float* adv, const float* ret, int64_t N,
                                 int32_t mini_batch, int32_t k_epochs, int64_t nb,
                                 const int64_t* counts, int64_t step0, float clip, float vf_coef,
                                 float ent_coef, float lr, double beta1, double beta2, float eps,
                                 float weight_decay, float max_norm, float* grad, float* loss_out,
                                 void* workspace, int64_t workspace_bytes, void* comm, void* stream) {
  UpdArgs args{};
  PRL_REQUIRE(upd_layout(D, A, discrete, args.net), "prl_ppo_update_dp: D=%d A=%d not supported", D, A);
  PRL_REQUIRE(N >= 0 && mini_batch > 0 && k_epochs >= 0 && nb >= 0 && counts, "prl_ppo_update_dp: bad sizes");
  PRL_REQUIRE(img_params && img_m && img_v && grad && workspace && comm, "prl_ppo_update_dp: null pointer");
  PRL_REQUIRE(g_rccl.all_reduce, "prl_ppo_update_dp: RCCL not opened (prl_dp_rccl_open)");
  PRL_REQUIRE(N == 0 || (S && actions && old_logp && adv && ret), "prl_ppo_update_dp: null input");
  const int G = upd_grid(mini_batch);
  UpdWs ws;
  const size_t need = upd_ws_carve(args.net, G, reinterpret_cast<char*>(workspace), &ws);
  PRL_REQUIRE((size_t)workspace_bytes >= need, "prl_ppo_update_dp: workspace too small");
  PRL_REQUIRE((int64_t)k_epochs * nb < (int64_t)(1u << 31) / 256, "prl_ppo_update_dp: too many steps");
  for (int64_t j = 0; j < nb; ++j) PRL_REQUIRE(counts[j] > 0, "prl_ppo_update_dp: empty union minibatch %lld", (long long)j);
  args.S = S;
  args.act = actions;
  args.old_logp = old_logp;
  args.adv = adv;
  args.ret = ret;
  args.N = N;
  args.mb = mini_batch;
  args.G = G;
  args.Gt = G;
  args.R = (int)cdiv(cdiv((int64_t)mini_batch, (int64_t)G), (int64_t)UPD_RT) * UPD_RT;
  args.clip = clip;
  args.vf_coef = vf_coef;
  args.part = ws.part;
  args.ctr = ws.ctr;
  const size_t lds = upd_lds_bytes(args.net, false);
  hipStream_t st = as_stream(stream);
  const void* kern = upd_grad_kernel_for(args.net);
  PRL_HIP_TRY(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  PRL_HIP_TRY(hipMemsetAsync(ws.ctr, 0, 16, st));
  const int nt = upd_nt(args.net);
  const unsigned adam_grid = (unsigned)cdiv(args.net.Lp / 4, UPD_THREADS);
  const size_t count = (size_t)args.net.Lp + 4;   // the image + its loss quad
  const ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
  // Per step: ONE launch (the previous step's AdamW folded in front of this step's gradient) and
  // the all-reduce; the last step's AdamW is a separate ppo_adam_kernel.  State and gradient
  // double-buffered: set 0 = the caller's images / grad, set 1 = the workspace's persistent-launch
  // images (unused in stepped mode) and reduction buffer.
  float* sp[2] = {img_params, ws.img};
  float* sm[2] = {img_m, ws.img + count};
  float* sv[2] = {img_v, ws.img + 2 * count};
  float* gb[2] = {grad, ws.red};
  int cur = 0;
  int64_t step = step0;
  unsigned launches = 0;
  const int64_t total = (int64_t)k_epochs * nb;
  float inv_prev = 0.f;
  for (int64_t s = 0; s < total; ++s) {
    const int64_t j = s % nb;
    const int64_t row0 = j * (int64_t)mini_batch;
    int B_local = (int)std::max<int64_t>(0, std::min<int64_t>(mini_batch, N - row0));
    float inv = 1.0f / (float)counts[j];
    int64_t r0 = row0;
    float* gout = gb[s & 1];
    UpdFold f{};
    const float* img = sp[cur];
    if (s > 0) {
      f = UpdFold{gb[(s - 1) & 1], sp[cur], sm[cur], sv[cur], sp[cur ^ 1], sm[cur ^ 1], sv[cur ^ 1],
                  (double)step, lr, beta1, beta2, eps, weight_decay, max_norm, inv_prev, vf_coef,
                  ent_coef, loss_out};
      cur ^= 1;
    }
    args.grad_target = (unsigned)G * (++launches);
    void* kargs[] = {&args, &img, &gout, &r0, &B_local, &inv, &f};
    PRL_HIP_TRY(hipLaunchKernel(kern, dim3(G), dim3(nt), kargs, lds, st));
    PRL_RCCL_TRY(g_rccl.all_reduce(gout, gout, count, ncclFloat32, ncclSum, c, st), "ncclAllReduce");
    ++step;
    inv_prev = inv;
  }
  if (total > 0) {
    hipLaunchKernelGGL(ppo_adam_kernel, dim3(adam_grid), dim3(UPD_THREADS), 0, st, args.net.Lp,
                       sp[cur], sm[cur], sv[cur], gb[(total - 1) & 1], (double)step, lr, beta1,
                       beta2, eps, weight_decay, max_norm, inv_prev, vf_coef, ent_coef, loss_out);
    PRL_LAUNCH_CHECK("ppo_adam_step");
    if (cur != 0) {
      for (int a = 0; a < 3; ++a) {
        float* src = a == 0 ? sp[1] : a == 1 ? sm[1] : sv[1];
        float* dst = a == 0 ? sp[0] : a == 1 ? sm[0] : sv[0];
        PRL_HIP_TRY(hipMemcpyAsync(dst, src, sizeof(float) * args.net.Lp, hipMemcpyDeviceToDevice, st));
      }
    }
    if (((total - 1) & 1) != 0)   // the caller's grad holds the last all-reduced gradient
      PRL_HIP_TRY(hipMemcpyAsync(grad, ws.red, sizeof(float) * count, hipMemcpyDeviceToDevice, st));
  }
  return PRL_OK;
}
