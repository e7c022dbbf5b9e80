// prl_gae.hip — GAE(lambda) reverse scan, advantage statistics and normalisation.
//
// Replaces PPO.compute_gae (PPO/PPO.py:107-120) and `advantages = returns - V;
// (adv - mean) / (std + 1e-8)` (PPO.py:198-199).
//
// Bit-exactness.  The reference runs, over float32 numpy values (NumPy 2 / NEP 50: Python floats
// are weak, so every step stays float32):
//     delta = r[t] + gamma * nv * (1 - d[t]) - V[t]          ((r + ((gamma*nv)*(1-d))) - V)
//     gae   = delta + gamma * lambda * (1 - d[t]) * gae      (gamma*lambda formed in float64)
//     ret[t] = gae + V[t];  nv = V[t]
// with gae = 0 and nv = V[-1] initially (PPO.py:110, :188).  A float32 affine recurrence is not
// associative, so a parallel prefix over (c_t, delta_t) pairs would change the rounding.  Instead
// the scan is parallel across SEGMENTS: wherever c_t = gamma*lambda*(1-d_t) == 0 (an episode end)
// the recurrence restarts and everything to its left is independent of everything to its right.
// Within a segment the recurrence is evaluated sequentially in the reference's order, so every
// output is bit-identical for finite inputs (a non-finite carry would leak through 0*inf = NaN in
// the reference; here the chain restarts at d = 1).
//
// Work decomposition (single pass, ONE launch, no host-side memset):
//   * tile = 256 threads x 8 consecutive elements = 2048 elements, 16-B vector loads; delta_t and
//     c_t are formed elementwise and staged in LDS;
//   * each thread finishes everything at or left of the LAST break in its own chunk; the carries
//     between chunks are chained once per RUN of break-free chunks (gae_kernel), the runs listed
//     in LDS and walked by the lowest threads, packed into the fewest waves;
//   * tiles are taken in reverse, in R interleaved streams (gae_kernel): a tile's successor was
//     dispatched one round of resident workgroups earlier.  A tile publishes its carry-out
//     g[first element] as one 8-byte {epoch, value} granule with one agent-scope store (data =
//     flag, MI355X guide Guideline 16 R2) as soon as it is known, before it ever waits; the tile
//     to its left reads it.  A stream's first tile computes its successor's carry itself (that
//     tile runs last); a tile that still finds no granule after a bounded poll computes the carry
//     by a scalar look-ahead — the same sequential chain, so the result is bit-identical and
//     correctness never depends on placement or order.  No ticket atomic: a single contended word
//     caps at ~88 ops/us on MI355X (guide: dequeue row), i.e. ~73 us at 6400 tiles.
//   * statistics: when adv is requested each tile stores {sum adv, sum adv^2} (f64) to its slot;
//     a one-workgroup fold kernel behind the scan sums the slots in tile order -> sums_out
//     (deterministic) and advances the epoch used as the granule tag;
//   * the workspace is zero-initialised once by the caller; its layout depends only on the
//     buffer's size, so calls of different n can share it.  Two launches per call (scan, fold).
#include "prl_common.h"

#include <algorithm>

namespace prl {

// Phase marks for tools/exp/gae_phases.hip (which defines PRL_GAE_MARK before including this
// file); empty in the product build.
#ifndef PRL_GAE_MARK
#define PRL_GAE_MARK(i)
#endif
#ifndef PRL_GAE_MARK_TAIL   // same, recorded by the tail-run thread (255)
#define PRL_GAE_MARK_TAIL(i)
#endif

constexpr int GAE_THREADS = 256;
constexpr int GAE_EPT = 8;
constexpr int GAE_TILE = GAE_THREADS * GAE_EPT;
constexpr int GAE_GROUP = 64;                 // tiles per arrival group
constexpr unsigned GAE_SPIN_LIMIT = 4096;     // ~100 us of s_sleep(1) polls before look-ahead

__host__ __device__ inline int64_t gae_ntiles(int64_t n) { return (n + GAE_TILE - 1) / GAE_TILE; }
__host__ __device__ inline int64_t gae_ngroups(int64_t nt) { return (nt + GAE_GROUP - 1) / GAE_GROUP; }

struct GaeWs {
  unsigned* ctrs;               // [0] spare, [1] group arrivals, [2] look-ahead count, [3] epoch
  unsigned* group_ctr;          // [ngroups], one per 64-B line (stride 16 words)
  unsigned long long* gran;     // [ntiles] {epoch << 32 | float bits}
  double2* tile_sums;           // [ntiles]
  double2* group_sums;          // [ngroups]
};

inline int64_t gae_ws_bytes_tiles(int64_t nt) {
  const int64_t ng = gae_ngroups(nt);
  return 64 + 64 * ng + ((8 * nt + 15) / 16) * 16 + 16 * nt + 16 * ng + 64;
}
inline int64_t gae_ws_bytes(int64_t n) { return gae_ws_bytes_tiles(gae_ntiles(n)); }
// The layout is carved for the largest tile count the BUFFER can hold, never for the current n:
// one buffer serves calls of every size, and the counters it keeps armed between launches must
// sit at the same offsets in all of them.  Exact: the largest nt with bytes(nt) <= bytes (the
// estimate from bytes(nt) <= 216 + 25.25 * nt is only a starting point; rounding down from it
// once under-sized the carve by a tile, so the last tile's carry granule overwrote tile 0's
// statistics).
inline int64_t gae_capacity_tiles(int64_t bytes) {
  int64_t nt = std::max<int64_t>(1, (int64_t)((double)(bytes - 216) / 25.25));
  while (nt > 1 && gae_ws_bytes_tiles(nt) > bytes) --nt;
  while (gae_ws_bytes_tiles(nt + 1) <= bytes) ++nt;
  return nt;
}
inline GaeWs gae_ws_carve(void* ws, int64_t nt) {
  const int64_t ng = gae_ngroups(nt);
  char* p = static_cast<char*>(ws);
  GaeWs w;
  w.ctrs = reinterpret_cast<unsigned*>(p);
  p += 64;
  w.group_ctr = reinterpret_cast<unsigned*>(p);
  p += 64 * ng;
  w.gran = reinterpret_cast<unsigned long long*>(p);
  p += ((8 * nt + 15) / 16) * 16;
  w.tile_sums = reinterpret_cast<double2*>(p);
  p += 16 * nt;
  w.group_sums = reinterpret_cast<double2*>(p);
  return w;
}

__device__ inline unsigned long long ld_sc1(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_sc1(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_sc1_d2(double2* p, double2 v) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  st_sc1(q, __double_as_longlong(v.x));
  st_sc1(q + 1, __double_as_longlong(v.y));
}
__device__ inline double2 ld_sc1_d2(const double2* p) {
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
  return double2{__longlong_as_double(ld_sc1(q)), __longlong_as_double(ld_sc1(q + 1))};
}

// one GAE step in the reference's float32 order
__device__ inline float gae_delta(float r, float d, float v, float nv, float gf) {
  float a = gf * nv;
  a = a * (1.0f - d);
  const float s = r + a;
  return s - v;
}

struct ChunkDC {
  float4 da, db, ca, cb;
};
__device__ inline ChunkDC chunk_load(const float* s_delta, const float* s_c, int chunk) {
  const float4* d4 = reinterpret_cast<const float4*>(s_delta + chunk * GAE_EPT);
  const float4* c4 = reinterpret_cast<const float4*>(s_c + chunk * GAE_EPT);
  return ChunkDC{d4[0], d4[1], c4[0], c4[1]};
}
// the reference's recurrence over one 8-element chunk, last element first
__device__ inline float chunk_apply(const ChunkDC& x, float carry) {
  carry = x.db.w + x.cb.w * carry;
  carry = x.db.z + x.cb.z * carry;
  carry = x.db.y + x.cb.y * carry;
  carry = x.db.x + x.cb.x * carry;
  carry = x.da.w + x.ca.w * carry;
  carry = x.da.z + x.ca.z * carry;
  carry = x.da.y + x.ca.y * carry;
  carry = x.da.x + x.ca.x * carry;
  return carry;
}
// Walk chunks hi, hi-1, ..., lo: write each one's carry-in (g at the first element of the chunk to
// its right) to s_cin, and apply every chunk > stop to the carry.  The walk is the kernel's serial
// path (~500 dependent mul/add pairs for a trained CartPole episode); two chunks' LDS reads are
// issued together, so one LDS latency is exposed per two chunks (a prefetch carried across the
// loop's back edge was sunk back behind its branch by the compiler; four chunks cost occupancy).
__device__ inline float chunk_walk(const float* s_delta, const float* s_c, float* s_cin, int hi,
                                   int lo, int stop, float carry) {
  int k = hi;
  for (; k - 1 > stop && k - 1 >= lo; k -= 2) {   // two chunks' reads in flight at once
    const ChunkDC x0 = chunk_load(s_delta, s_c, k), x1 = chunk_load(s_delta, s_c, k - 1);
    s_cin[k] = carry;
    carry = chunk_apply(x0, carry);
    s_cin[k - 1] = carry;
    carry = chunk_apply(x1, carry);
  }
  for (; k >= lo; --k) {
    s_cin[k] = carry;
    if (k > stop) carry = chunk_apply(chunk_load(s_delta, s_c, k), carry);
  }
  return carry;
}

// g at index `start` computed from global memory: walk forward to the first break (c == 0) or
// the end, then run the chain backward in the reference's order.  Used only when a successor's
// granule did not show up in time; bit-identical to the granule path.
__device__ float gae_lookahead(const float* r, const float* d, const float* V, float nv_end,
                               int64_t n, float gf, float glf, int64_t start) {
  int64_t p = start;
  while (p < n && glf * (1.0f - d[p]) != 0.0f) ++p;
  float g = 0.0f;
  for (int64_t t = (p < n ? p : n - 1); t >= start; --t) {
    const float nv = (t + 1 < n) ? V[t + 1] : nv_end;
    g = gae_delta(r[t], d[t], V[t], nv, gf) + (glf * (1.0f - d[t])) * g;
  }
  return g;
}

// Block end: the tile's {sum adv, sum adv^2} go to tile_sums[tile] with a plain store; the fold
// kernel launched behind this one (gae_fold_kernel) sums them in tile order after the kernel
// boundary.  (An in-launch hand-off to a last arriver cost every tile a write-through drain plus
// a returning atomic, ~2 us of a ~19 us tile lifetime at 7 tiles per CU.)
__device__ inline void gae_tile_sums(const GaeWs& ws, int64_t tile, bool with_sums, double2 mine) {
  if (with_sums && threadIdx.x == 0) ws.tile_sums[tile] = mine;
}

// One workgroup: sums_out = the tile sums folded in a fixed order (thread t: tiles t, t + 1024,
// ... ascending; then the waves' partials in wave order), and the workspace's granule epoch
// advanced to this launch's tag.  Deterministic.
constexpr int GAE_FOLD_THREADS = 1024;
__global__ __launch_bounds__(GAE_FOLD_THREADS) void gae_fold_kernel(GaeWs ws, int64_t ntiles,
                                                                    int with_sums,
                                                                    double* __restrict__ out) {
  __shared__ double s_part[2][GAE_FOLD_THREADS / 64];
  if (with_sums) {
    double a = 0.0, b = 0.0;
    for (int64_t t = threadIdx.x; t < ntiles; t += GAE_FOLD_THREADS) {
      const double2 v = ws.tile_sums[t];
      a += v.x;
      b += v.y;
    }
    a = wave_sum(a);
    b = wave_sum(b);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
      s_part[0][wid] = a;
      s_part[1][wid] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double sa = 0.0, sb = 0.0;
      for (int w = 0; w < GAE_FOLD_THREADS / 64; ++w) {
        sa += s_part[0][w];
        sb += s_part[1][w];
      }
      out[0] = sa;
      out[1] = sb;
    }
  }
  if (threadIdx.x == 0) {
    const unsigned t = ws.ctrs[3] + 1u;
    ws.ctrs[3] = t ? t : 1u;   // the tag the launch before used (gae_tag)
  }
}

__device__ inline unsigned gae_tag(const GaeWs& ws) {
  const unsigned t = __hip_atomic_load(&ws.ctrs[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  return t ? t : 1u;
}

// Stage one tile: load its r / d / V (16-B vector loads when aligned and full), form delta_t and
// c_t in the reference's order into LDS, run every chunk's recurrence at or left of its last
// break, and publish the wave's break ballot to s_mask; g0 = g at the chunk's first element
// when it has a break (pb >= 0).  No barrier inside.
template <bool VEC>
__device__ inline void gae_stage(const float* __restrict__ r, const float* __restrict__ d,
                                 const float* __restrict__ V, int64_t n, float nv_end, float gf,
                                 float glf, int64_t tile, float* s_delta, float* s_c,
                                 unsigned long long* s_mask, float (&vv)[GAE_EPT],
                                 float& g0, int& pb) {
  const int tid = threadIdx.x;
  const int64_t i0 = tile * GAE_TILE + (int64_t)tid * GAE_EPT;
  float rr[GAE_EPT], dd[GAE_EPT];
  if (VEC && i0 + GAE_EPT <= n) {
    const float4* r4 = reinterpret_cast<const float4*>(r + i0);
    const float4* d4 = reinterpret_cast<const float4*>(d + i0);
    const float4* v4 = reinterpret_cast<const float4*>(V + i0);
    const float4 ra = r4[0], rb = r4[1], da = d4[0], db = d4[1], va = v4[0], vb = v4[1];
    rr[0] = ra.x; rr[1] = ra.y; rr[2] = ra.z; rr[3] = ra.w; rr[4] = rb.x; rr[5] = rb.y; rr[6] = rb.z; rr[7] = rb.w;
    dd[0] = da.x; dd[1] = da.y; dd[2] = da.z; dd[3] = da.w; dd[4] = db.x; dd[5] = db.y; dd[6] = db.z; dd[7] = db.w;
    vv[0] = va.x; vv[1] = va.y; vv[2] = va.z; vv[3] = va.w; vv[4] = vb.x; vv[5] = vb.y; vv[6] = vb.z; vv[7] = vb.w;
  } else {
#pragma unroll
    for (int k = 0; k < GAE_EPT; ++k) {
      const int64_t i = i0 + k;
      const bool in = i < n;
      rr[k] = in ? r[i] : 0.f;
      dd[k] = in ? d[i] : 1.f;  // padding: c = 0, delta = 0
      vv[k] = in ? V[i] : 0.f;
    }
  }
  PRL_GAE_MARK(1);
  const int64_t inext = i0 + GAE_EPT;
  const float vnext = (inext < n) ? V[inext] : nv_end;
  float dl[GAE_EPT], cc[GAE_EPT];
#pragma unroll
  for (int k = 0; k < GAE_EPT; ++k) {
    const int64_t i = i0 + k;
    float nv = (k + 1 < GAE_EPT) ? vv[k + 1] : vnext;
    if (i + 1 == n) nv = nv_end;
    dl[k] = gae_delta(rr[k], dd[k], vv[k], nv, gf);
    cc[k] = glf * (1.0f - dd[k]);
  }
  {
    float4* sd4 = reinterpret_cast<float4*>(s_delta + tid * GAE_EPT);
    float4* sc4 = reinterpret_cast<float4*>(s_c + tid * GAE_EPT);
    sd4[0] = float4{dl[0], dl[1], dl[2], dl[3]};
    sd4[1] = float4{dl[4], dl[5], dl[6], dl[7]};
    sc4[0] = float4{cc[0], cc[1], cc[2], cc[3]};
    sc4[1] = float4{cc[4], cc[5], cc[6], cc[7]};
  }
  pb = -1;
#pragma unroll
  for (int k = 0; k < GAE_EPT; ++k)
    if (cc[k] == 0.0f) pb = k;
  float gg = 0.0f;
#pragma unroll
  for (int k = GAE_EPT - 1; k >= 0; --k)
    if (k <= pb) gg = dl[k] + cc[k] * gg;
  g0 = gg;
  const unsigned long long bal = __ballot(pb >= 0);   // chunks of this wave with a break
  if ((tid & 63) == 0) s_mask[tid >> 6] = bal;
}

// Tile order.  Dispatch index b runs tile ntiles-1-t', t' = (b % R) * Q + b / R: R streams of
// Q consecutive tiles each, stream r's tiles one ROUND (R dispatches) apart.  A tile's successor
// (the tile to its right, whose carry-out it needs) was therefore dispatched a round earlier and
// has normally published long before — with t' = b the successor was the block dispatched just
// before, still walking its own first run, so every tile waited out a whole run (trained
// CartPole: 500 steps) before its tail walk could start.  A stream's first tile (q = 0) has its
// successor at the END of the order; it computes that carry itself: it stages the successor tile
// first and walks its first run (bit-identical to what the successor publishes).
template <bool VEC>
__global__ __launch_bounds__(GAE_THREADS) void gae_kernel(
    const float* __restrict__ r, const float* __restrict__ d, const float* __restrict__ V,
    const float* __restrict__ next_value, int64_t n, float gf, float glf, float* __restrict__ ret,
    float* __restrict__ adv, GaeWs ws, int64_t ntiles, int64_t R, int64_t Q,
    double* __restrict__ sums_out) {
  __shared__ __attribute__((aligned(16))) float s_delta[GAE_TILE];
  __shared__ __attribute__((aligned(16))) float s_c[GAE_TILE];
  __shared__ unsigned long long s_mask[GAE_THREADS / 64];
  __shared__ float s_cin[GAE_THREADS];
  __shared__ float s_pre;
  __shared__ int s_run_hi[GAE_THREADS], s_run_lo[GAE_THREADS];   // the tile's runs (below)
  __shared__ float s_run_g[GAE_THREADS];
  __shared__ unsigned s_tag;

  const int tid = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int64_t q = b / R;
  const int64_t tp = (b - q * R) * Q + q;
  if (tp >= ntiles) return;   // past the last stream's end (the whole block: no barrier yet)
  const int64_t tile = ntiles - 1 - tp;
  const int64_t i0 = tile * GAE_TILE + (int64_t)tid * GAE_EPT;
  PRL_GAE_MARK(0);
  if (tid == 0) s_tag = gae_tag(ws);
  // nv for the final element (PPO.py:188: next_value = V[-1])
  const float nv_end = next_value ? *next_value : V[n - 1];
  const bool has_succ = tile + 1 < ntiles;
  const bool pre = has_succ && q == 0;   // the successor is run at the end: compute its carry
  float vv[GAE_EPT], g0;
  int pb;
  if (pre) {
    // stage tiles tile+1, tile+2, ... until one has a break (normally the first): its first run
    // gives its carry-out; then every break-free tile back to tile+1 is walked whole
    int64_t tb = tile + 1;
    int F = -1;   // first chunk of tile tb with a break
    // first wave 0's quarter of tile tb alone (512 elements: any episode of <= 500 steps ends
    // in it, so the re-read is a quarter tile); only a break-free quarter stages the whole tile
    if (tid < 64) {
      gae_stage<VEC>(r, d, V, n, nv_end, gf, glf, tb, s_delta, s_c, s_mask, vv, g0, pb);
    }
    __syncthreads();
    if (s_mask[0]) F = __builtin_ctzll(s_mask[0]);
    __syncthreads();   // every wave has read s_mask[0] before a full stage rewrites it
    for (; F < 0;) {
      gae_stage<VEC>(r, d, V, n, nv_end, gf, glf, tb, s_delta, s_c, s_mask, vv, g0, pb);
      __syncthreads();
      for (int w2 = 0; w2 < GAE_THREADS / 64; ++w2) {
        const unsigned long long mk = s_mask[w2];
        if (mk) {
          F = w2 * 64 + __builtin_ctzll(mk);
          break;
        }
      }
      if (F >= 0 || tb + 1 >= ntiles) break;
      __syncthreads();   // everyone has read s_mask before the next stage rewrites it
      ++tb;
    }
    if (F >= 0) {
      if (tid == F) s_pre = chunk_walk(s_delta, s_c, s_cin, F - 1, 0, -1, g0);
    } else if (tid == 0) {   // the array's last tile, no break: the chain starts at gae = 0
      s_pre = chunk_walk(s_delta, s_c, s_cin, GAE_THREADS - 1, 0, -1, 0.0f);
    }
    __syncthreads();
    for (int64_t tw = tb - 1; tw > tile; --tw) {   // break-free tiles (rare): whole-tile walks
      gae_stage<VEC>(r, d, V, n, nv_end, gf, glf, tw, s_delta, s_c, s_mask, vv, g0, pb);
      __syncthreads();
      if (tid == 0) s_pre = chunk_walk(s_delta, s_c, s_cin, GAE_THREADS - 1, 0, -1, s_pre);
      __syncthreads();
    }
  }
  // the successor's granule, polled early (a round old, so normally there)
  unsigned long long gw = 0ull;
  if (tid == GAE_THREADS - 1 && has_succ && !pre) gw = ld_sc1(&ws.gran[tile + 1]);
  gae_stage<VEC>(r, d, V, n, nv_end, gf, glf, tile, s_delta, s_c, s_mask, vv, g0, pb);
  __syncthreads();
  PRL_GAE_MARK(2);
  const unsigned tag = s_tag;
  const bool hb = pb >= 0;
  auto publish = [&](float carry_out) {   // g at the tile's first element -> predecessor tile
    st_sc1(&ws.gran[tile], ((unsigned long long)tag << 32) | __float_as_uint(carry_out));
  };
  // chunk 0 with a break: the tile's carry-out is local — publish before anything else
  if (tid == 0 && hb) publish(g0);

  // Carries between chunks, each chained ONCE.  A RUN is the stretch of break-free chunks left
  // of a chunk with a break (down to, and including as a carry target, the previous chunk with a
  // break), walked right to left from that chunk's g at its first element, writing each chunk's
  // carry-in (g at the first element of the chunk to its right) to s_cin; the run at the tile's
  // end starts from the successor tile's carry.  The runs are listed in LDS in chunk order and
  // walked by threads 0, 1, ... — packed into the fewest waves: a walk keeps one lane of its
  // wave busy, so with every chunk walking its own run (one lane in each of four waves) the
  // walks of trained 500-step episodes filled the SIMDs' issue slots four times over.
  // Same recurrence order as the reference throughout.
  const int lane = tid & 63, wv = tid >> 6;
  int nb = 0;   // chunks with a break
#pragma unroll
  for (int w2 = 0; w2 < GAE_THREADS / 64; ++w2) nb += __popcll(s_mask[w2]);
  if (hb) {
    int rank = __popcll(s_mask[wv] & ((1ull << lane) - 1ull));
    for (int w2 = 0; w2 < wv; ++w2) rank += __popcll(s_mask[w2]);
    int p = -1;   // previous chunk with a break
    const unsigned long long below = lane == 0 ? 0ull : (s_mask[wv] << (64 - lane));
    if (below) {
      p = tid - 1 - __builtin_clzll(below);
    } else {
      for (int w2 = wv - 1; w2 >= 0; --w2) {
        const unsigned long long mk = s_mask[w2];
        if (mk) {
          p = w2 * 64 + 63 - __builtin_clzll(mk);
          break;
        }
      }
    }
    s_run_hi[rank] = tid - 1;
    s_run_lo[rank] = p;
    s_run_g[rank] = g0;
  }
  // the tail run exists when chunk 255 has no break at all (a break that is not its last
  // element leaves only that chunk's own tail, fed by s_cin[255])
  const bool tail_run = (s_mask[GAE_THREADS / 64 - 1] >> 63) == 0ull && s_c[GAE_TILE - 1] != 0.0f;
  if (tid == GAE_THREADS - 1 && pb != GAE_EPT - 1) {
    float cin = 0.0f;  // beyond the last element: gae = 0 (PPO.py:110)
    PRL_GAE_MARK_TAIL(8);
    if (pre) {
      cin = s_pre;
    } else if (has_succ) {
      unsigned spins = 0;
      bool got = false;
      for (;;) {
        if ((unsigned)(gw >> 32) == tag) {
          cin = __uint_as_float((unsigned)(gw & 0xffffffffull));
          got = true;
          break;
        }
        if (++spins >= GAE_SPIN_LIMIT) break;
        __builtin_amdgcn_s_sleep(1);
        gw = ld_sc1(&ws.gran[tile + 1]);
      }
      if (!got) {
        cin = gae_lookahead(r, d, V, nv_end, n, gf, glf, (tile + 1) * (int64_t)GAE_TILE);
        __hip_atomic_fetch_add(&ws.ctrs[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    PRL_GAE_MARK_TAIL(9);
    if (tail_run) {
      int L = -1;   // last chunk with a break
      for (int w2 = GAE_THREADS / 64 - 1; w2 >= 0; --w2) {
        const unsigned long long mk = s_mask[w2];
        if (mk) {
          L = w2 * 64 + 63 - __builtin_clzll(mk);
          break;
        }
      }
      s_run_hi[nb] = GAE_THREADS - 1;
      s_run_lo[nb] = L;
      s_run_g[nb] = cin;
    } else {
      s_cin[GAE_THREADS - 1] = cin;
    }
  }
  __syncthreads();
  if (tid < nb + (tail_run ? 1 : 0)) {
    const int hi = s_run_hi[tid], lo = s_run_lo[tid];
    const float carry = chunk_walk(s_delta, s_c, s_cin, hi, lo < 0 ? 0 : lo, lo, s_run_g[tid]);
    if (lo < 0 && hi >= 0) publish(carry);   // walked to chunk 0: g(tile start)
  }
  if (tid == GAE_THREADS - 1) PRL_GAE_MARK_TAIL(10);
  __syncthreads();
  PRL_GAE_MARK(3);
  // the chunk's outputs: g at or left of its last break again (the local recurrence, recomputed
  // rather than kept in registers across the walks), then after it from its carry-in; delta / c
  // re-read from LDS
  float g[GAE_EPT];
  {
    const ChunkDC x = chunk_load(s_delta, s_c, tid);
    const float dl2[GAE_EPT] = {x.da.x, x.da.y, x.da.z, x.da.w, x.db.x, x.db.y, x.db.z, x.db.w};
    const float cc2[GAE_EPT] = {x.ca.x, x.ca.y, x.ca.z, x.ca.w, x.cb.x, x.cb.y, x.cb.z, x.cb.w};
    float carry = pb != GAE_EPT - 1 ? s_cin[tid] : 0.0f;
#pragma unroll
    for (int k = GAE_EPT - 1; k >= 0; --k) {
      if (k == pb) carry = 0.0f;   // the local chain starts from gae = 0 at the last break
      carry = dl2[k] + cc2[k] * carry;
      g[k] = carry;
    }
  }

  PRL_GAE_MARK(4);
  // outputs: ret = gae + V (PPO.py:116), adv = ret - V (PPO.py:198)
  float rt[GAE_EPT], av[GAE_EPT];
#pragma unroll
  for (int k = 0; k < GAE_EPT; ++k) {
    rt[k] = g[k] + vv[k];
    av[k] = rt[k] - vv[k];
  }
  if (VEC && i0 + GAE_EPT <= n) {
    float4* o4 = reinterpret_cast<float4*>(ret + i0);
    o4[0] = float4{rt[0], rt[1], rt[2], rt[3]};
    o4[1] = float4{rt[4], rt[5], rt[6], rt[7]};
    if (adv) {
      float4* a4 = reinterpret_cast<float4*>(adv + i0);
      a4[0] = float4{av[0], av[1], av[2], av[3]};
      a4[1] = float4{av[4], av[5], av[6], av[7]};
    }
  } else {
#pragma unroll
    for (int k = 0; k < GAE_EPT; ++k) {
      if (i0 + k < n) {
        ret[i0 + k] = rt[k];
        if (adv) adv[i0 + k] = av[k];
      }
    }
  }
  PRL_GAE_MARK(5);
  double2 mine{0.0, 0.0};
  if (adv) {
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int k = 0; k < GAE_EPT; ++k) {
      if (i0 + k < n) {
        const double x = (double)av[k];
        s1 += x;
        s2 += x * x;
      }
    }
    __shared__ double s_red[2][GAE_THREADS / 64];
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    const int lane = tid & 63, wid = tid >> 6;
    if (lane == 0) { s_red[0][wid] = s1; s_red[1][wid] = s2; }
    __syncthreads();
    if (tid == 0)
      for (int w = 0; w < GAE_THREADS / 64; ++w) { mine.x += s_red[0][w]; mine.y += s_red[1][w]; }
  }
  gae_tile_sums(ws, tile, adv != nullptr, mine);
  PRL_GAE_MARK(6);
}

// Plain statistics pass (prl_adv_stats): per-tile sums + grouped ordered fold.
__global__ __launch_bounds__(GAE_THREADS) void stats_kernel(const float* __restrict__ x, int64_t n,
                                                            GaeWs ws, int64_t ntiles,
                                                            double* __restrict__ sums_out) {
  const int64_t tile = blockIdx.x;
  const int64_t i0 = tile * GAE_TILE + (int64_t)threadIdx.x * GAE_EPT;
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int k = 0; k < GAE_EPT; ++k) {
    const int64_t i = i0 + k;
    if (i < n) {
      const double v = (double)x[i];
      s1 += v;
      s2 += v * v;
    }
  }
  __shared__ double s_red[2][GAE_THREADS / 64];
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { s_red[0][wid] = s1; s_red[1][wid] = s2; }
  __syncthreads();
  double2 mine{0.0, 0.0};
  if (threadIdx.x == 0)
    for (int w = 0; w < GAE_THREADS / 64; ++w) { mine.x += s_red[0][w]; mine.y += s_red[1][w]; }
  gae_tile_sums(ws, tile, true, mine);
}

// (x - mean) / (std_unbiased + eps) in float32, statistics from f64 sums (PPO.py:199).
__global__ __launch_bounds__(256) void normalize_kernel(const float* __restrict__ x, int64_t n,
                                                        const double* __restrict__ sums, double count,
                                                        float eps, float* __restrict__ out) {
  const double mean = sums[0] / count;
  double var = (count > 1.0) ? (sums[1] - sums[0] * mean) / (count - 1.0) : __builtin_nan("");
  if (var < 0.0) var = 0.0;
  const float mean_f = (float)mean;
  const float den = (float)sqrt(var) + eps;
  const int64_t n4 = n >> 2;
  const bool vec = aligned16(x) && aligned16(out);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (vec) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
    float4* o4 = reinterpret_cast<float4*>(out);
    for (int64_t j = i; j < n4; j += stride) {
      const float4 v = x4[j];
      o4[j] = float4{(v.x - mean_f) / den, (v.y - mean_f) / den, (v.z - mean_f) / den,
                     (v.w - mean_f) / den};
    }
    for (int64_t j = n4 * 4 + i; j < n; j += stride) out[j] = (x[j] - mean_f) / den;
  } else {
    for (int64_t j = i; j < n; j += stride) out[j] = (x[j] - mean_f) / den;
  }
}

}  // namespace prl

using namespace prl;

int64_t prl_gae_workspace_bytes(int64_t n) { return gae_ws_bytes(n); }

namespace {
// workgroups of the scan resident at once on the current device (cached per device)
int64_t gae_resident_blocks() {
  static int cached[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, reinterpret_cast<const void*>(gae_kernel<true>), GAE_THREADS, 0) != hipSuccess ||
        cus <= 0 || per_cu <= 0)
      return 1792;
    cached[dev] = cus * per_cu;
  }
  return cached[dev];
}
}  // namespace

extern "C" int prl_gae(const float* r, const float* d, const float* V, const float* next_value,
                       int64_t n, double gamma, double lam, float* ret, float* adv,
                       double* sums_out, void* workspace, int64_t workspace_bytes, void* stream) {
  PRL_REQUIRE(n >= 0, "prl_gae: n < 0");
  if (n == 0) return PRL_OK;
  PRL_REQUIRE(r && d && V && ret, "prl_gae: null pointer");
  PRL_REQUIRE(!adv || sums_out, "prl_gae: adv requested without sums_out");
  PRL_REQUIRE(n < ((int64_t)1 << 40), "prl_gae: n too large");
  const int64_t nt = gae_ntiles(n);
  PRL_REQUIRE(nt < (int64_t)0x7fffffff, "prl_gae: too many tiles");
  PRL_REQUIRE(workspace && workspace_bytes >= gae_ws_bytes(n),
              "prl_gae: workspace too small (%lld < %lld)", (long long)workspace_bytes,
              (long long)gae_ws_bytes(n));
  PRL_REQUIRE(gae_capacity_tiles(workspace_bytes) >= nt, "prl_gae: workspace layout too small");
  hipStream_t s = as_stream(stream);
  GaeWs ws = gae_ws_carve(workspace, gae_capacity_tiles(workspace_bytes));
  // gamma * nv * (1 - d): gamma is a weak Python float -> float32; gamma * lambda is a Python
  // float product (float64), rounded to float32 when it meets the float32 (1 - d).
  const float gf = (float)gamma;
  const float glf = (float)(gamma * lam);
  const bool vec = aligned16(r) && aligned16(d) && aligned16(V) && aligned16(ret) &&
                   (!adv || aligned16(adv));
  // R streams (gae_kernel's tile order): about one round of resident workgroups, but at least
  // 4 tiles per stream (a stream's first tile also stages its successor's first quarter, or the
  // whole successor when that quarter has no episode end: <= 1/16 extra reads, 1/4 at worst)
  // (measured on trained 500-step segments: R = 1/2 or 3/4 of a round 10-20 % slower, 1.5 or 2
  // rounds 4 % slower)
  const int64_t R = std::max<int64_t>(1, std::min<int64_t>(gae_resident_blocks(), (nt + 3) / 4));
  const int64_t Q = (nt + R - 1) / R;
  const unsigned grid = (unsigned)(R * Q);
  if (vec)
    hipLaunchKernelGGL(gae_kernel<true>, dim3(grid), dim3(GAE_THREADS), 0, s, r, d, V,
                       next_value, n, gf, glf, ret, adv, ws, nt, R, Q, sums_out);
  else
    hipLaunchKernelGGL(gae_kernel<false>, dim3(grid), dim3(GAE_THREADS), 0, s, r, d, V,
                       next_value, n, gf, glf, ret, adv, ws, nt, R, Q, sums_out);
  PRL_LAUNCH_CHECK("gae");
  hipLaunchKernelGGL(gae_fold_kernel, dim3(1), dim3(GAE_FOLD_THREADS), 0, s, ws, nt,
                     adv ? 1 : 0, sums_out);
  PRL_LAUNCH_CHECK("gae_fold");
  return PRL_OK;
}

extern "C" int prl_adv_stats(const float* x, int64_t n, double* sums_out, void* workspace,
                             int64_t workspace_bytes, void* stream) {
  PRL_REQUIRE(n >= 0, "prl_adv_stats: n < 0");
  PRL_REQUIRE(sums_out, "prl_adv_stats: null sums_out");
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    PRL_HIP_TRY(hipMemsetAsync(sums_out, 0, 2 * sizeof(double), s));
    return PRL_OK;
  }
  PRL_REQUIRE(x, "prl_adv_stats: null x");
  const int64_t nt = gae_ntiles(n);
  PRL_REQUIRE(workspace && workspace_bytes >= gae_ws_bytes(n), "prl_adv_stats: workspace too small");
  PRL_REQUIRE(gae_capacity_tiles(workspace_bytes) >= nt, "prl_adv_stats: workspace layout too small");
  GaeWs ws = gae_ws_carve(workspace, gae_capacity_tiles(workspace_bytes));
  hipLaunchKernelGGL(stats_kernel, dim3((unsigned)nt), dim3(GAE_THREADS), 0, s, x, n, ws, nt, sums_out);
  PRL_LAUNCH_CHECK("adv_stats");
  hipLaunchKernelGGL(gae_fold_kernel, dim3(1), dim3(GAE_FOLD_THREADS), 0, s, ws, nt, 1, sums_out);
  PRL_LAUNCH_CHECK("adv_stats_fold");
  return PRL_OK;
}

extern "C" int prl_adv_normalize(const float* x, int64_t n, const double* sums, double count,
                                 float eps, float* out, void* stream) {
  PRL_REQUIRE(n >= 0, "prl_adv_normalize: n < 0");
  if (n == 0) return PRL_OK;
  PRL_REQUIRE(x && sums && out, "prl_adv_normalize: null pointer");
  PRL_REQUIRE(count >= (double)n, "prl_adv_normalize: count < n");
  const int64_t work = aligned16(x) && aligned16(out) ? cdiv(n, 4) : n;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(work, 256), 2048);
  hipLaunchKernelGGL(normalize_kernel, dim3(grid), dim3(256), 0, as_stream(stream), x, n, sums,
                     count, eps, out);
  PRL_LAUNCH_CHECK("adv_normalize");
  return PRL_OK;
}
