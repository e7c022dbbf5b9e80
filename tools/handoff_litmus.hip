// handoff_litmus.hip — litmus test for the engine's cross-workgroup hand-offs (DESIGN.md §3,
// "A round-1 race"): G workgroups (one per CU, 256 threads) repeatedly publish small payloads with
// sc1 stores, drain them (s_waitcnt vmcnt(0)), pass a workgroup barrier, arrive at an 8-way
// sharded agent-scope counter, poll it with sc1 loads, and then EVERY wave of EVERY workgroup
// reads EVERY published word with sc1 loads and checks it against the value of this iteration.
// A second counter closes each iteration (no writer runs ahead of a slow reader).  Workgroups are
// delayed unevenly per iteration; the buffer is zero-filled by a plain-store kernel before every
// launch (as torch's ws.zero_() did in the round-1 diagnostic).
//
// Layouts of the published words (mode):
//   0 packed-4B      word (g, w) at NW g + w: each wave's lane 63 stores 4 B; 8 workgroups share
//                    one 128-B line (round 1's clip-norm pieces)
//   1 padded-4B      word (g, w) at 32 g + w: the same 4-B stores, each workgroup's own line
//   2 padded-16B     the workgroup's 4 words gathered in LDS, one lane stores them as ONE 16-B
//                    store into its own line
//   3 packed-16B     one 16-B store per workgroup at 4 g: 8 workgroups' stores share one line
//   4 straddle-16B   each workgroup stores Q = 70 quads (1,120 B) at quad offset 70 g with 16-B
//                    stores from consecutive lanes: slices that start mid-line, so the two ends
//                    of every slice share a 128-B line with a neighbour (the engine's phase-B
//                    slices of Qtot = 2,258 quads over G = 32)
//   5 aligned-16B    the same slices padded to whole 128-B lines (quad offset 72 g)
//   6 engine-r1      round 1's phase B -> C as it ran: each workgroup stores its slice of a
//                    QT = 2,258-quad reduced gradient (16-B sc1 stores, slices [QT g / G,
//                    QT (g + 1) / G)) and then its 4 packed 4-B norm pieces (lane 63 per wave);
//                    readers issue their 16-B loads of the WHOLE gradient first, then sum the
//                    pieces (round 1's phase C order); both are checked
// Readers load 4-B words (modes 0-3) or 16-B quads (modes 4-5), all sc1 (mode 6: both).
//
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/handoff_litmus tools/handoff_litmus.hip
// Run:   tools/handoff_litmus <G> <iterations> <reps>    (one JSON line per mode)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                            \
    }                                                                                     \
  } while (0)

constexpr int NT = 256, NW = 4, SHARDS = 8;
constexpr int QS = 70;                 // quads per slice (modes 4-5)
constexpr int QT = 2258, RED0 = 2048;  // mode 6: gradient quads, its first word
constexpr unsigned SPIN_LIMIT = 1u << 22;
constexpr int CTR_A = 32, CTR_B = CTR_A + 32 * SHARDS, CTR_WORDS = CTR_B + 32 * SHARDS;

typedef unsigned v4u __attribute__((ext_vector_type(4)));
__device__ inline __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ inline unsigned ld_sc1u(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_sc1u(unsigned* p, unsigned x) {
  __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline v4u ld16_sc1(__amdgpu_buffer_rsrc_t rs, unsigned byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16);
}
__device__ inline void st16_sc1(__amdgpu_buffer_rsrc_t rs, unsigned byte_off, v4u v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, byte_off, 0, 16);
}

__device__ inline unsigned isum8(unsigned v) {
  v += (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  v += (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  v += (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
  return v;
}
// one whole wave: wait until the shards of counter `base` sum to >= target (bounded)
__device__ inline bool wait_sharded(unsigned* ctr, int base, unsigned target) {
  const int l = threadIdx.x & 63;
  for (unsigned spins = 0;; ++spins) {
    const unsigned v = l < SHARDS ? ld_sc1u(ctr + base + 32 * l) : 0u;
    const unsigned tot = (unsigned)__builtin_amdgcn_readlane((int)isum8(v), 0);
    if (tot >= target) return true;
    if (ld_sc1u(ctr + 2) != 0u) return false;
    if (spins > SPIN_LIMIT) {
      if (l == 0) st_sc1u(ctr + 2, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ inline unsigned hash(unsigned a, unsigned b) {
  unsigned h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  return h ^ (h >> 13);
}
// the value word idx carries in iteration it: a hash (never 0, the fill value; two iterations'
// values of one word differ with probability 1 - 2^-31)
__device__ inline unsigned expect(int it, int idx) { return hash((unsigned)it, (unsigned)idx * 0x10001u + 7u) | 1u; }

// returns whether the iteration's published words are visible; errors counted per wave
__global__ __launch_bounds__(NT, 1) void litmus_kernel(int mode, int iters, unsigned* buf,
                                                       unsigned* ctr, unsigned* err,
                                                       unsigned* first) {
  extern __shared__ unsigned lds[];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, g = blockIdx.x, G = gridDim.x;
  __shared__ int s_abort;
  const __amdgpu_buffer_rsrc_t rs = rsrc(buf);
  unsigned nerr = 0;
  for (int it = 0; it < iters; ++it) {
    // uneven load: 0..255 s_sleep(1) before publishing
    const unsigned d = hash((unsigned)it, (unsigned)g) & 255u;
    for (unsigned k = 0; k < d; ++k) __builtin_amdgcn_s_sleep(1);
    // ---- publish
    if (mode == 0 || mode == 1) {
      const int idx = mode == 0 ? NW * g + w : 32 * g + w;
      if (l == 63) st_sc1u(buf + idx, expect(it, idx));
    } else if (mode == 2 || mode == 3) {
      if (l == 63) lds[w] = 0u;   // (placeholder so every wave touches LDS)
      __syncthreads();
      if (t == 0) {
        const int idx = mode == 2 ? 32 * g : NW * g;
        v4u v;
        v.x = expect(it, idx);
        v.y = expect(it, idx + 1);
        v.z = expect(it, idx + 2);
        v.w = expect(it, idx + 3);
        st16_sc1(rs, (unsigned)idx * 4u, v);
      }
    } else if (mode == 6) {
      const int qlo = QT * g / G, qhi = QT * (g + 1) / G;
      for (int q = qlo + t; q < qhi; q += NT) {
        const int idx = RED0 + 4 * q;
        v4u v;
        v.x = expect(it, idx);
        v.y = expect(it, idx + 1);
        v.z = expect(it, idx + 2);
        v.w = expect(it, idx + 3);
        st16_sc1(rs, (unsigned)idx * 4u, v);
      }
      if (l == 63) st_sc1u(buf + NW * g + w, expect(it, NW * g + w));
    } else {
      const int q0 = mode == 4 ? QS * g : 72 * g;
      for (int q = t; q < QS; q += NT) {
        const int idx = 4 * (q0 + q);
        v4u v;
        v.x = expect(it, idx);
        v.y = expect(it, idx + 1);
        v.z = expect(it, idx + 2);
        v.w = expect(it, idx + 3);
        st16_sc1(rs, (unsigned)idx * 4u, v);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t < 64) {
      if (t == 0)
        __hip_atomic_fetch_add(ctr + CTR_A + 32 * (g & (SHARDS - 1)), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      const bool ok = wait_sharded(ctr, CTR_A, (unsigned)G * (unsigned)(it + 1));
      if (t == 0) s_abort = ok ? 0 : 1;
    }
    __syncthreads();
    if (s_abort) break;
    // ---- every wave reads every published word (sc1) and checks it
    if (mode == 6) {
      constexpr int NQ = (QT + NT - 1) / NT;
      v4u gq[NQ];
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int q = t + i * NT;
        if (q < QT) gq[i] = ld16_sc1(rs, (unsigned)(RED0 + 4 * q) * 4u);
      }
      for (int i = l; i < NW * G; i += 64) {
        const unsigned got = ld_sc1u(buf + i);
        if (got != expect(it, i)) {
          ++nerr;
          if (atomicCAS(first, 0u, 1u) == 0u) {
            first[1] = (unsigned)it; first[2] = (unsigned)g; first[3] = (unsigned)i;
            first[4] = got; first[5] = expect(it, i);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int q = t + i * NT;
        const int idx = RED0 + 4 * q;
        if (q < QT && (gq[i].x != expect(it, idx) || gq[i].y != expect(it, idx + 1) ||
                       gq[i].z != expect(it, idx + 2) || gq[i].w != expect(it, idx + 3))) {
          ++nerr;
          if (atomicCAS(first, 0u, 1u) == 0u) {
            first[1] = (unsigned)it; first[2] = (unsigned)g; first[3] = (unsigned)idx;
            first[4] = gq[i].x; first[5] = expect(it, idx);
          }
        }
      }
    } else if (mode <= 3) {
      const int words = mode == 0 || mode == 3 ? NW * G : 32 * G;
      for (int i = l; i < words; i += 64) {
        if ((mode == 1 || mode == 2) && (i & 31) >= NW) continue;
        const unsigned got = ld_sc1u(buf + i);
        if (got != expect(it, i)) {
          ++nerr;
          if (atomicCAS(first, 0u, 1u) == 0u) {
            first[1] = (unsigned)it; first[2] = (unsigned)g; first[3] = (unsigned)i;
            first[4] = got; first[5] = expect(it, i);
          }
        }
      }
    } else {
      const int stride = mode == 4 ? QS : 72;
      for (int s = 0; s < G; ++s) {
        for (int q = l; q < QS; q += 64) {
          const int idx = 4 * (stride * s + q);
          const v4u got = ld16_sc1(rs, (unsigned)idx * 4u);
          const unsigned e0 = expect(it, idx);
          const bool bad = got.x != e0 || got.y != expect(it, idx + 1) ||
                           got.z != expect(it, idx + 2) || got.w != expect(it, idx + 3);
          if (bad) {
            ++nerr;
            if (atomicCAS(first, 0u, 1u) == 0u) {
              first[1] = (unsigned)it; first[2] = (unsigned)g; first[3] = (unsigned)idx;
              first[4] = got.x; first[5] = e0;
            }
          }
        }
      }
    }
    // ---- close the iteration: nobody republishes before every reader is done
    __syncthreads();
    if (t < 64) {
      if (t == 0)
        __hip_atomic_fetch_add(ctr + CTR_B + 32 * (g & (SHARDS - 1)), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      const bool ok = wait_sharded(ctr, CTR_B, (unsigned)G * (unsigned)(it + 1));
      if (t == 0) s_abort = ok ? 0 : 1;
    }
    __syncthreads();
    if (s_abort) break;
  }
  if (nerr) atomicAdd(err, nerr);
}

// a torch-like zero fill with plain stores, spread over every XCD
__global__ void plain_fill(unsigned* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = 0u;
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 32;
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  const int reps = argc > 3 ? atoi(argv[3]) : 4;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  if (G < 8 || G > prop.multiProcessorCount || iters < 1 || iters > 16000) {
    fprintf(stderr, "need 8 <= G <= %d CUs and 1 <= iterations <= 16000\n", prop.multiProcessorCount);
    return 2;
  }
  const int words = (4 * 72 * G > RED0 + 4 * QT ? 4 * 72 * G : RED0 + 4 * QT) + 64;
  unsigned *buf, *ctr, *err;
  CK(hipMalloc(&buf, words * 4));
  CK(hipMalloc(&ctr, CTR_WORDS * 4));
  CK(hipMalloc(&err, 8 * 4));
  const size_t lds = 96 * 1024;   // one workgroup per CU
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&litmus_kernel),
                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const char* names[] = {"packed-4B", "padded-4B", "padded-16B", "packed-16B", "straddle-16B",
                         "aligned-16B", "engine-r1"};
  int rc = 0;
  for (int mode = 0; mode < 7; ++mode) {
    unsigned total = 0, aborted = 0, firstrec[6] = {0, 0, 0, 0, 0, 0};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms = 0.f;
    for (int r = 0; r < reps; ++r) {
      hipLaunchKernelGGL(plain_fill, dim3(1024), dim3(256), 0, 0, buf, words);
      CK(hipMemset(ctr, 0, CTR_WORDS * 4));
      CK(hipMemset(err, 0, 8 * 4));
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(litmus_kernel, dim3(G), dim3(NT), lds, 0, mode, iters, buf, ctr, err, err + 1);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipDeviceSynchronize());
      float m = 0.f;
      CK(hipEventElapsedTime(&m, e0, e1));
      ms += m;
      unsigned h[8], c2;
      CK(hipMemcpy(h, err, 32, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&c2, ctr + 2, 4, hipMemcpyDeviceToHost));
      total += h[0];
      aborted += c2 ? 1u : 0u;
      if (h[1] && !firstrec[0]) memcpy(firstrec, h + 1, sizeof(firstrec));
    }
    printf("{\"mode\": \"%s\", \"G\": %d, \"iterations\": %d, \"reps\": %d, \"stale_reads\": %u, "
           "\"aborted_reps\": %u, \"us_per_iteration\": %.3f, \"first\": {\"it\": %u, \"reader_wg\": %u, "
           "\"word\": %u, \"got\": \"0x%08x\", \"want\": \"0x%08x\"}}\n",
           names[mode], G, iters, reps, total, aborted, 1000.0 * ms / (reps * (double)iters),
           firstrec[1], firstrec[2], firstrec[3], firstrec[4], firstrec[5]);
    fflush(stdout);
    if (aborted) rc = 1;
  }
  CK(hipFree(buf));
  CK(hipFree(ctr));
  CK(hipFree(err));
  return rc;
}
