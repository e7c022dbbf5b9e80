// prl_common.h — shared device helpers for libprl_hip.so (gfx950 only).
//
// Error plumbing for the C-ABI (include/prl_abi.h), the counter/seeded RNGs the env kernels use
// (Philox4x32-10 for action sampling, numpy-exact PCG64 + SeedSequence for gymnasium-exact
// seeded resets) and a deterministic double-precision sin/cos (fdlibm kernels + Cody-Waite
// medium-range reduction).  Everything here is compiled with -ffp-contract=off so that the
// float sequences are the reference's sequences, operation for operation.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/prl_abi.h"

namespace prl {

// ---- error plumbing ------------------------------------------------------------------------
int set_error(int code, const char* fmt, ...);
#define PRL_HIP_TRY(expr)                                                                  \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return ::prl::set_error(PRL_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)
#define PRL_REQUIRE(cond, ...)                                 \
  do {                                                         \
    if (!(cond)) return ::prl::set_error(PRL_ERR_ARG, __VA_ARGS__); \
  } while (0)
// Check the launch that was just enqueued.
#define PRL_LAUNCH_CHECK(name) PRL_HIP_TRY(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
__host__ __device__ inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- Philox4x32-10 (counter-based; action sampling) ----------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ inline uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = mulhi32(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = mulhi32(M1, c.z), lo1 = M1 * c.z;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// [0,1) float with 24 random bits: exact in f32, identical on host and device.
__host__ __device__ inline float u01(uint32_t x) { return (float)(x >> 8) * 0x1p-24f; }
// (0,1] float, for logs.
__host__ __device__ inline float u01_open0(uint32_t x) { return (float)((x >> 8) + 1u) * 0x1p-24f; }

// ---- PCG64 (numpy's default bit generator: 128-bit LCG, XSL-RR output) ---------------------
// state packed as {state_hi, state_lo, inc_hi, inc_lo}.
struct pcg64 { uint64_t shi, slo, ihi, ilo; };

__host__ __device__ inline uint64_t umulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

__host__ __device__ inline void pcg64_step(pcg64& g) {
  const uint64_t MHI = 0x2360ED051FC65DA4ull, MLO = 0x4385DF649FCCF645ull;
  // state = state * MULT + inc  (mod 2^128)
  const uint64_t lo = g.slo * MLO;
  const uint64_t hi = g.shi * MLO + g.slo * MHI + umulhi64(g.slo, MLO);
  const uint64_t nlo = lo + g.ilo;
  const uint64_t nhi = hi + g.ihi + (nlo < lo ? 1ull : 0ull);
  g.slo = nlo;
  g.shi = nhi;
}

__host__ __device__ inline uint64_t pcg64_next64(pcg64& g) {
  pcg64_step(g);
  const uint64_t x = g.shi ^ g.slo;
  const unsigned rot = (unsigned)(g.shi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

// numpy random_standard_uniform / next_double: 53 random bits.
__host__ __device__ inline double pcg64_next_double(pcg64& g) {
  return (double)(pcg64_next64(g) >> 11) * (1.0 / 9007199254740992.0);
}

// numpy Generator.uniform(low, high): low + (high - low) * next_double   (range formed first).
__host__ __device__ inline double pcg64_uniform(pcg64& g, double low, double high) {
  const double range = high - low;
  return low + range * pcg64_next_double(g);
}

// numpy SeedSequence(seed).generate_state(4, uint64) -> PCG64 seeding (pcg64_set_seed).
__host__ __device__ inline uint32_t ss_hashmix(uint32_t value, uint32_t& hc) {
  value ^= hc;
  hc *= 0x931e8875u;
  value *= hc;
  value ^= value >> 16;
  return value;
}
__host__ __device__ inline uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
  r ^= r >> 16;
  return r;
}

__host__ __device__ inline pcg64 pcg64_from_seed(uint64_t seed) {
  uint32_t ent[2];
  int nent;
  ent[0] = (uint32_t)seed;
  ent[1] = (uint32_t)(seed >> 32);
  nent = (seed >> 32) ? 2 : 1;
  uint32_t pool[4];
  uint32_t hc = 0x43b0d7e5u;
  for (int i = 0; i < 4; ++i) pool[i] = ss_hashmix(i < nent ? ent[i] : 0u, hc);
  for (int s = 0; s < 4; ++s)
    for (int d = 0; d < 4; ++d)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
  // (nent <= pool size: no remaining entropy to fold in)
  uint32_t w[8];
  uint32_t hb = 0x8b51f9ddu;
  for (int i = 0; i < 8; ++i) {
    uint32_t v = pool[i & 3];
    v ^= hb;
    hb *= 0x58f38dedu;
    v *= hb;
    v ^= v >> 16;
    w[i] = v;
  }
  uint64_t val[4];
  for (int i = 0; i < 4; ++i) val[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  // pcg_setseq_128_srandom_r(initstate = val0:val1, initseq = val2:val3)
  pcg64 g;
  g.shi = 0;
  g.slo = 0;
  g.ihi = (val[2] << 1) | (val[3] >> 63);
  g.ilo = (val[3] << 1) | 1ull;
  pcg64_step(g);
  const uint64_t lo = g.slo + val[1];
  g.shi = g.shi + val[0] + (lo < g.slo ? 1ull : 0ull);
  g.slo = lo;
  pcg64_step(g);
  return g;
}

// ---- deterministic double sin/cos (fdlibm __kernel_sin/__kernel_cos + __ieee754_rem_pio2) ---
__host__ __device__ inline int32_t hi_word(double x) {
  return (int32_t)(__builtin_bit_cast(uint64_t, x) >> 32);
}

__host__ __device__ inline double k_sin(double x, double y, int iy) {
  const double S1 = -0x1.5555555555549p-3, S2 = 0x1.111111110f8a6p-7,
               S3 = -0x1.a01a019c161d5p-13, S4 = 0x1.71de357b1fe7dp-19,
               S5 = -0x1.ae5e68a2b9cebp-26, S6 = 0x1.5d93a5acfd57cp-33;
  const double z = x * x;
  const double v = z * x;
  const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

__host__ __device__ inline double k_cos(double x, double y) {
  const double C1 = 0x1.555555555554cp-5, C2 = -0x1.6c16c16c15177p-10,
               C3 = 0x1.a01a019cb159p-16, C4 = -0x1.27e4f809c52adp-22,
               C5 = 0x1.1ee9ebdb4b1c4p-29, C6 = -0x1.8fae9be8838d4p-37;
  const double z = x * x;
  const double w = z * z;
  const double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  const double hz = 0.5 * z;
  const double ww = 1.0 - hz;
  return ww + (((1.0 - ww) - hz) + (z * r - x * y));
}

// Medium-range reduction, valid for |x| < 2^19 * pi/2 (covers every env state we step; larger
// arguments are reduced by fmod with 2*pi first, which is exact).  Returns n, y0 + y1 = x - n*pi/2.
__host__ __device__ inline int rem_pio2(double x, double& y0, double& y1) {
  const double invpio2 = 0x1.45f306dc9c883p-1, pio2_1 = 0x1.921fb544p+0,
               pio2_1t = 0x1.0b4611a626331p-34, pio2_2 = 0x1.0b4611a6p-34,
               pio2_2t = 0x1.3198a2e037073p-69, pio2_3 = 0x1.3198a2ep-69,
               pio2_3t = 0x1.b839a252049c1p-104;
  const int32_t ix = hi_word(x) & 0x7fffffff;
  const double fn = rint(x * invpio2);
  const int n = (int)fn;
  double r = x - fn * pio2_1;
  double w = fn * pio2_1t;
  y0 = r - w;
  const int j = ix >> 20;
  int i = j - ((hi_word(y0) >> 20) & 0x7ff);
  if (i > 16) {
    double t = r;
    w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    y0 = r - w;
    i = j - ((hi_word(y0) >> 20) & 0x7ff);
    if (i > 49) {
      t = r;
      w = fn * pio2_3;
      r = t - w;
      w = fn * pio2_3t - ((t - r) - w);
      y0 = r - w;
    }
  }
  y1 = (r - y0) - w;
  return n;
}

__host__ __device__ inline double prl_sin(double x) {
  const int32_t ix = hi_word(x) & 0x7fffffff;
  if (ix <= 0x3fe921fb) {                // |x| <= pi/4
    if (ix < 0x3e400000) return x;       // |x| < 2^-27
    return k_sin(x, 0.0, 0);
  }
  if (ix >= 0x7ff00000) return x - x;    // inf / nan
  if (ix >= 0x41200000) x = fmod(x, 0x1.921fb54442d18p+2);  // |x| >= 2^19: exact 2*pi fold
  double y0, y1;
  const int n = rem_pio2(x, y0, y1);
  switch (n & 3) {
    case 0: return k_sin(y0, y1, 1);
    case 1: return k_cos(y0, y1);
    case 2: return -k_sin(y0, y1, 1);
    default: return -k_cos(y0, y1);
  }
}

__host__ __device__ inline double prl_cos(double x) {
  const int32_t ix = hi_word(x) & 0x7fffffff;
  if (ix <= 0x3fe921fb) {
    if (ix < 0x3e400000) return 1.0;
    return k_cos(x, 0.0);
  }
  if (ix >= 0x7ff00000) return x - x;
  if (ix >= 0x41200000) x = fmod(x, 0x1.921fb54442d18p+2);
  double y0, y1;
  const int n = rem_pio2(x, y0, y1);
  switch (n & 3) {
    case 0: return k_cos(y0, y1);
    case 1: return -k_sin(y0, y1, 1);
    case 2: return -k_cos(y0, y1);
    default: return k_sin(y0, y1, 1);
  }
}

// ---- block-level helpers -------------------------------------------------------------------
// Inclusive scan of one int64 per thread across a 256-thread block (4 waves of 64).
__device__ inline int64_t block_inclusive_scan_256(int64_t v, int64_t* lds_wave_tot /*[4]*/,
                                                   int64_t& block_total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t u = __shfl_up(v, off, 64);
    if (lane >= off) v += u;
  }
  if (lane == 63) lds_wave_tot[wid] = v;
  __syncthreads();
  int64_t prefix = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int64_t t = lds_wave_tot[w];
    if (w < wid) prefix += t;
    tot += t;
  }
  block_total = tot;
  __syncthreads();  // lds_wave_tot may be reused by the caller
  return v + prefix;
}

// Sum of a double over the 64 lanes of a wave by DPP (no LDS round trips), result in lane 63:
// xor-1 / xor-2 quad perms, half-row and row mirrors, then row_bcast:15 / row_bcast:31 (GFX9 DPP).
template <int CTRL, int ROWS>
__device__ inline double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWS, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ inline double wave_sum_f64_to63(double v) {
  v += dpp_f64<0xB1, 0xF>(v);    // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E, 0xF>(v);    // quad_perm [2,3,0,1]
  v += dpp_f64<0x141, 0xF>(v);   // row_half_mirror
  v += dpp_f64<0x140, 0xF>(v);   // row_mirror: every lane holds its row's sum
  v += dpp_f64<0x142, 0xA>(v);   // row_bcast:15 -> rows 1, 3
  v += dpp_f64<0x143, 0xC>(v);   // row_bcast:31 -> rows 2, 3
  return v;                      // lane 63: the wave's sum
}

// the same DPP tree for a float (result in lane 63)
template <int CTRL, int ROWS>
__device__ inline float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xF, false));
}
__device__ inline float wave_sum_f32_to63(float v) {
  v += dpp_f32<0xB1, 0xF>(v);
  v += dpp_f32<0x4E, 0xF>(v);
  v += dpp_f32<0x141, 0xF>(v);
  v += dpp_f32<0x140, 0xF>(v);
  v += dpp_f32<0x142, 0xA>(v);
  v += dpp_f32<0x143, 0xC>(v);
  return v;
}

template <typename T>
__device__ inline T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

}  // namespace prl
