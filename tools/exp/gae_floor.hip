// Experiment (tools/, not product): the memory floor of the GAE scan's traffic pattern.
// 3 float arrays in, 2 out, n elements.  V0: 8 consecutive elements per thread (the GAE
// kernel's mapping, 2 x float4 per array per thread); V1: one float4 per lane per step, lanes
// contiguous (fully coalesced), grid-stride.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void copy_v0(const float* r, const float* d, const float* V,
                                               float* o1, float* o2, int64_t n) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i0 + 8 > n) return;
  const float4* r4 = (const float4*)(r + i0);
  const float4* d4 = (const float4*)(d + i0);
  const float4* v4 = (const float4*)(V + i0);
  float4 a = r4[0], b = r4[1], c = d4[0], e = d4[1], f = v4[0], g = v4[1];
  float4 x = {a.x + c.x + f.x, a.y + c.y + f.y, a.z + c.z + f.z, a.w + c.w + f.w};
  float4 y = {b.x + e.x + g.x, b.y + e.y + g.y, b.z + e.z + g.z, b.w + e.w + g.w};
  ((float4*)(o1 + i0))[0] = x;
  ((float4*)(o1 + i0))[1] = y;
  ((float4*)(o2 + i0))[0] = f;
  ((float4*)(o2 + i0))[1] = g;
}

__global__ __launch_bounds__(256) void copy_v1(const float4* r, const float4* d, const float4* V,
                                               float4* o1, float4* o2, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 a = r[i], c = d[i], f = V[i];
    o1[i] = float4{a.x + c.x + f.x, a.y + c.y + f.y, a.z + c.z + f.z, a.w + c.w + f.w};
    o2[i] = f;
  }
}

extern "C" int run_copy(int variant, const float* r, const float* d, const float* V, float* o1,
                        float* o2, int64_t n, int grid, void* stream) {
  if (variant == 0)
    hipLaunchKernelGGL(copy_v0, dim3((unsigned)((n / 8 + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, r, d, V, o1, o2, n);
  else
    hipLaunchKernelGGL(copy_v1, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float4*)r,
                       (const float4*)d, (const float4*)V, (float4*)o1, (float4*)o2, n / 4);
  return (int)hipGetLastError();
}
