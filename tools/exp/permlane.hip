// Semantics probe: v_permlane16_swap / v_permlane32_swap on gfx950 (one wave, lane ids).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(l, l + 100u, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
  auto r2 = __builtin_amdgcn_permlane32_swap(l, l + 100u, false, false);
  out[128 + l] = r2[0];
  out[192 + l] = r2[1];
}
int main() {
  unsigned* d;
  hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[4] = {"p16 r0", "p16 r1", "p32 r0", "p32 r1"};
  for (int a = 0; a < 4; ++a) {
    printf("%s:", nm[a]);
    for (int l = 0; l < 64; ++l) printf(" %u", h[a * 64 + l]);
    printf("\n");
  }
  return 0;
}
