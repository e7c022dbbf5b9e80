// prl_abi.hip — C-ABI housekeeping: version, thread-local error message, workspace sizes.
#include "prl_common.h"

#include <stdarg.h>
#include <stdio.h>

int64_t prl_gae_workspace_bytes(int64_t n);
int64_t prl_surrogate_workspace_bytes(int64_t mb);
int64_t prl_scan_workspace_bytes(int64_t n);
int64_t prl_gn_workspace_bytes(int64_t n);

namespace prl {
static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
}  // namespace prl

extern "C" int prl_abi_version(void) { return PRL_ABI_VERSION; }

extern "C" const char* prl_last_error(void) { return prl::g_err; }

#ifndef PRL_SOURCE_ID
#define PRL_SOURCE_ID "unstamped"
#endif
extern "C" const char* prl_source_id(void) { return PRL_SOURCE_ID; }

extern "C" int64_t prl_workspace_bytes(int op, int64_t n) {
  if (n < 0) n = 0;
  switch (op) {
    case PRL_OP_GAE:
    case PRL_OP_STATS: return prl_gae_workspace_bytes(n);
    case PRL_OP_SURROGATE: return prl_surrogate_workspace_bytes(n);
    case PRL_OP_SCAN: return prl_scan_workspace_bytes(n);
    case PRL_OP_GN: return prl_gn_workspace_bytes(n);
    default: return -1;
  }
}

// Test utility: fill every CU's LDS with `value` (workgroups of 256 threads holding the whole
// 160 KB each, several rounds over the CUs).  LDS is not cleared between launches, so a kernel
// that reads LDS it did not write this launch sees what the previous launch left; tests run a
// kernel after a NaN fill and after a zero fill and require the same bits.
namespace prl {
__global__ __launch_bounds__(256) void fill_lds_kernel(float value, int nfloat4) {
  extern __shared__ float4 lds_fill[];
  const float4 v{value, value, value, value};
  for (int i = threadIdx.x; i < nfloat4; i += blockDim.x) lds_fill[i] = v;
  __syncthreads();
  if (threadIdx.x == 0 && lds_fill[0].x == 12345.0f && value != 12345.0f) lds_fill[1] = v;   // keep the stores
}
}  // namespace prl

extern "C" int prl_debug_fill_lds(float value, void* stream) {
  constexpr int bytes = 160 * 1024;
  PRL_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(prl::fill_lds_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  int dev = 0, cus = 0;
  PRL_HIP_TRY(hipGetDevice(&dev));
  PRL_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipLaunchKernelGGL(prl::fill_lds_kernel, dim3((unsigned)(4 * cus)), dim3(256), bytes,
                     prl::as_stream(stream), value, bytes / 16);
  PRL_LAUNCH_CHECK("fill_lds");
  return PRL_OK;
}
