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
