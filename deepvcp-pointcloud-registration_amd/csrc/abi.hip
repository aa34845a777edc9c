// abi.hip -- error reporting and version query of the C ABI (include/dvcp.h).
#include <cstdarg>
#include <cstdio>

#include "common.h"

namespace dvcp {

static thread_local char g_err[512] = "ok";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return DVCP_EHIP;
  }
  return DVCP_OK;
}

}  // namespace dvcp

extern "C" const char* dvcp_last_error(void) { return dvcp::g_err; }

// 2: dvcp_paper_pose gained inlier_ratio, dvcp_sa_bn_stats gained zrows, dvcp_fps_split_probe gained out_xyz
// (round 3); a consumer built against an older header must fail cleanly, not pass shifted pointers.
extern "C" int dvcp_abi_version(void) { return DVCP_ABI_VERSION; }
