// C-ABI plumbing of libsavqa.so: version and thread-local error reporting.
#include <hip/hip_runtime.h>

#include <string>

#include "common.h"

namespace savqa {
static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return (int)e;
  }
  return 0;
}
}  // namespace savqa

extern "C" int savqa_version(void) { return 1; }
extern "C" const char* savqa_last_error(void) { return savqa::g_err.c_str(); }

extern "C" int savqa_struct_sizes(int64_t* out, int32_t n) {
  if (!out || n < 3) return savqa::fail(SAVQA_EINVAL, "savqa_struct_sizes: out needs 3 slots");
  out[0] = (int64_t)sizeof(savqa_gemm_desc);
  out[1] = (int64_t)sizeof(savqa_gemm_lp_desc);
  out[2] = (int64_t)sizeof(savqa_collate_field);
  if (n >= 4) out[3] = (int64_t)sizeof(savqa_x6_planes_job);
  return 0;
}
