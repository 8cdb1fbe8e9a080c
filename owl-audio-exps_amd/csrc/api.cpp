// C-ABI plumbing for libowlk: error reporting and version.  Declarations: include/owlk.h.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

namespace owlk {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return 2;
  }
  return 0;
}

}  // namespace owlk

extern "C" const char* owlk_last_error(void) { return owlk::g_err; }

extern "C" int owlk_version(void) { return 1; }

// 1 when this build carries gfx950 code objects and a device is visible, else 0 (never throws)
extern "C" int owlk_device_ok(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 0;
  return (prop.gcnArchName[0] == 'g' && prop.gcnArchName[3] == '9' && prop.gcnArchName[4] == '5') ? 1 : 0;
}
