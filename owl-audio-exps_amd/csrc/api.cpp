// C-ABI plumbing for libowlk: error reporting and version.  Declarations: include/owlk.h.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <mutex>

#include "common.hpp"

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

// Grow-only scratch per (device, slot).  Users are stream-ordered on the caller's stream; a slot
// per user keeps two users' buffers apart.  Growth drains the device before freeing the old one.
void* workspace(size_t bytes, int slot) {
  static std::mutex mu;
  static void* buf[64][WS_SLOTS] = {};
  static size_t cap[64][WS_SLOTS] = {};
  int dev = 0;
  if (slot < 0 || slot >= WS_SLOTS || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (cap[dev][slot] < bytes) {
    if (buf[dev][slot]) {
      if (hipDeviceSynchronize() != hipSuccess) return nullptr;
      (void)hipFree(buf[dev][slot]);
      buf[dev][slot] = nullptr;
      cap[dev][slot] = 0;
    }
    if (hipMalloc(&buf[dev][slot], bytes) != hipSuccess) {
      buf[dev][slot] = nullptr;
      return nullptr;
    }
    cap[dev][slot] = bytes;
  }
  return buf[dev][slot];
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
