// common.hip -- error plumbing and device checks shared by every libogbx entry point.
#include "common.h"

#include <cstring>

namespace ogbx {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

ogbx_status fail(ogbx_status code, const std::string& msg) {
  set_error(msg);
  return code;
}

ogbx_status hip_fail(hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
  set_error(m);
  return e == hipErrorOutOfMemory ? OGBX_ENOMEM : OGBX_EDEVICE;
}

ogbx_status use_device(int32_t device) {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0)
    return fail(OGBX_EDEVICE, "no HIP device visible (libogbx has no CPU fallback)");
  if (device < 0 || device >= count)
    return fail(OGBX_EDEVICE, "device index " + std::to_string(device) + " out of range (" +
                                  std::to_string(count) + " visible)");
  hipDeviceProp_t prop;
  OGBX_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(OGBX_EDEVICE, std::string("libogbx is built for gfx950; device reports ") +
                                  prop.gcnArchName);
  OGBX_HIP(hipSetDevice(device));
  return OGBX_OK;
}

}  // namespace ogbx

extern "C" {

const char* ogbx_last_error(void) { return ogbx::g_last_error.c_str(); }

int32_t ogbx_abi_version(void) { return OGBX_ABI_VERSION; }
int32_t ogbx_stream_version(void) { return OGBX_STREAM_VERSION; }

const char* ogbx_build_arch(void) { return "gfx950"; }

}  // extern "C"
