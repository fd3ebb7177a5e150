// Library identity / device query entries of the deeprank2_amd C ABI.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/deeprank2_amd.h"

extern "C" const char* dr_version(void) { return "deeprank2_amd 0.1.0 (gfx950)"; }

extern "C" int dr_device_arch(char* buf, int32_t len) {
  if (!buf || len <= 0) return DR_E_ARG;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return (int)e;
  std::strncpy(buf, prop.gcnArchName, (size_t)len - 1);
  buf[len - 1] = 0;
  return DR_OK;
}
