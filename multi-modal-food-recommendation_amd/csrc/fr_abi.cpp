// Library-level exports that need the HIP runtime (device query).  Error reporting lives in
// fr_error.cpp, the host sampler in fr_sampler.cpp.
#include <hip/hip_runtime.h>

#include "fr_engine.h"

extern "C" int fr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
