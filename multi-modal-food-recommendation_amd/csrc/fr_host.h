// Host-only helpers shared by every export: the last-error string and the argument check.  No HIP
// device code here, so host-only sources (fr_comm.cpp) build with any C++ compiler (make asan).
#pragma once
#include <string>

#include "fr_engine.h"

namespace fr {

void set_error(const std::string& msg);

inline int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

#define FR_REQUIRE(cond, msg)                                        \
  do {                                                               \
    if (!(cond)) return ::fr::fail(FR_EINVAL, std::string(__func__) + ": " + (msg)); \
  } while (0)

}  // namespace fr
