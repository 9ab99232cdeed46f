// Library version and the thread-local last-error string every export sets on failure.
// Host code only (no HIP): also built with -fsanitize=address,undefined (make asan).
#include <string>

#include "fr_engine.h"

namespace fr {
thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace fr

extern "C" int fr_version(void) { return 1; }

extern "C" const char* fr_last_error(void) { return fr::g_last_error.c_str(); }
