// Error reporting shared by every libabd entry point.
#include <cstdarg>
#include <cstdio>

#include "../../include/abd.h"

namespace abd {

static thread_local char g_err[512] = "";

void set_last_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

}  // namespace abd

extern "C" {
const char* abd_last_error(void) { return abd::g_err; }
int abd_version(void) { return 1; }
}
