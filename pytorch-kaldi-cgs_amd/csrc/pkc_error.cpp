// pkc_error.cpp — thread-local error string and ABI version of libpkc.so.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/pkc.h"

namespace pkc {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace pkc

extern "C" int pkc_abi_version(void) { return PKC_ABI_VERSION; }
extern "C" const char* pkc_last_error(void) { return pkc::g_err; }
