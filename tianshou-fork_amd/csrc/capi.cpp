// libtsrl: library identity and the thread-local error channel (include/tsrl.h).
#include <stdarg.h>
#include <stdio.h>

#include "tsrl_common.h"

namespace tsrl {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

}  // namespace tsrl

extern "C" const char* tsrl_version(void) { return "tsrl 0.1.0 gfx950"; }
extern "C" const char* tsrl_last_error(void) { return tsrl::g_err; }
