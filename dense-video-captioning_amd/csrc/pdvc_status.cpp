// pdvc_status.cpp -- thread-local error message + ABI version for libpdvc_hip.so.
#include <cstdarg>
#include <cstdio>

#include "pdvc_msda.h"

namespace {
thread_local char g_msg[512] = "";
}

extern "C" int pdvc_set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_msg, sizeof(g_msg), fmt, ap);
    va_end(ap);
    return code;
}

extern "C" const char* pdvc_last_error(void) { return g_msg; }
extern "C" int pdvc_abi_version(void) { return PDVC_ABI_VERSION; }
