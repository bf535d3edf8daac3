// ou_common.h -- shared host helpers for the ouhip C ABI (error reporting).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

namespace ouhip_detail {
inline char* err_buf()
{
    static thread_local char buf[512] = {0};
    return buf;
}
}  // namespace ouhip_detail

inline int ou_fail(int code, const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(ouhip_detail::err_buf(), 512, fmt, ap);
    va_end(ap);
    return code;
}

inline int ou_check_launch(const char* what)
{
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ou_fail(-100, "%s: launch failed: %s", what, hipGetErrorString(e));
    return 0;
}

#define OU_HIP_CHECK(expr, what)                                                        \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess) return ou_fail(-100, "%s: %s", what, hipGetErrorString(_e)); \
    } while (0)
