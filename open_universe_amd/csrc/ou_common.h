// ou_common.h -- shared host helpers for the ouhip C ABI (error reporting).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

// Raw buffer resource over [p, p + bytes) (bytes clamped to 2^31 - 1), with
// every word forced uniform: readfirstlane keeps the resource in SGPRs even
// when its inputs were computed on the VALU -- a resource in VGPRs makes the
// compiler wrap every load/store that uses it in a waterfall loop.  Offsets
// at or past `bytes` read 0 / are dropped (the range check covers the
// voffset only, never the soffset).
#ifndef OU_EMU
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ou_rsrc(const void* p, long long bytes)
{
    const unsigned long long a = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0 ? 0 : bytes > 0x7fffffffLL ? 0x7fffffffLL : bytes));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, n,
                                             0x00020000);
}
#endif

// dynamic LDS of a kernel (tests/emu replaces it with a bounds-checked block)
#ifndef OU_DYNAMIC_LDS
#define OU_DYNAMIC_LDS(T, name) extern __shared__ T name[]
#endif

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
