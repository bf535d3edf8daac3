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

// LDS-DMA of one dword per lane: lane l's *src lands at dst + 4 l (dst is
// wave-uniform).  Ordered for this wave's ds_reads only by a covering vmcnt:
// OU_WAIT_VMCNT0.  Issued from inline asm on purpose: hipcc (ROCm 7.2) cannot
// tell an LDS-DMA from the kernel's other LDS traffic and drains vmcnt(0)
// before the next ds_read (here: the MFMA fragment reads right after the
// prefetch), which would expose the DMA latency the prefetch exists to hide.
// The asm is invisible to the compiler's counters, so a kernel using it must
// not rely on compiler-inserted vmcnt waits for other vector loads issued
// after it (the MFMA waves of conv_wkernel issue none).
__device__ __forceinline__ void ou_glds4(const void* src, const void* lds_dst)
{
    const unsigned m0v = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(m0v)
                 : "memory");
}
__device__ __forceinline__ void ou_glds16(const void* src, const void* lds_dst)
{
    const unsigned m0v = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(m0v)
                 : "memory");
}
// Buffer-resource LDS-DMA (range-checked: an out-of-range voffset lands 0):
// lane l's dword / 16 bytes at voff + soff land at LDS byte address
// lds_addr + 4 l / 16 l.  soff and lds_addr are wave-uniform (SGPRs), so the
// per-piece address arithmetic stays on the scalar unit.
__device__ __forceinline__ void ou_blds4(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff, unsigned lds_addr)
{
    soff = __builtin_amdgcn_readfirstlane(soff);          // wave-uniform by contract
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dword %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(rs), "s"(soff), "s"(lds_addr)
                 : "memory");
}
__device__ __forceinline__ void ou_blds16(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff, unsigned lds_addr)
{
    soff = __builtin_amdgcn_readfirstlane(soff);          // wave-uniform by contract
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(rs), "s"(soff), "s"(lds_addr)
                 : "memory");
}
// LDS byte address of a pointer into the kernel's dynamic LDS (wave-uniform)
typedef unsigned ou_ldsa_t;
#define OU_LDS_ADDR(p) __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)(const void*)(p))
#define OU_GLDS4(src, dst) ou_glds4((const void*)(src), (const void*)(dst))
#define OU_GLDS16(src, dst) ou_glds16((const void*)(src), (const void*)(dst))
// Kernel-argument prefetch: one scalar load per 64-B line of the kernarg
// segment (the explicit descriptor and the hidden block counts after it), all
// issued before one wait.  The compiler loads the descriptor's fields where
// they are first used, behind branches and arithmetic, so a kernel's start
// otherwise pays a chain of dependent scalar-cache misses on the same few
// lines; afterwards every field load hits the scalar cache.  Reads only.
__device__ __forceinline__ void ou_kernarg_prefetch6()
{
    const auto kp = __builtin_amdgcn_kernarg_segment_ptr();
    unsigned a, b, c, d, e, f;
    asm volatile("s_load_dword %0, %[kp], 0x0\n\t"
                 "s_load_dword %1, %[kp], 0x40\n\t"
                 "s_load_dword %2, %[kp], 0x80\n\t"
                 "s_load_dword %3, %[kp], 0xc0\n\t"
                 "s_load_dword %4, %[kp], 0x100\n\t"
                 "s_load_dword %5, %[kp], 0x140\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b), "=&s"(c), "=&s"(d), "=&s"(e), "=&s"(f)
                 : [kp] "s"(kp)
                 : "memory");
}
__device__ __forceinline__ void ou_kernarg_prefetch8()
{
    const auto kp = __builtin_amdgcn_kernarg_segment_ptr();
    unsigned a, b, c, d, e, f, g, h;
    asm volatile("s_load_dword %0, %[kp], 0x0\n\t"
                 "s_load_dword %1, %[kp], 0x40\n\t"
                 "s_load_dword %2, %[kp], 0x80\n\t"
                 "s_load_dword %3, %[kp], 0xc0\n\t"
                 "s_load_dword %4, %[kp], 0x100\n\t"
                 "s_load_dword %5, %[kp], 0x140\n\t"
                 "s_load_dword %6, %[kp], 0x180\n\t"
                 "s_load_dword %7, %[kp], 0x1c0\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b), "=&s"(c), "=&s"(d), "=&s"(e), "=&s"(f), "=&s"(g), "=&s"(h)
                 : [kp] "s"(kp)
                 : "memory");
}
// A wave reads LDS rows its own lanes just stored: in hardware the wave's
// LDS instructions run in order (nothing to do); the CPU fiber emulator runs
// lanes one after another and needs a rendezvous here (tests/emu).
#define OU_WAVE_SYNC() do { } while (0)
#define OU_WAIT_VMCNT0() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#define OU_WAIT_VMCNT(n) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory")
#endif

// Range flag of a split-f16 operand.  omax: the running max |staged value|
// of a lane (fmaxf: a NaN input is skipped).  Sets bit `big` when a finite
// value reached 2^15 (this operand's exponent is too small: the host widens
// it) and bit 4 when a value was infinite (an overflow upstream propagating).
#define OU_RANGE_FINITE_MAX 3.4028235e38f
// Bits 8-10 say how far: set when a finite value reached 2^23 / 2^31 / 2^39,
// i.e. the exponent needs 2 / 3 / 4 steps of 8 (a thermometer code, so the
// OR over waves keeps the largest).
__device__ __forceinline__ void ou_range_flag(int* status, float omax, int big, int lane)
{
    if (__any(omax >= 32768.f) && status) {
        const bool fin = omax >= 32768.f && omax <= OU_RANGE_FINITE_MAX;
        const int code = (__any(fin) ? big : 0) | (__any(omax > OU_RANGE_FINITE_MAX) ? 4 : 0) |
                         (__any(fin && omax >= 8388608.f) ? 256 : 0) |          // 2^23
                         (__any(fin && omax >= 2147483648.f) ? 512 : 0) |       // 2^31
                         (__any(fin && omax >= 549755813888.f) ? 1024 : 0);     // 2^39
        if (lane == 0) atomicOr(status, code);
    }
}

// 2^e for |e| <= 126 (exact: the exponent field)
__device__ __forceinline__ float ou_exp2i(int e)
{
    return __uint_as_float((unsigned)(127 + e) << 23);
}

// Split-image store (include/ouhip.h, ou_conv_desc.sy): 4 consecutive
// channels of one sample, p = prelu_slope(v) * scale split into f16 hi (8 B at
// byte `off` of `rs`) and lo (8 B at off + 64).  `off` is the sentinel for
// elements that are not stored; omax tracks max |p| of the stored ones.
typedef _Float16 ou_h4_t __attribute__((ext_vector_type(4)));
typedef uint32_t ou_u2_t __attribute__((ext_vector_type(2)));
typedef uint32_t ou_u4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ou_split_store4(__amdgpu_buffer_rsrc_t rs, int off, bool ok, float v0, float v1,
                                                float v2, float v3, float scale, float slope, float& omax)
{
    float p[4] = {v0 * scale, v1 * scale, v2 * scale, v3 * scale};
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = p[j] >= 0.f ? p[j] : p[j] * slope;
    const ou_h4_t hi = {(_Float16)p[0], (_Float16)p[1], (_Float16)p[2], (_Float16)p[3]};
    const ou_h4_t lo = {(_Float16)((p[0] - (float)hi[0]) * 2048.f), (_Float16)((p[1] - (float)hi[1]) * 2048.f),
                        (_Float16)((p[2] - (float)hi[2]) * 2048.f), (_Float16)((p[3] - (float)hi[3]) * 2048.f)};
    const float m = fmaxf(fmaxf(fabsf(p[0]), fabsf(p[1])), fmaxf(fabsf(p[2]), fabsf(p[3])));
    omax = fmaxf(omax, ok ? m : 0.f);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(ou_u2_t, hi), rs, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(ou_u2_t, lo), rs, off, 64, 0);
}

// XCD-aware workgroup order (speed only, never correctness).  Workgroups
// are dealt round-robin over the 8 XCDs, so the neighbouring workgroups that
// share a weight panel (the N tiles of one m-group) land on 8 different L2s
// and every XCD fetches every panel.  ou_xcd_block maps the dispatch index to
// a logical one -- each set of workgroups that share an XCD gets a contiguous
// logical range, bijective for any grid size -- and returns the logical
// (x, y, z) block, x fastest.  OU_NO_XCD_ORDER builds the identity (A/B runs).
__device__ __forceinline__ void ou_xcd_block(int& bx, int& by, int& bz)
{
    const int gx = (int)gridDim.x, gy = (int)gridDim.y;
#ifdef OU_NO_XCD_ORDER
    bx = (int)blockIdx.x, by = (int)blockIdx.y, bz = (int)blockIdx.z;
#else
    const int n = gx * gy * (int)gridDim.z;
    const int p = (int)blockIdx.x + gx * ((int)blockIdx.y + gy * (int)blockIdx.z);
    const int x = p & 7, k = p >> 3, q = n >> 3, r = n & 7;
    const int l = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
    bx = l % gx;
    by = (l / gx) % gy;
    bz = l / (gx * gy);
#endif
}

// The same bijection with y (the m-groups of a conv) fastest: the workgroups
// that read one input window (all its m-groups) run back to back on one XCD,
// so the window is fetched from HBM once and re-read from that XCD's L2 --
// for inputs far larger than the weights (batched, long signals), where the
// x-fastest order re-reads every window once per m-group from HBM.
__device__ __forceinline__ void ou_xcd_block_m(int& bx, int& by, int& bz)
{
    const int gx = (int)gridDim.x, gy = (int)gridDim.y;
    const int n = gx * gy * (int)gridDim.z;
    const int p = (int)blockIdx.x + gx * ((int)blockIdx.y + gy * (int)blockIdx.z);
    const int x = p & 7, k = p >> 3, q = n >> 3, r = n & 7;
    const int l = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
    by = l % gy;
    bx = (l / gy) % gx;
    bz = l / (gx * gy);
}

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
