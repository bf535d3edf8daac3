// Host emulation shim for bounds-checking ouhip kernels on the CPU (test
// infrastructure only; never part of the product build).
//
// The kernel source is compiled for the host with this header in place of
// the HIP runtime.  Every thread of every (sampled) workgroup runs to
// completion one after another: __syncthreads() is a no-op, LDS is an exact-
// size heap block, MFMAs leave the accumulator unchanged, and the raw buffer
// builtins are range-checked loads/stores.  Built with AddressSanitizer, any
// access outside an allocation aborts with its location.  The values computed
// are meaningless -- only the addresses are checked.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__

using std::max;
using std::min;

struct dim3 {
    unsigned x, y, z;
    dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
struct emu_idx {
    unsigned x = 0, y = 0, z = 0;
};
inline emu_idx threadIdx, blockIdx;
inline dim3 gridDim, blockDim;

struct float4 {
    float x, y, z, w;
    float& operator[](int i) { return (&x)[i]; }
    const float& operator[](int i) const { return (&x)[i]; }
};
inline float4 make_float4(float a, float b, float c, float d) { return {a, b, c, d}; }
// IEEE round-to-nearest arithmetic (the host's default mode)
// v_mul_i32_i24: signed 24-bit operands, low 32 bits of the product
inline int __mul24(int a, int b)
{
    const long long sa = (long long)(a << 8) >> 8, sb = (long long)(b << 8) >> 8;
    return (int)(sa * sb);
}
inline float __fadd_rn(float a, float b) { return a + b; }
inline float __fsub_rn(float a, float b) { return a - b; }
inline float __fmul_rn(float a, float b) { return a * b; }
inline float __fdiv_rn(float a, float b) { return a / b; }
inline float __uint_as_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline uint32_t __float_as_uint(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
#ifdef OU_EMU_FIBERS
void emu_barrier();
void emu_wave_sync();
inline void __syncthreads() { emu_barrier(); }
#else
inline void __syncthreads() {}
inline void emu_wave_sync() {}
#endif

typedef int hipError_t;
typedef void* hipStream_t;
constexpr hipError_t hipSuccess = 0;
enum { hipFuncAttributeMaxDynamicSharedMemorySize = 8 };
inline hipError_t hipGetLastError() { return hipSuccess; }
inline const char* hipGetErrorString(hipError_t) { return "emu"; }
inline hipError_t hipFuncSetAttribute(const void*, int, int) { return hipSuccess; }
inline hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
enum { hipDeviceAttributeSharedMemPerBlockOptin = 74, hipDeviceAttributeMultiprocessorCount = 63 };
// a few "CUs" (OUHIP_EMU_CUS, default 3) so persistent kernels walk several tiles
inline hipError_t hipDeviceGetAttribute(int* v, int attr, int)
{
    if (attr == hipDeviceAttributeMultiprocessorCount) {
        const char* e = std::getenv("OUHIP_EMU_CUS");
        *v = e ? std::atoi(e) : 3;
    } else {
        *v = 163840;
    }
    return hipSuccess;
}
template <typename K>
inline hipError_t hipOccupancyMaxActiveBlocksPerMultiprocessor(int* n, K, int, size_t) { *n = 1; return hipSuccess; }
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) { std::memset(p, v, n); return hipSuccess; }
#define HIP_SYMBOL(x) (&(x))
// wave vote / atomics: lanes run one after another here, so a vote sees only
// the calling lane (used by the split-f16 range flag, never taken in tests)
inline bool __any(bool p) { return p; }
inline bool __all(bool p) { return p; }
inline int atomicOr(int* p, int v) { const int o = *p; *p |= v; return o; }
inline unsigned atomicMax(unsigned* p, unsigned v) { const unsigned o = *p; *p = o > v ? o : v; return o; }
inline float __shfl_xor(float v, int) { return v; }

// ---- buffer resources ----------------------------------------------------
struct emu_rsrc {
    const char* base;
    uint32_t size;
};
#define __amdgpu_buffer_rsrc_t emu_rsrc
inline emu_rsrc emu_make_rsrc(const void* p, short, int n, int) { return {(const char*)p, (uint32_t)n}; }
#define __builtin_amdgcn_make_buffer_rsrc(p, s, n, f) emu_make_rsrc((const void*)(p), s, n, f)

inline bool emu_in_range(const emu_rsrc& r, uint32_t voff, uint32_t soff, uint32_t nbytes, const char* what)
{
    if (voff >= r.size) return false;   // hardware range check: dropped / reads 0
    if ((uint64_t)voff + soff + nbytes > (uint64_t)r.size) {
        // the hardware checks voffset only: this access would go past the
        // resource (and possibly past the allocation)
        std::fprintf(stderr, "EMU: %s voffset %u + soffset %u + %u > resource size %u\n", what, voff, soff,
                     nbytes, r.size);
        std::abort();
    }
    return true;
}
inline uint32_t emu_load_b32(emu_rsrc r, int voff, int soff, int)
{
    if (!emu_in_range(r, (uint32_t)voff, (uint32_t)soff, 4, "load_b32")) return 0;
    uint32_t v;
    std::memcpy(&v, r.base + (uint32_t)voff + (uint32_t)soff, 4);
    return v;
}
typedef uint32_t emu_u4 __attribute__((ext_vector_type(4)));
inline emu_u4 emu_load_b128(emu_rsrc r, int voff, int soff, int)
{
    emu_u4 v = {0, 0, 0, 0};
    if (!emu_in_range(r, (uint32_t)voff, (uint32_t)soff, 16, "load_b128")) return v;
    std::memcpy(&v, r.base + (uint32_t)voff + (uint32_t)soff, 16);
    return v;
}
inline void emu_store_b32(uint32_t v, emu_rsrc r, int voff, int soff, int)
{
    if (!emu_in_range(r, (uint32_t)voff, (uint32_t)soff, 4, "store_b32")) return;
    std::memcpy((char*)r.base + (uint32_t)voff + (uint32_t)soff, &v, 4);
}
inline void emu_store_b128(emu_u4 v, emu_rsrc r, int voff, int soff, int)
{
    if (!emu_in_range(r, (uint32_t)voff, (uint32_t)soff, 16, "store_b128")) return;
    std::memcpy((char*)r.base + (uint32_t)voff + (uint32_t)soff, &v, 16);
}
typedef uint32_t emu_u2 __attribute__((ext_vector_type(2)));
inline emu_u2 emu_load_b64(emu_rsrc r, int voff, int soff, int)
{
    emu_u2 v = {0, 0};
    if (!emu_in_range(r, (uint32_t)voff, (uint32_t)soff, 8, "load_b64")) return v;
    std::memcpy(&v, r.base + (uint32_t)voff + (uint32_t)soff, 8);
    return v;
}
inline void emu_store_b64(emu_u2 v, emu_rsrc r, int voff, int soff, int)
{
    if (!emu_in_range(r, (uint32_t)voff, (uint32_t)soff, 8, "store_b64")) return;
    std::memcpy((char*)r.base + (uint32_t)voff + (uint32_t)soff, &v, 8);
}
#define __builtin_amdgcn_raw_buffer_load_b64 emu_load_b64
#define __builtin_amdgcn_raw_buffer_store_b64 emu_store_b64
#define __builtin_amdgcn_raw_buffer_store_b128 emu_store_b128
#define __builtin_amdgcn_readfirstlane(x) (x)
#define __builtin_amdgcn_s_waitcnt(x) ((void)0)
#define __builtin_amdgcn_raw_buffer_load_b32 emu_load_b32
#define __builtin_amdgcn_raw_buffer_load_b128 emu_load_b128
#define __builtin_amdgcn_raw_buffer_store_b32 emu_store_b32

typedef float emu_f16v __attribute__((ext_vector_type(16)));
#ifdef OU_EMU_FIBERS
emu_f16v emu_mfma(float a, float b, emu_f16v c, int, int, int);
#else
inline emu_f16v emu_mfma(float, float, emu_f16v c, int, int, int) { return c; }
#endif
#define __builtin_amdgcn_mfma_f32_32x32x2f32 emu_mfma
typedef _Float16 emu_h8 __attribute__((ext_vector_type(8)));
#ifdef OU_EMU_FIBERS
emu_f16v emu_mfma16(emu_h8 a, emu_h8 b, emu_f16v c, int, int, int);
#else
inline emu_f16v emu_mfma16(emu_h8, emu_h8, emu_f16v c, int, int, int) { return c; }
#endif
#define __builtin_amdgcn_mfma_f32_32x32x16_f16 emu_mfma16

// ---- dynamic LDS: an exact-size heap block per workgroup ------------------
inline void* emu_lds_ptr = nullptr;
#define OU_DYNAMIC_LDS(T, name) T* name = (T*)emu_lds_ptr

// ---- launches -------------------------------------------------------------
// OUHIP_EMU_BLOCKS: how many workgroups to run per launch (first, last and an
// even spread between); 0 = all.
inline int emu_block_budget()
{
    const char* e = std::getenv("OUHIP_EMU_BLOCKS");
    return e ? std::atoi(e) : 6;
}
#ifndef OU_EMU_FIBERS
template <typename K, typename... A>
inline void emu_launch(K kern, dim3 grid, dim3 block, size_t lds, hipStream_t, A... args)
{
    gridDim = grid;
    blockDim = block;
    const long nb = (long)grid.x * grid.y * grid.z;
    std::vector<long> ids;
    const int budget = emu_block_budget();
    if (budget <= 0 || nb <= budget) {
        for (long i = 0; i < nb; ++i) ids.push_back(i);
    } else {
        for (int i = 0; i < budget; ++i) ids.push_back(i * (nb - 1) / (budget - 1));
    }
    for (long id : ids) {
        blockIdx.x = id % grid.x;
        blockIdx.y = (id / grid.x) % grid.y;
        blockIdx.z = id / ((long)grid.x * grid.y);
        emu_lds_ptr = lds ? std::malloc(lds) : nullptr;
        for (unsigned t = 0; t < block.x; ++t) {
            threadIdx.x = t;
            kern(args...);
        }
        std::free(emu_lds_ptr);
        emu_lds_ptr = nullptr;
    }
}
#else
// ---- fiber mode: all threads of a workgroup interleave at barriers and
// MFMAs, so LDS sharing and the cross-lane MFMA give real values ----------
#include <ucontext.h>
#include <functional>
struct emu_fiber {
    ucontext_t ctx;
    std::vector<char> stack;
    int state = 0;   // 0 runnable, 1 at barrier, 2 at mfma, 3 done, 4 at a wave-level wait
    float a = 0, b = 0;
    float a8[8] = {}, b8[8] = {};   // v_mfma_f32_32x32x16_f16 operands
    int k16 = 0;
    emu_f16v c;
};
struct emu_block_state {
    std::vector<emu_fiber> f;
    ucontext_t sched;
    int cur = -1;
    std::function<void()> body;
};
inline emu_block_state* emu_bs = nullptr;
inline void emu_fiber_entry()
{
    emu_bs->body();
    emu_bs->f[emu_bs->cur].state = 3;
    swapcontext(&emu_bs->f[emu_bs->cur].ctx, &emu_bs->sched);
}
// s_waitcnt on LDS-DMA: the wave's 64 lanes issued the DMA as ONE instruction,
// so after the wait every lane sees every lane's slots -- a wave rendezvous
inline void emu_wave_sync()
{
    emu_fiber& me = emu_bs->f[emu_bs->cur];
    me.state = 4;
    swapcontext(&me.ctx, &emu_bs->sched);
}
inline void emu_barrier()
{
    emu_fiber& me = emu_bs->f[emu_bs->cur];
    me.state = 1;
    swapcontext(&me.ctx, &emu_bs->sched);
}
// v_mfma_f32_32x32x2_f32: lane l supplies A[l&31][l>>5], B[l>>5][l&31] and
// C/D rows (r&3) + 8(r>>2) + 4(l>>5), column l&31.
inline emu_f16v emu_mfma(float a, float b, emu_f16v c, int, int, int)
{
    emu_fiber& me = emu_bs->f[emu_bs->cur];
    me.a = a;
    me.b = b;
    me.c = c;
    me.k16 = 0;
    me.state = 2;
    swapcontext(&me.ctx, &emu_bs->sched);
    return me.c;
}
// v_mfma_f32_32x32x16_f16: lane l supplies A[l&31][8(l>>5) + j] and
// B[8(l>>5) + j][l&31] in element j; f16 products are exact in f32
inline emu_f16v emu_mfma16(emu_h8 a, emu_h8 b, emu_f16v c, int, int, int)
{
    emu_fiber& me = emu_bs->f[emu_bs->cur];
    for (int j = 0; j < 8; ++j) {
        me.a8[j] = (float)a[j];
        me.b8[j] = (float)b[j];
    }
    me.c = c;
    me.k16 = 1;
    me.state = 2;
    swapcontext(&me.ctx, &emu_bs->sched);
    return me.c;
}
inline void emu_do_mfma(int wave)
{
    emu_fiber* L = &emu_bs->f[wave * 64];
    if (L[0].k16) {
        float A16[32][16], B16[16][32];
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j) {
                A16[l & 31][8 * (l >> 5) + j] = L[l].a8[j];
                B16[8 * (l >> 5) + j][l & 31] = L[l].b8[j];
            }
        for (int l = 0; l < 64; ++l) {
            emu_f16v d = L[l].c;
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
                float acc = d[r];
                for (int k = 0; k < 16; ++k) acc = std::fma(A16[row][k], B16[k][col], acc);
                d[r] = acc;
            }
            L[l].c = d;
            L[l].state = 0;
        }
        return;
    }
    float A[32][2], B[2][32];
    for (int l = 0; l < 64; ++l) {
        A[l & 31][l >> 5] = L[l].a;
        B[l >> 5][l & 31] = L[l].b;
    }
    for (int l = 0; l < 64; ++l) {
        emu_f16v d = L[l].c;
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
            float acc = d[r];
            acc = std::fma(A[row][0], B[0][col], acc);   // exact fp32 FMA chain, k = 0 then 1
            acc = std::fma(A[row][1], B[1][col], acc);
            d[r] = acc;
        }
        L[l].c = d;
        L[l].state = 0;
    }
}
template <typename K, typename... A>
inline void emu_launch(K kern, dim3 grid, dim3 block, size_t lds, hipStream_t, A... args)
{
    gridDim = grid;
    blockDim = block;
    const long nb = (long)grid.x * grid.y * grid.z;
    const int nt = block.x;
    for (long id = 0; id < nb; ++id) {
        blockIdx.x = id % grid.x;
        blockIdx.y = (id / grid.x) % grid.y;
        blockIdx.z = id / ((long)grid.x * grid.y);
        emu_lds_ptr = lds ? std::calloc(lds, 1) : nullptr;
        emu_block_state bs;
        emu_bs = &bs;
        bs.f.resize(nt);
        bs.body = [&]() { kern(args...); };
        for (int t = 0; t < nt; ++t) {
            emu_fiber& f = bs.f[t];
            f.stack.resize(256 * 1024);
            getcontext(&f.ctx);
            f.ctx.uc_stack.ss_sp = f.stack.data();
            f.ctx.uc_stack.ss_size = f.stack.size();
            f.ctx.uc_link = nullptr;
            makecontext(&f.ctx, emu_fiber_entry, 0);
        }
        while (true) {
            bool progressed = false;
            for (int t = 0; t < nt; ++t) {
                if (bs.f[t].state != 0) continue;
                bs.cur = t;
                threadIdx.x = t;
                swapcontext(&bs.sched, &bs.f[t].ctx);
                progressed = true;
            }
            // waves whose live lanes all wait at a wave-level wait continue together
            for (int w = 0; w * 64 < nt; ++w) {
                bool all = true, any = false;
                for (int l = 0; l < 64; ++l) {
                    const int st = bs.f[w * 64 + l].state;
                    all &= st == 4 || st == 3;
                    any |= st == 4;
                }
                if (all && any) {
                    for (int l = 0; l < 64; ++l)
                        if (bs.f[w * 64 + l].state == 4) bs.f[w * 64 + l].state = 0;
                    progressed = true;
                }
            }
            // waves whose 64 lanes all wait at an MFMA execute it
            for (int w = 0; w * 64 < nt; ++w) {
                bool all = true, any = false;
                for (int l = 0; l < 64; ++l) {
                    all &= bs.f[w * 64 + l].state == 2;
                    any |= bs.f[w * 64 + l].state == 2;
                }
                if (all) {
                    emu_do_mfma(w);
                    progressed = true;
                } else if (any) {
                    bool other = false;   // some lanes at the MFMA, others elsewhere: divergent MFMA
                    for (int l = 0; l < 64; ++l) other |= bs.f[w * 64 + l].state == 0;
                    (void)other;
                }
            }
            int live = 0, at_bar = 0;
            for (auto& f : bs.f) {
                live += f.state != 3;
                at_bar += f.state == 1;
            }
            if (live == 0) break;
            if (!progressed) {
                if (at_bar == live) {
                    for (auto& f : bs.f)
                        if (f.state == 1) f.state = 0;
                } else {
                    std::fprintf(stderr, "EMU: deadlock (live %d, at barrier %d)\n", live, at_bar);
                    std::abort();
                }
            }
        }
        std::free(emu_lds_ptr);
        emu_lds_ptr = nullptr;
        emu_bs = nullptr;
    }
}
#endif
#define hipLaunchKernelGGL(kern, grid, block, lds, stream, ...) emu_launch(kern, grid, block, lds, stream, __VA_ARGS__)

// LDS-DMA (ou_common.h OU_GLDS4): lane l's dword lands at dst + 4 l
#define OU_GLDS4(src, dst) std::memcpy((char*)(dst) + 4 * (threadIdx.x & 63), (const void*)(src), 4)
#define OU_GLDS16(src, dst) std::memcpy((char*)(dst) + 16 * (threadIdx.x & 63), (const void*)(src), 16)
// buffer LDS-DMA: lds_addr is the host address of the LDS block here (OU_LDS_ADDR)
inline void emu_blds(emu_rsrc r, unsigned voff, unsigned soff, uintptr_t lds, int size)
{
    char* dst = (char*)lds + size * (threadIdx.x & 63);
    if (!emu_in_range(r, voff, soff, size, "blds")) { std::memset(dst, 0, size); return; }
    std::memcpy(dst, r.base + voff + soff, size);
}
#define ou_blds4(r, v, s, l) emu_blds((r), (v), (s), (l), 4)
#define ou_blds16(r, v, s, l) emu_blds((r), (v), (s), (l), 16)
typedef uintptr_t ou_ldsa_t;
#define OU_LDS_ADDR(p) ((uintptr_t)(const void*)(p))
inline void ou_kernarg_prefetch6() {}
inline void ou_kernarg_prefetch8() {}
#define OU_WAIT_VMCNT0() emu_wave_sync()
#define OU_WAIT_VMCNT(n) emu_wave_sync()
#define OU_WAVE_SYNC() emu_wave_sync()

// the product's uniform-resource helper (ou_common.h), host version
inline emu_rsrc ou_rsrc(const void* p, long long bytes)
{
    return {(const char*)p, (uint32_t)(bytes < 0 ? 0 : bytes > 0x7fffffffLL ? 0x7fffffffLL : bytes)};
}
#define OU_EMU 1
