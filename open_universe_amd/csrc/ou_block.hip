// ou_block.hip -- fused ConvBlock main path for channel-complete workgroups
// (gfx950 / MI355X).
//
// Replaces the three PReLU_Conv calls of one ConvBlock and the arithmetic
// between them (networks/universe/blocks.py:393-416):
//   c1 = conv1(h)                            k5, PReLU on its input
//   c1 = (c1 + input_cond) * s_sc            (score decoder, optional)
//   c1 = film(c1)                            (gamma * c1 + beta, optional)
//   cond_out = c1                            (conditioner decoder, optional store)
//   c2 = conv2(c1)                           k3
//   c3 = conv3(c2)                           k3
//   y  = ((h + c3) * s_res [+ res2]) * s2
// in ONE launch instead of three.  A workgroup owns F = 32*NT - 4 output
// frames of every channel: it stages PReLU(h) over its frames plus a 4-frame
// halo on each side (2 + 1 + 1 taps of the three convs) in LDS, computes
// conv1 over F + 4 frames, conv2 over F + 2 and conv3 over F, each into LDS,
// and writes only y (and cond_out) to HBM.  The intermediates never leave
// the CU: per block the HBM traffic drops from 3 reads + 3 writes (+ the
// residual re-read) of a C x T tensor to 1 read + 1 write, and 3 kernel
// latencies become 1.  Halo frames are recomputed by the neighbouring
// workgroup (F = 124 / 60 / 28 frames at C = 32 / 64 / 128; 124 / 60 at
// PP24's 96 / 192).
//
// Arithmetic is the split-f16 form of ou_conv (P = 1): every operand is
// v = hi + lo * 2^-11 (f16 halves; weights packed by ou_block_pack with a
// per-conv power-of-two scale, activations split while they are written to
// LDS, staged as x * 2^-6) and a product is ha hb + (ha lb + la hb) 2^-11 on
// v_mfma_f32_32x32x16_f16 with f32 accumulation -- f32-class accuracy.  P = 2
// is plain f16 (hi halves only).  A staged |x| >= 2^21 sets *status (the
// host reruns the enhance with f32 operands), exactly as ou_conv does.
//
// Frames outside [0, T) are the zero padding of each conv's input ('same'
// convs pad their PReLU'd input with zeros), so the conv1/conv2 results are
// zeroed there before they become the next conv's input.
//
// MFMA mapping: 4 waves as WM x WN; wave (wm, wn) owns MR x NR 32 x 32 output
// tiles (rows = channels, columns = frames).  A fragments (weights) stream
// from global memory (L2-resident: every workgroup reads the same weights)
// through a 3-deep register ring; B fragments are one ds_read_b128 of 8
// consecutive channels of one frame row.  LDS rows are [frame][channel] with
// a stride of C + 8 halves (an odd number of 16-B slots: conflict-free).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>
#include <vector>

#include "../../include/ouhip.h"
#include "ou_common.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

namespace {

constexpr int kStageShift = 6;   // the exponent ou_block_pack's w_unscale assumes (ou_conv's kSplitShift)


#ifndef OU_BLOCK_NT32
#define OU_BLOCK_NT32 4
#endif
#ifndef OU_BLOCK_NT64
#define OU_BLOCK_NT64 2
#endif
#ifndef OU_BLOCK_NT128
#define OU_BLOCK_NT128 1
#endif
#ifndef OU_BLOCK_NT48
#define OU_BLOCK_NT48 4    // PP24 level 0 (2 x 2 waves, rows padded to 64)
#endif
#ifndef OU_BLOCK_NT96
#define OU_BLOCK_NT96 4    // PP24 level 1 (a multiple of its 4 waves along N)
#endif
#ifndef OU_BLOCK_NT192
#define OU_BLOCK_NT192 2   // PP24 level 2 (2 x 2 waves)
#endif
#ifndef OU_BLOCK_RING1
#define OU_BLOCK_RING1 6   // weight-fragment ring depth (k-steps) of one-m-tile waves
#endif
#ifndef OU_BLOCK_FENCE
#define OU_BLOCK_FENCE 1   // pin each ring load ahead of the step's LDS reads (128 ch: 36.6 -> 32.7 us)
#endif
#ifndef OU_BLOCK_BPIPE
#define OU_BLOCK_BPIPE 1   // LDS B fragments read one k-step ahead of their MFMAs
#endif
#ifndef OU_BLOCK_RING_EARLY
#define OU_BLOCK_RING_EARLY 0   // 1: issue a stage's first weight fragments before the previous stage's epilogue (measured slower in the C2 bench: profiles/bench_ab_ring_mel_r03n.txt)
#endif
#ifndef OU_BLOCK_HV_EARLY
#define OU_BLOCK_HV_EARLY 0   // load the block residual before the conv3 MFMA stage
#endif

template <int C, int NT, int P>
struct BCfg {
    static constexpr int MT = (C + 31) / 32;       // 32-row M tiles (output channels; 48: rows 48-63
                                                   // are zero-weight padding, computed, never stored)
    static constexpr int WAVES = 4;                // waves per workgroup (block_threads() must agree;
                                                   // 8 waves at C = 256 measured slower: 64 vs 53 us)
    static constexpr int NTH = 64 * WAVES;
    // waves along M: the largest of 4 / 2 / 1 that divides the M tiles
    // (96 channels: 1 x 4 waves, 3 M tiles each; 192: 2 x 2, 3 each)
    static constexpr int WM = MT % WAVES == 0 ? WAVES : MT % 2 == 0 ? 2 : 1;
    static constexpr int WN = WAVES / WM;          // waves along N (frames)
    static constexpr int MR = MT / WM;             // M tiles per wave
    static constexpr int NR = NT / WN;             // N tiles per wave
    static constexpr int NF = 32 * NT;             // frames of one conv stage
    static constexpr int F = NF - 4;               // output frames per workgroup
    // LDS element: f16 halves (split-f16 hi | lo planes, f16), f32 (prec 0)
    using E = std::conditional_t<P == 0, float, _Float16>;
    // row stride in elements, an odd number of 16-B slots (conflict-free
    // 16-B reads of 32 consecutive rows)
    static constexpr int SX = P == 0 ? C + 4 : C + 8;
    static constexpr int R1 = NF + 4;              // conv1 input rows (frames t0-4 ..)
    static constexpr int R2 = NF + 2;              // conv2 / conv3 input rows
    static constexpr int NPL = P == 1 ? 2 : 1;     // planes: hi (+ lo)
    static constexpr int PA = R1 * SX;             // plane stride of region A (elements)
    static constexpr int PB = R2 * SX;             // plane stride of region B
    static constexpr int A_OFF = 0;                // region A: conv1 input, then conv3 input
    static constexpr int B_OFF = NPL * PA;         // region B: conv2 input
    static constexpr int LDS_BYTES = (int)sizeof(E) * (NPL * PA + NPL * PB);
    static constexpr int KS = C / 16;              // 16-channel k-steps per tap
    static constexpr int RING = MR == 1 ? OU_BLOCK_RING1 : 4;   // weight-fragment ring depth (k-steps)
    static_assert(C % 16 == 0 && WM * WN == WAVES && MT % WM == 0 && NT % WN == 0, "block tiling");
    static_assert((SX * (int)sizeof(E) / 16) % 2 == 1 && (SX * (int)sizeof(E)) % 16 == 0,
                  "LDS row stride must be an odd number of 16-B slots");
};

__device__ __forceinline__ float prelu(float v, float a) { return v >= 0.f ? v : a * v; }

// One conv stage: acc[mr][nr] (+ accx for the split cross terms) over KT taps
// x C channels.  xin: LDS base of the stage's input (hi plane; lo plane at
// + pstride); wp: packed weights [mt][tap][ks][plane][lane][8].
// Weight-fragment ring of a split-f16 / f16 stage: step s's A fragments (hi |
// lo) of the wave's m-tiles.  ring_pro issues the first D - 1 steps of a
// stage; the kernel calls it for the NEXT stage before the current stage's
// epilogue and barrier (and for conv1 before the input staging), so the L2
// round trip of a stage's first fragments overlaps work instead of stalling
// the stage's first MFMAs (OU_BLOCK_RING_EARLY=0: at the stage start).
template <int KT, int C, int NT, int P>
__device__ __forceinline__ void ring_load(const half8_t* __restrict__ wp, int wm, int lane, int s,
                                          half8_t (&dst)[BCfg<C, NT, P>::MR][2])
{
    using K = BCfg<C, NT, P>;
    const int k = s / K::KS, ks = s - (s / K::KS) * K::KS;
#pragma unroll
    for (int mr = 0; mr < K::MR; ++mr) {
        const half8_t* p = wp + ((((int64_t)(wm * K::MR + mr) * KT + k) * K::KS + ks) * 2) * 64 + lane;
        dst[mr][0] = p[0];
        if constexpr (P == 1) dst[mr][1] = p[64];
    }
}
template <int KT, int C, int NT, int P>
__device__ __forceinline__ void ring_pro(const void* wp, int wm, int lane,
                                         half8_t (&ra)[BCfg<C, NT, P>::RING][BCfg<C, NT, P>::MR][2])
{
    using K = BCfg<C, NT, P>;
    constexpr int NS = KT * K::KS, D = NS < K::RING ? NS : K::RING;
#pragma unroll
    for (int s = 0; s < D - 1; ++s) ring_load<KT, C, NT, P>((const half8_t*)wp, wm, lane, s, ra[s]);
}

template <int KT, int C, int NT, int P>
__device__ __forceinline__ void stage_mma(const half8_t* __restrict__ wp, const _Float16* xin, int pstride, int wm,
                                          int wn, int lane, int dbg, floatx16 (&acc)[BCfg<C, NT, P>::MR][BCfg<C, NT, P>::NR],
                                          floatx16 (&accx)[BCfg<C, NT, P>::MR][BCfg<C, NT, P>::NR],
                                          half8_t (&ra)[BCfg<C, NT, P>::RING][BCfg<C, NT, P>::MR][2], bool pre)
{
    using K = BCfg<C, NT, P>;
    constexpr int MR = K::MR, NR = K::NR, KS = K::KS, NS = KT * KS;
    const int l32 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int mr = 0; mr < MR; ++mr)
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mr][nr][r] = 0.f, accx[mr][nr][r] = 0.f;
        }
    // weight fragments stream from L2 through a D-deep register ring: the
    // loads of step s + D - 1 are issued before the MFMAs of step s
    if (dbg & 2) return;   // diagnostics (tools/block_bench.py --dbg): no MFMA stage
    constexpr int D = NS < K::RING ? NS : K::RING;
    auto load_a = [&](int s, half8_t (&dst)[MR][2]) { ring_load<KT, C, NT, P>(wp, wm, lane, s, dst); };
    if (!pre) {
#pragma unroll
        for (int s = 0; s < D - 1; ++s) load_a(s, ra[s]);
    }
    const _Float16* xb = xin + (wn * NR * 32 + l32) * K::SX + 8 * h;
    // B fragments (LDS) one step ahead: step s + 1's reads are issued before
    // step s's MFMAs, so an MFMA never waits on the read that feeds it
    // (OU_BLOCK_BPIPE=0: read right before use)
    half8_t b[2][NR], bl[2][NR];
    auto load_b = [&](int s, half8_t (&bq)[NR], half8_t (&bo)[NR]) {
        const int k = s / KS, ks = s - (s / KS) * KS;
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
            const _Float16* q = xb + (nr * 32 + k) * K::SX + 16 * ks;
            bq[nr] = *(const half8_t*)q;
            if constexpr (P == 1) bo[nr] = *(const half8_t*)(q + pstride);
        }
    };
    if constexpr (OU_BLOCK_BPIPE) load_b(0, b[0], bl[0]);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (s + D - 1 < NS) load_a(s + D - 1, ra[(s + D - 1) % D]);
        const int c = OU_BLOCK_BPIPE ? (s & 1) : 0;
        if constexpr (OU_BLOCK_BPIPE) {
            if (s + 1 < NS) load_b(s + 1, b[c ^ 1], bl[c ^ 1]);
        } else {
            load_b(s, b[0], bl[0]);
        }
        // the fully unrolled loop otherwise lets the scheduler sink the ring
        // loads next to their use (2-3 steps of latency cover instead of D - 1)
        if constexpr (OU_BLOCK_FENCE) asm volatile("" ::: "memory");
#pragma unroll
        for (int mr = 0; mr < MR; ++mr)
#pragma unroll
            for (int nr = 0; nr < NR; ++nr) {
                acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s % D][mr][0], b[c][nr], acc[mr][nr], 0, 0, 0);
                if constexpr (P == 1) {
                    accx[mr][nr] =
                        __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s % D][mr][0], bl[c][nr], accx[mr][nr], 0, 0, 0);
                    accx[mr][nr] =
                        __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s % D][mr][1], b[c][nr], accx[mr][nr], 0, 0, 0);
                }
            }
    }
}

// The f32-operand form (prec 0) of one conv stage: v_mfma_f32_32x32x2_f32
// over KT taps x C / 2 channel pairs.  LDS rows hold f32 channels in
// pair-split order (even channels in the first half row, odd in the second:
// ch_pos), so lane half h reads channel 2s + h of 4 consecutive pair steps
// as one 16-B read; wp: ou_block_pack_f32, [mt][tap][s4][lane][4].
template <int C>
__device__ __forceinline__ int ch_pos(int c)
{
    return (c & 1) * (C / 2) + (c >> 1);
}

template <int KT, int C, int NT>
__device__ __forceinline__ void stage_mma_f32(const f32x4_t* __restrict__ wp, const float* xin, int wm, int wn,
                                              int lane, int dbg,
                                              floatx16 (&acc)[BCfg<C, NT, 0>::MR][BCfg<C, NT, 0>::NR])
{
    using K = BCfg<C, NT, 0>;
    constexpr int MR = K::MR, NR = K::NR, S4 = C / 8, NS = KT * S4;
    const int l32 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int mr = 0; mr < MR; ++mr)
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mr][nr][r] = 0.f;
        }
    if (dbg & 2) return;
    constexpr int D = NS < 4 ? NS : 4;
    f32x4_t ra[D][MR];
    auto load_a = [&](int s, f32x4_t (&dst)[MR]) {
        const int k = s / S4, s4 = s - (s / S4) * S4;
#pragma unroll
        for (int mr = 0; mr < MR; ++mr) dst[mr] = wp[(((int64_t)(wm * MR + mr) * KT + k) * S4 + s4) * 64 + lane];
    };
#pragma unroll
    for (int s = 0; s < D - 1; ++s) load_a(s, ra[s]);
    const float* xb = xin + (wn * NR * 32 + l32) * K::SX + h * (C / 2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (s + D - 1 < NS) load_a(s + D - 1, ra[(s + D - 1) % D]);
        if constexpr (OU_BLOCK_FENCE) asm volatile("" ::: "memory");
        const int k = s / S4, s4 = s - (s / S4) * S4;
        f32x4_t bq[NR];
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) bq[nr] = *(const f32x4_t*)(xb + (nr * 32 + k) * K::SX + 4 * s4);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                for (int nr = 0; nr < NR; ++nr)
                    acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[s % D][mr][j], bq[nr][j], acc[mr][nr], 0, 0, 0);
    }
}

// One conv stage on a wave's tiles: split-f16 / f16 (acc + the cross terms in
// accx) or f32 operands (accx stays zero).
template <int KT, int C, int NT, int P>
__device__ __forceinline__ void run_stage(const void* w, const typename BCfg<C, NT, P>::E* xin, int pstride, int wm,
                                          int wn, int lane, int dbg,
                                          floatx16 (&acc)[BCfg<C, NT, P>::MR][BCfg<C, NT, P>::NR],
                                          floatx16 (&accx)[BCfg<C, NT, P>::MR][BCfg<C, NT, P>::NR],
                                          half8_t (&ra)[BCfg<C, NT, P>::RING][BCfg<C, NT, P>::MR][2], bool pre)
{
    if constexpr (P == 0) {
        stage_mma_f32<KT, C, NT>((const f32x4_t*)w, xin, wm, wn, lane, dbg, acc);
#pragma unroll
        for (int mr = 0; mr < BCfg<C, NT, P>::MR; ++mr)
#pragma unroll
            for (int nr = 0; nr < BCfg<C, NT, P>::NR; ++nr) accx[mr][nr] = floatx16{};
    } else {
        stage_mma<KT, C, NT, P>((const half8_t*)w, xin, pstride, wm, wn, lane, dbg, acc, accx, ra, pre);
    }
}

// Epilogue variants (template EPI bits, so the per-element code has no
// run-time branches): the score encoder's FiLM, the score decoder's
// input_cond residual + FiLM, the conditioner decoder's cond_out store.
constexpr int kEpiFilm = 1, kEpiSc = 2, kEpiCond = 4, kEpiRes2 = 8;
// fusions at the score network's 32-channel ends: kEpiIn computes the block
// input h = input_conv(in_scale * x) (1 -> C channels, k3, score.py:244-246,285)
// instead of reading it; kEpiHead runs the score head (two PReLUs,
// output_conv C -> 1 k3, EDM wrapper and sampler update, as ou_head) on the
// block output instead of storing it.  With the head, conv3 covers one extra
// frame on each side (the head's taps), so a workgroup owns F - 2 frames.
constexpr int kEpiIn = 16, kEpiHead = 32;
// kEpiDown: the encoder's strided rate-change conv (blocks.py:203-231,268-275)
// as a fourth MFMA stage on the block output, which is still stored: e =
// conv(PReLU(y)), stride R, 2C rows, KF frames of R samples per output frame
// (KF = 3: the anti-alias FIR folded in, centred; KF = 1: plain).  conv3 then
// covers the conv's sample halo (R (KF-1)/2 on each side) and a workgroup owns
// a multiple of R frames.
constexpr int kEpiDown = 64;

// conv3 frames before t0 (the halo of whatever consumes the block output)
template <int EPI, int R, int KF>
constexpr int block_off()
{
    return (EPI & kEpiHead) ? 1 : (EPI & kEpiDown) ? R * ((KF - 1) / 2) : 0;
}

template <int C, int NT, int P, int EPI, int R = 1, int KF = 1>
constexpr int block_f()
{
    if constexpr (EPI & kEpiDown) {
        constexpr int halo = 2 * R * ((KF - 1) / 2);
        return (BCfg<C, NT, P>::NF - 4 - halo) / R * R;
    }
    return BCfg<C, NT, P>::NF - 4 - ((EPI & kEpiHead) ? 2 : 0);
}

typedef float float2_t __attribute__((ext_vector_type(2)));
// per-element fma on a pair: one v_pk_fma_f32, the same bits as two fmaf
__device__ __forceinline__ float2_t fma2(float2_t a, float2_t b, float2_t c) { return __builtin_elementwise_fma(a, b, c); }
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

// x (already scaled by the stage's 2^-shift) -> hi (+ lo) halves of 4
// consecutive channels; omax = max(omax, |x|) (the stage's range flag)
template <int P>
__device__ __forceinline__ void split4(float x0, float x1, float x2, float x3, half4_t& hi, half4_t& lo, float& omax)
{
    const float2_t a = {x0, x1}, b = {x2, x3};
    const half2_t ha = __builtin_convertvector(a, half2_t), hb = __builtin_convertvector(b, half2_t);
    hi = half4_t{ha[0], ha[1], hb[0], hb[1]};
    if constexpr (P == 1) {
        const half2_t la = __builtin_convertvector((a - __builtin_convertvector(ha, float2_t)) * 2048.f, half2_t);
        const half2_t lb = __builtin_convertvector((b - __builtin_convertvector(hb, float2_t)) * 2048.f, half2_t);
        lo = half4_t{la[0], la[1], lb[0], lb[1]};
    }
    const float m = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(x0), __builtin_fabsf(x1)),
                                    __builtin_fmaxf(__builtin_fabsf(x2), __builtin_fabsf(x3)));
    omax = __builtin_fmaxf(omax, m);
}

// kEpiDown's fourth stage: e = conv(PReLU_down(y)) over region A (rows w <->
// frames t0 - OFF + w, split like every stage input).  Output frame
// t0 / R + u reads rows u R + j, j < KF R (tap j = k R + phase of the tap-major
// packed weights, ou_block_pack of [2C][C][KF R]).  2C / 32 x ceil(F / R / 32)
// 32 x 32 tiles, dealt over the 4 waves.
template <int C, int P, int R, int KF, int F, int SX>
__device__ __forceinline__ void down_stage(const ou_block_desc& d, const _Float16* xa, int pstride, int t0, int T,
                                           int TS, int b, int wave, int lane)
{
    constexpr int KT = KF * R, KS = C / 16, NS = KT * KS;
    constexpr int M4 = 2 * C / 32, NU = F / R, N4 = (NU + 31) / 32;
    constexpr int D = NS < 6 ? NS : 6;
    const int l32 = lane & 31, h = lane >> 5;
    const half8_t* wp = (const half8_t*)d.w_down;
    const int TE = (TS + R - 1) / R;   // e stored for output frames < ceil(TS / R)
    const int e0 = t0 / R;
    const float un = d.w_down_unscale * ou_exp2i(d.shift[3] - kStageShift);
    for (int tile = wave; tile < M4 * N4; tile += 4) {
        const int m4 = tile % M4, n4 = tile / M4;
        const int u = n4 * 32 + l32;
        const _Float16* xb = xa + (u < NU ? u * R : 0) * SX + 8 * h;
        floatx16 acc, accx;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f, accx[r] = 0.f;
        half8_t ra[D][2];
        auto load_a = [&](int s, half8_t (&dst)[2]) {
            const int k = s / KS, ks = s - (s / KS) * KS;
            const half8_t* p = wp + (((int64_t)(m4 * KT + k) * KS + ks) * 2) * 64 + lane;
            dst[0] = p[0];
            if constexpr (P == 1) dst[1] = p[64];
        };
#pragma unroll
        for (int s = 0; s < D - 1; ++s) load_a(s, ra[s]);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (s + D - 1 < NS) load_a(s + D - 1, ra[(s + D - 1) % D]);
            const int k = s / KS, ks = s - (s / KS) * KS;
            const _Float16* q = xb + k * SX + 16 * ks;
            const half8_t bq = *(const half8_t*)q;
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s % D][0], bq, acc, 0, 0, 0);
            if constexpr (P == 1) {
                const half8_t bl = *(const half8_t*)(q + pstride);
                accx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s % D][0], bl, accx, 0, 0, 0);
                accx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s % D][1], bq, accx, 0, 0, 0);
            }
        }
        const int te = e0 + u;
        if (u >= NU || te >= TE) continue;
        float* eb = d.e + (int64_t)b * d.e_bstride + te;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m4 * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            const float bias = d.b_down ? d.b_down[m] : 0.f;
            eb[(int64_t)m * d.e_cstride] = __builtin_fmaf(__builtin_fmaf(accx[r], 1.f / 2048.f, acc[r]), un, bias);
        }
    }
}

template <int C>
constexpr int block_threads()
{
    return C > 0 ? 256 : 0;
}

// resident workgroups per CU the register budget is sized for: two (256
// VGPRs a lane) where a wave owns one or two M tiles; one (512) for PP24's
// 96 / 192 channels, whose waves own three M tiles (their ~107 KB of LDS
// allows one workgroup per CU anyway)
template <int C>
constexpr int block_min_wgs()
{
    return (C == 96 || C == 192) ? 1 : 2;
}

constexpr int kBlkSentinel = 0x7ffffff0;   // byte offset past any buffer: loads return 0

template <int C, int NT, int P, int EPI, int R = 1, int KF = 1>
__global__ __launch_bounds__(block_threads<C>(), block_min_wgs<C>()) void block_kernel(ou_block_desc d)
{
    using K = BCfg<C, NT, P>;
    ou_kernarg_prefetch8();
    constexpr int MR = K::MR, NR = K::NR, NF = K::NF, SX = K::SX;
    constexpr int OFF = block_off<EPI, R, KF>();   // conv3 starts OFF frames before t0
    constexpr int F = block_f<C, NT, P, EPI, R, KF>();
    // per-stage staging exponents (the host widens one whose range flag trips)
    const float kIn0 = ou_exp2i(-d.shift[0]), kIn1 = ou_exp2i(-d.shift[1]), kIn2 = ou_exp2i(-d.shift[2]),
                kInD = ou_exp2i(-d.shift[3]);
    OU_DYNAMIC_LDS(half8_t, lds8);
    using E = typename K::E;
    E* lds = (E*)lds8;
    E* xa = lds + K::A_OFF;
    E* xbuf = lds + K::B_OFF;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave % K::WM, wn = wave / K::WM;
    const int l32 = lane & 31, h = lane >> 5;
    const int b = blockIdx.y;
    const int T = d.length;
    const int t0 = d.f0 + blockIdx.x * F;   // first output frame of the workgroup (global)
    const int TS = d.f1 > 0 ? min(d.f1, T) : T;   // outputs stored for frames < TS
    const int hlo = d.h0, hhi = d.h1 > 0 ? min(d.h1, T) : T;   // h frames the caller produced
    const float* __restrict__ hb = d.h + (int64_t)b * d.h_bstride;
    float om0 = 0.f, om1 = 0.f, om2 = 0.f, omd = 0.f;   // max |staged value| of the conv1 / 2 / 3 / down inputs
    float oms = 0.f;                                     // max |split-image value| (d.sy)
    // weight-fragment ring shared by the three split-f16 / f16 stages; conv1's
    // first fragments are requested before the input staging
    constexpr bool early = OU_BLOCK_RING_EARLY && P != 0;
    half8_t ring[K::RING][MR][2];
    if constexpr (early) ring_pro<5, C, NT, P>(d.w[0], wm, lane, ring);

    // scaled input sample of the fused input conv (zero outside [0, T))
    const float* __restrict__ xin = (EPI & kEpiIn) ? d.x + (int64_t)b * d.x_bstride : nullptr;
    const float xsc = (EPI & kEpiIn) ? (d.in_scale ? d.in_scale[b] : 1.f) : 0.f;
    auto xs = [&](int t) { return (t >= 0 && t < T) ? xsc * xin[t] : 0.f; };
    auto in_conv = [&](int c, float xl, float xm, float xr) {   // conv1d(1 -> C, k3) at one frame
        return __builtin_fmaf(d.w_in[3 * c + 2], xr,
                              __builtin_fmaf(d.w_in[3 * c + 1], xm, __builtin_fmaf(d.w_in[3 * c], xl, d.b_in[c])));
    };

    // ---- stage 0: PReLU1(h) * 2^-shift over frames [t0 - 4 - OFF, ...) -> region A.
    // A work item is (8-channel group, frame): 8 coalesced loads (consecutive
    // lanes = consecutive frames), then one 16-B LDS write per plane.  All
    // loads of a thread are issued before any arithmetic.  With a split image
    // of the operand (d.xs, stored by the producing conv) an item is two 16-B
    // loads (hi, lo) copied to LDS as they are.
    if (P == 1 && !(EPI & kEpiIn) && d.xs) {
        constexpr int NI = (C / 8) * K::R1;
        constexpr int NIT = (NI + K::NTH - 1) / K::NTH;
        const __amdgpu_buffer_rsrc_t xrs =
            ou_rsrc((const char*)d.xs + (int64_t)b * d.xs_bstride, (int64_t)(C / 32) * d.xs_rows * 128);
        ou_u4_t vh[NIT], vl[NIT];
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int item = min(tid + K::NTH * it, NI - 1);
            const int g = item / K::R1, r = item - g * K::R1;
            const int t = t0 - 4 - OFF + r;
            const bool ok = t >= 0 && t < T && !(d.dbg & 1);
            const int vo = ok ? ((g >> 2) * d.xs_rows + t) * 128 + (g & 3) * 16 : kBlkSentinel;
            vh[it] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vo, 0, 0);
            vl[it] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vo, 64, 0);
        }
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int item = tid + K::NTH * it;
            if (NIT * K::NTH > NI && item >= NI) break;
            const int g = item / K::R1, r = item - g * K::R1;
            E* dst = xa + r * SX + 8 * g;
            *(ou_u4_t*)dst = vh[it];
            *(ou_u4_t*)(dst + K::PA) = vl[it];
        }
    } else {
        constexpr int NI = (C / 8) * K::R1;
        constexpr int NIT = (NI + K::NTH - 1) / K::NTH;
        const float a1 = d.slope[0];
        float v[NIT][8];
        // h as a buffer resource: one voffset per item, the 8 channel rows as
        // scalar soffsets i * h_cstride, frames outside [max(0, h0), min(T, h1))
        // at the sentinel voffset (they load 0): no per-load address math
        const int hcs = (int)d.h_cstride;
        const __amdgpu_buffer_rsrc_t hrs = ou_rsrc(hb, (int64_t)C * d.h_cstride * 4);
        const int tlo = max(0, hlo), thi = min(T, hhi);
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int item = min(tid + K::NTH * it, NI - 1);
            const int g = item / K::R1, r = item - g * K::R1;
            const int t = t0 - 4 - OFF + r;
            if constexpr (EPI & kEpiIn) {
                const float xl = xs(t - 1), xm = xs(t), xr = xs(t + 1);
#pragma unroll
                for (int i = 0; i < 8; ++i) v[it][i] = in_conv(8 * g + i, xl, xm, xr);
                if (t < tlo || t >= thi || (d.dbg & 1)) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[it][i] = 0.f;
                }
            } else {
                const bool ok = t >= tlo && t < thi && !(d.dbg & 1);
                const int vo = ok ? (8 * g * hcs + t) * 4 : kBlkSentinel;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    v[it][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(hrs, vo, i * hcs * 4, 0));
            }
        }
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int item = tid + K::NTH * it;
            if (NIT * K::NTH > NI && item >= NI) break;
            const int g = item / K::R1, r = item - g * K::R1;
            float x[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = (v[it][i] >= 0.f ? kIn0 : a1 * kIn0) * v[it][i];
            if constexpr (P == 0) {   // f32, pair-split channel order (ch_pos)
                E* row = xa + r * SX;
                *(f32x4_t*)(row + 4 * g) = f32x4_t{x[0], x[2], x[4], x[6]};
                *(f32x4_t*)(row + C / 2 + 4 * g) = f32x4_t{x[1], x[3], x[5], x[7]};
            } else {
                half4_t h0, h1, l0, l1;
                split4<P>(x[0], x[1], x[2], x[3], h0, l0, om0);
                split4<P>(x[4], x[5], x[6], x[7], h1, l1, om0);
                E* dst = xa + r * SX + 8 * g;
                *(half8_t*)dst = half8_t{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
                if constexpr (P == 1)
                    *(half8_t*)(dst + K::PA) = half8_t{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
            }
        }
    }
    __syncthreads();

    floatx16 acc[MR][NR], accx[MR][NR];
    // per-row constants of this wave's output rows: m = row(mr, r)
    auto row = [&](int mr, int r) { return (wm * MR + mr) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h; };
    // C not a multiple of 32 (48): rows >= C are padding -- loads clamp to a
    // real row (the value is never stored), stores skip them
    constexpr bool PADM = C % 32 != 0;
    auto rowc = [&](int mr, int r) { return PADM ? min(row(mr, r), C - 1) : row(mr, r); };
    // row(mr, r) - 4 h: wave-uniform, so an f32 plane [C][cs] is read and
    // written through a buffer resource with the row in the scalar soffset and
    // the lane's frame (plus its half's 4 rows) in the voffset -- no per-element
    // 64-bit address arithmetic (channel counts without padded rows)
    auto rbase = [&](int mr, int r) { return (wm * MR + mr) * 32 + (r & 3) + 8 * (r >> 2); };
    auto rok = [&](int mr, int r) { return !PADM || row(mr, r) < C; };
    auto gok = [&](int mr, int j) { return !PADM || (wm * MR + mr) * 32 + 8 * j + 4 * h < C; };
    // a stage output: channels c0 .. c0 + 3 (c0 % 4 == 0) of one LDS row, as
    // the next stage's operand (split halves, or f32 in ch_pos order)
    auto put4 = [&](E* row, int c0, const float (&x)[4], int pstride, float& om) {
        if constexpr (P == 0) {
            *(float2_t*)(row + (c0 >> 1)) = float2_t{x[0], x[2]};
            *(float2_t*)(row + C / 2 + (c0 >> 1)) = float2_t{x[1], x[3]};
        } else {
            half4_t hi, lo;
            split4<P>(x[0], x[1], x[2], x[3], hi, lo, om);
            *(half4_t*)(row + c0) = hi;
            if constexpr (P == 1) *(half4_t*)(row + c0 + pstride) = lo;
        }
    };
    auto zero8 = [&](E* row, int c0, int pstride) {   // channels c0 .. c0 + 7 (c0 % 8 == 0)
        if constexpr (P == 0) {
            *(f32x4_t*)(row + (c0 >> 1)) = f32x4_t{};
            *(f32x4_t*)(row + C / 2 + (c0 >> 1)) = f32x4_t{};
        } else {
            *(half8_t*)(row + c0) = half8_t{};
            if constexpr (P == 1) *(half8_t*)(row + c0 + pstride) = half8_t{};
        }
    };

    // ---- stage 1: conv1 (k5) over frames t0 - 2 + u, u in [0, NF) -> region B
    run_stage<5, C, NT, P>(d.w[0], xa, K::PA, wm, wn, lane, d.dbg, acc, accx, ring, early);
    if (early) ring_pro<3, C, NT, P>(d.w[1], wm, lane, ring);   // conv2's first fragments
    {
        const float a2 = d.slope[1];
        // operands of the epilogue, loaded before anything is stored
        float bia[MR][16], gam[MR][16], bet[MR][16], scv[MR][NR][16];
        const float* film = d.film + (int64_t)b * d.film_bstride;
#pragma unroll
        for (int mr = 0; mr < MR; ++mr)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = rowc(mr, r);
                bia[mr][r] = d.bias[0] ? d.bias[0][m] : 0.f;
                if constexpr (EPI & kEpiFilm) {
                    gam[mr][r] = film[m];
                    bet[mr][r] = film[C + m];
                }
                if constexpr (EPI & kEpiSc) {
#pragma unroll
                    for (int nr = 0; nr < NR; ++nr) {   // frames outside [0, T) are zeroed below
                        const int t = min(max(t0 - 2 - OFF + (wn * NR + nr) * 32 + l32, 0), T - 1);
                        if constexpr (PADM) {
                            scv[mr][nr][r] = d.sc[(int64_t)b * d.sc_bstride + (int64_t)m * d.sc_cstride + t];
                        } else {
                            const int cs4 = (int)d.sc_cstride * 4;
                            scv[mr][nr][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                                ou_rsrc(d.sc + (int64_t)b * d.sc_bstride, (int64_t)C * cs4), t * 4 + 4 * h * cs4,
                                rbase(mr, r) * cs4, 0));
                        }
                    }
                }
            }
        const float un = d.w_unscale[0] * ou_exp2i(d.shift[0] - kStageShift);
#pragma unroll
        for (int mr = 0; mr < MR; ++mr)
#pragma unroll
            for (int nr = 0; nr < NR; ++nr) {
                const int u = (wn * NR + nr) * 32 + l32;
                const int t = t0 - 2 - OFF + u;
                const bool inside = t >= 0 && t < T;
                float o[16];
#pragma unroll
                for (int r = 0; r < 16; r += 2) {   // pairs: packed fma / add / mul, bit-identical to scalar
                    float2_t v = fma2(fma2(float2_t{accx[mr][nr][r], accx[mr][nr][r + 1]}, 1.f / 2048.f,
                                           float2_t{acc[mr][nr][r], acc[mr][nr][r + 1]}),
                                      un, float2_t{bia[mr][r], bia[mr][r + 1]});
                    if constexpr (EPI & kEpiSc) v = (v + float2_t{scv[mr][nr][r], scv[mr][nr][r + 1]}) * d.s_sc;
                    if constexpr (EPI & kEpiFilm)
                        v = fma2(float2_t{gam[mr][r], gam[mr][r + 1]}, v, float2_t{bet[mr][r], bet[mr][r + 1]});
                    o[r] = inside ? v.x : 0.f, o[r + 1] = inside ? v.y : 0.f;
                }
                if constexpr (EPI & kEpiCond) {
                    const bool st = inside && t >= t0 && t < t0 + F && t < TS;
                    if constexpr (PADM) {
                        if (st) {
                            float* co = d.cond_out + (int64_t)b * d.co_bstride + t;
#pragma unroll
                            for (int r = 0; r < 16; ++r)
                                if (rok(mr, r)) co[(int64_t)row(mr, r) * d.co_cstride] = o[r];
                        }
                    } else {
                        const int cs4 = (int)d.co_cstride * 4;
                        const __amdgpu_buffer_rsrc_t crs =
                            ou_rsrc(d.cond_out + (int64_t)b * d.co_bstride, (int64_t)C * cs4);
                        const int vo = st ? t * 4 + 4 * h * cs4 : kBlkSentinel;
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o[r]), crs, vo, rbase(mr, r) * cs4, 0);
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (!gok(mr, j)) continue;
                    float x[4];
#pragma unroll
                    for (int i = 0; i < 4; i += 2) {
                        const float2_t q = {o[4 * j + i], o[4 * j + i + 1]};
                        const float2_t xx = q * float2_t{q.x >= 0.f ? kIn1 : a2 * kIn1, q.y >= 0.f ? kIn1 : a2 * kIn1};
                        x[i] = xx.x, x[i + 1] = xx.y;
                    }
                    put4(xbuf + u * SX, (wm * MR + mr) * 32 + 8 * j + 4 * h, x, K::PB, om1);
                }
            }
        // rows NF, NF + 1 feed only discarded conv2 columns: keep them zero
        for (int e = tid; e < 2 * (C / 8); e += K::NTH) zero8(xbuf + (NF + e / (C / 8)) * SX, 8 * (e % (C / 8)), K::PB);
    }
    __syncthreads();

    // ---- stage 2: conv2 (k3) over frames t0 - 1 + v -> region A
    run_stage<3, C, NT, P>(d.w[1], xbuf, K::PB, wm, wn, lane, d.dbg, acc, accx, ring, early);
    if (early) ring_pro<3, C, NT, P>(d.w[2], wm, lane, ring);   // conv3's first fragments
    {
        const float a3 = d.slope[2], un = d.w_unscale[1] * ou_exp2i(d.shift[1] - kStageShift);
        float bia[MR][16];
#pragma unroll
        for (int mr = 0; mr < MR; ++mr)
#pragma unroll
            for (int r = 0; r < 16; ++r) bia[mr][r] = d.bias[1] ? d.bias[1][rowc(mr, r)] : 0.f;
#pragma unroll
        for (int mr = 0; mr < MR; ++mr)
#pragma unroll
            for (int nr = 0; nr < NR; ++nr) {
                const int v_ = (wn * NR + nr) * 32 + l32;
                const int t = t0 - 1 - OFF + v_;
                const float keep = (t >= 0 && t < T) ? kIn2 : 0.f, akeep = a3 * keep;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (!gok(mr, j)) continue;
                    float x[4];
#pragma unroll
                    for (int i = 0; i < 4; i += 2) {   // pairs: packed fma / mul, bit-identical to the scalar chain
                        const int r = 4 * j + i;
                        const float2_t q = fma2(fma2(float2_t{accx[mr][nr][r], accx[mr][nr][r + 1]}, 1.f / 2048.f,
                                                     float2_t{acc[mr][nr][r], acc[mr][nr][r + 1]}),
                                                un, float2_t{bia[mr][r], bia[mr][r + 1]});
                        const float2_t xx = q * float2_t{q.x >= 0.f ? keep : akeep, q.y >= 0.f ? keep : akeep};
                        x[i] = xx.x, x[i + 1] = xx.y;
                    }
                    put4(xa + v_ * SX, (wm * MR + mr) * 32 + 8 * j + 4 * h, x, K::PA, om2);
                }
            }
        for (int e = tid; e < 2 * (C / 8); e += K::NTH) zero8(xa + (NF + e / (C / 8)) * SX, 8 * (e % (C / 8)), K::PA);
    }
    __syncthreads();

    // ---- stage 3: conv3 (k3) over frames t0 - OFF + w, w < F + 2 OFF -> y
    // the block residual h (and res2) of this wave's output tiles: loaded
    // before the conv3 MFMAs when OU_BLOCK_HV_EARLY (their latency then hides
    // under the stage), else after it
    float hv[MR][NR][16], rv[MR][NR][16];
    auto load_res = [&]() {
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
            const int w = (wn * NR + nr) * 32 + l32;
            const int t = t0 - OFF + w;
            const int tc = min(max(t, 0), T - 1);   // frames outside [0, T) are not stored
            if constexpr (EPI & kEpiIn) {
                const float xl = xs(t - 1), xm = xs(t), xr = xs(t + 1);
#pragma unroll
                for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                    for (int r = 0; r < 16; ++r) hv[mr][nr][r] = in_conv(rowc(mr, r), xl, xm, xr);
            } else {
                // frames outside [h0, h1) (a chunk's caller has not produced
                // them) feed no stored output; zero, so that kEpiDown's
                // re-split of those frames cannot trip the range flag
                const bool hk = t >= hlo && t < hhi;
                if constexpr (PADM) {
#pragma unroll
                    for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const float v = hb[(int64_t)rowc(mr, r) * d.h_cstride + tc];
                            hv[mr][nr][r] = hk ? v : 0.f;
                        }
                } else {   // frames outside [h0, h1) at the sentinel: they load 0
                    const int cs4 = (int)d.h_cstride * 4;
                    const __amdgpu_buffer_rsrc_t rs = ou_rsrc(hb, (int64_t)C * cs4);
                    const int vo = hk ? tc * 4 + 4 * h * cs4 : kBlkSentinel;
#pragma unroll
                    for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            hv[mr][nr][r] =
                                __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, rbase(mr, r) * cs4, 0));
                }
            }
            if constexpr (EPI & kEpiRes2) {
                if constexpr (PADM) {
#pragma unroll
                    for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            rv[mr][nr][r] =
                                d.res2[(int64_t)b * d.r2_bstride + (int64_t)rowc(mr, r) * d.r2_cstride + tc];
                } else {
                    const int cs4 = (int)d.r2_cstride * 4;
                    const __amdgpu_buffer_rsrc_t rs = ou_rsrc(d.res2 + (int64_t)b * d.r2_bstride, (int64_t)C * cs4);
                    const int vo = tc * 4 + 4 * h * cs4;
#pragma unroll
                    for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            rv[mr][nr][r] =
                                __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, rbase(mr, r) * cs4, 0));
                }
            }
        }
    };
    if constexpr (OU_BLOCK_HV_EARLY && !(EPI & kEpiIn)) load_res();
    run_stage<3, C, NT, P>(d.w[2], xa, K::PA, wm, wn, lane, d.dbg, acc, accx, ring, early);
    if constexpr (!(OU_BLOCK_HV_EARLY && !(EPI & kEpiIn))) load_res();
    {
        const float un = d.w_unscale[2] * ou_exp2i(d.shift[2] - kStageShift);
        float bia[MR][16];
#pragma unroll
        for (int mr = 0; mr < MR; ++mr)
#pragma unroll
            for (int r = 0; r < 16; ++r) bia[mr][r] = d.bias[2] ? d.bias[2][rowc(mr, r)] : 0.f;
        if constexpr (EPI & kEpiHead) {
            // the score head on the block output: Y[w][c] = prelu2(prelu1(y))
            // (f32, region A, zero outside [0, T)), then one thread per frame
            __syncthreads();   // every wave is done reading region A (conv3 input)
            float* Y = (float*)xa;
            constexpr int YS = C + 1;
            const ou_head_desc& hd = d.head;
#pragma unroll
            for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                for (int nr = 0; nr < NR; ++nr) {
                    const int w = (wn * NR + nr) * 32 + l32;
                    const int t = t0 - OFF + w;
                    const bool inside = t >= 0 && t < T && w < F + 2;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        float v = __builtin_fmaf(__builtin_fmaf(accx[mr][nr][r], 1.f / 2048.f, acc[mr][nr][r]), un,
                                                 bia[mr][r]);
                        v = (v + hv[mr][nr][r]) * d.s_res;
                        v = v >= 0.f ? v : v * hd.slope1;
                        v = v >= 0.f ? v : v * hd.slope2;
                        if (w < F + 2 && rok(mr, r)) Y[w * YS + row(mr, r)] = inside ? v : 0.f;
                    }
                }
            __syncthreads();
            for (int f = tid; f < F; f += K::NTH) {
                const int t = t0 + f;
                if (t >= TS) break;
                float net = 0.f;
                for (int c = 0; c < C; ++c)
#pragma unroll
                    for (int k = 0; k < 3; ++k) net = __builtin_fmaf(hd.w[c * 3 + k], Y[(f + k) * YS + c], net);
                net += hd.bias;
                const int64_t o = (int64_t)b * T + t;
                float out;
                if (hd.mode == 0) {
                    out = net;
                } else {
                    const float x = hd.x[o];
                    float score = net;
                    if (hd.edm) {
                        const float est = __fadd_rn(__fmul_rn(hd.w_skip, x), __fmul_rn(hd.w_out, net));
                        score = __fdiv_rn(__fsub_rn(est, x), hd.s2);
                    }
                    out = __fadd_rn(x, __fmul_rn(hd.c_score, score));
                    if (hd.mode == 1) out = __fadd_rn(out, __fmul_rn(hd.c_noise, __fmul_rn(hd.z[o], hd.s_next)));
                }
                hd.out[o] = out;
            }
        } else {
            float* yb = d.y + (int64_t)b * d.y_bstride;
            const __amdgpu_buffer_rsrc_t srs =
                ou_rsrc(d.sy ? (const char*)d.sy + (int64_t)b * d.sy_bstride : (const char*)yb,
                        d.sy ? (int64_t)(C / 32) * d.sy_rows * 128 : 0);
            const float sscale = ou_exp2i(-d.sy_shift);
            const __amdgpu_buffer_rsrc_t yrs = ou_rsrc(yb, (int64_t)C * d.y_cstride * 4);
            // kEpiDown: PReLU_down(y) 2^-6 also goes to region A (split), rows
            // w <-> frames t0 - OFF + w, zero outside [0, T) and past the rows
            // the strided conv reads
            if constexpr (EPI & kEpiDown) __syncthreads();   // every wave is done reading region A
            const float ad = (EPI & kEpiDown) ? d.slope_down : 0.f;
#pragma unroll
            for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                for (int nr = 0; nr < NR; ++nr) {
                    const int w = (wn * NR + nr) * 32 + l32;
                    const int t = t0 - OFF + w;
                    const bool own = w >= OFF && w < OFF + F && t < TS && !((d.dbg & 4) && !(d.dbg & 1024));
                    float vv[16];
                    const int ycs4 = (int)d.y_cstride * 4;
                    const int yvo = own ? t * 4 + 4 * h * ycs4 : kBlkSentinel;
#pragma unroll
                    for (int r = 0; r < 16; r += 2) {   // pairs: packed arithmetic, bit-identical to scalar
                        float2_t v2 = fma2(fma2(float2_t{accx[mr][nr][r], accx[mr][nr][r + 1]}, 1.f / 2048.f,
                                                float2_t{acc[mr][nr][r], acc[mr][nr][r + 1]}),
                                           un, float2_t{bia[mr][r], bia[mr][r + 1]});
                        v2 = (v2 + float2_t{hv[mr][nr][r], hv[mr][nr][r + 1]}) * d.s_res;
                        if constexpr (EPI & kEpiRes2) v2 = (v2 + float2_t{rv[mr][nr][r], rv[mr][nr][r + 1]}) * d.s2;
                        vv[r] = v2.x, vv[r + 1] = v2.y;
                    }
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float v = vv[r];
                        if constexpr (PADM) {
                            if (own && rok(mr, r)) yb[(int64_t)row(mr, r) * d.y_cstride + t] = v;
                        } else {
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), yrs, yvo, rbase(mr, r) * ycs4, 0);
                        }
                    }
                    if (P == 1 && d.sy) {   // the next conv's split image (host-checked: C % 32 == 0)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int c0 = (wm * MR + mr) * 32 + 8 * j + 4 * h;
                            const int off = own ? ((c0 >> 5) * d.sy_rows + t) * 128 + (c0 & 31) * 2 : kBlkSentinel;
                            ou_split_store4(srs, off, own, vv[4 * j], vv[4 * j + 1], vv[4 * j + 2], vv[4 * j + 3],
                                            sscale, d.sy_slope, oms);
                        }
                    }
                    if constexpr (EPI & kEpiDown) {
                        constexpr int RH = R * (KF - 1 - (KF - 1) / 2);
                        const float keep = (t >= 0 && t < T && w < F + OFF + RH) ? kInD : 0.f;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            float x[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const float q = vv[4 * j + i];
                                x[i] = (q >= 0.f ? keep : ad * keep) * q;
                            }
                            half4_t hi, lo;
                            split4<P>(x[0], x[1], x[2], x[3], hi, lo, omd);
                            if (!gok(mr, j)) continue;
                            _Float16* dst = xa + w * SX + (wm * MR + mr) * 32 + 8 * j + 4 * h;
                            *(half4_t*)dst = hi;
                            if constexpr (P == 1) *(half4_t*)(dst + K::PA) = lo;
                        }
                    }
                }
            if constexpr (EPI & kEpiDown) {
                __syncthreads();
                down_stage<C, P, R, KF, F, SX>(d, xa, K::PA, t0, T, TS, b, wave, lane);
            }
        }
    }
    // range codes: 1 / 2 / 8 / 16 the conv1 / conv2 / conv3 / down input's
    // exponent is too small, 32 the split image's (d.sy), 4 an infinite
    // input (ou_range_flag)
    if constexpr (P != 0) {
        ou_range_flag(d.status, om0, 1, lane);
        ou_range_flag(d.status, om1, 2, lane);
        ou_range_flag(d.status, om2, 8, lane);
        if constexpr ((EPI & kEpiDown) != 0) ou_range_flag(d.status, omd, 16, lane);
        if (d.sy) ou_range_flag(d.status, oms, 32, lane);
    }
}

template <int C, int NT, int P, int EPI, int R = 1, int KF = 1>
int launch(const ou_block_desc& d, hipStream_t s)
{
    using K = BCfg<C, NT, P>;
    static bool attr = false;
    if (!attr) {
        OU_HIP_CHECK(hipFuncSetAttribute((const void*)block_kernel<C, NT, P, EPI, R, KF>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS_BYTES),
                     "block: LDS attribute");
        attr = true;
    }
    constexpr int F = block_f<C, NT, P, EPI, R, KF>();
    static_assert(F > 0 && F % R == 0, "block: frames per workgroup");
    const int f1 = d.f1 > 0 ? min(d.f1, d.length) : d.length;
    if (d.f0 < 0 || d.f0 >= f1 || d.f0 % R || (R > 1 && f1 % R && f1 != d.length))
        return ou_fail(-1, "block: frame range [%d, %d) (rate %d, length %d)", d.f0, f1, R, d.length);
    dim3 grid((f1 - d.f0 + F - 1) / F, d.batch);
    hipLaunchKernelGGL((block_kernel<C, NT, P, EPI, R, KF>), grid, dim3(K::NTH), K::LDS_BYTES, s, d);
    return ou_check_launch("block");
}

// rate-change variants instantiated (PP16 / ORIG16 encoders: rates 2 and 4
// at 32 and 64 channels; the score encoder folds the FIR, KF = 3, the
// conditioner's does not, KF = 1).  Every workgroup streams the stage's
// 2C x C x KF R weights for its F / R output frames: at 64 channels with the
// folded FIR (393 KB for 13 frames) that stream costs more than the separate
// launch saves (score encoder level 1: 70 -> 82 us per block with 60-frame
// windows, 77-92 us with 116-frame ones), so that variant stays unfused.
constexpr bool down_ok(int C, int rate, int kt)
{
    return (C == 32 && rate == 2 && (kt == 3 || kt == 1)) || (C == 64 && rate == 4 && kt == 1);
}

template <int C, int NT, int P, int EPI>
int launch_down(const ou_block_desc& d, hipStream_t s)
{
    if constexpr (C == 32) {
        if (d.rate == 2 && d.down_kt == 3) return launch<C, NT, P, EPI, 2, 3>(d, s);
        if (d.rate == 2 && d.down_kt == 1) return launch<C, NT, P, EPI, 2, 1>(d, s);
    } else if constexpr (C == 64) {
        if (d.rate == 4 && d.down_kt == 1) return launch<C, NT, P, EPI, 4, 1>(d, s);
    }
    return ou_fail(-1, "block: no fused rate-change conv for %d channels, rate %d, kt %d", C, d.rate, d.down_kt);
}

template <int C, int NT, int P>
int launch_epi(const ou_block_desc& d, hipStream_t s)
{
    const int epi = (d.film ? kEpiFilm : 0) | (d.sc ? kEpiSc : 0) | (d.cond_out ? kEpiCond : 0) |
                    (d.res2 ? kEpiRes2 : 0) | (d.x ? kEpiIn : 0) | (d.head.w ? kEpiHead : 0) |
                    (d.w_down ? kEpiDown : 0);
    if constexpr ((C == 32 || C == 64) && P != 0) {   // encoder blocks with their rate-change conv
        switch (epi) {
        case kEpiDown: return launch_down<C, NT, P, kEpiDown>(d, s);
        case kEpiFilm | kEpiDown: return launch_down<C, NT, P, kEpiFilm | kEpiDown>(d, s);
        }
        if constexpr (C == 32)
            if (epi == (kEpiFilm | kEpiIn | kEpiDown)) return launch_down<C, NT, P, kEpiFilm | kEpiIn | kEpiDown>(d, s);
    }
    switch (epi) {
    case 0: return launch<C, NT, P, 0>(d, s);
    case kEpiFilm: return launch<C, NT, P, kEpiFilm>(d, s);
    case kEpiFilm | kEpiSc: return launch<C, NT, P, kEpiFilm | kEpiSc>(d, s);
    case kEpiCond: return launch<C, NT, P, kEpiCond>(d, s);
    case kEpiRes2: return launch<C, NT, P, kEpiRes2>(d, s);
    }
    if constexpr (C == 32 || C == 48) {   // the score network's ends (32 / 48 channels at level 0)
        switch (epi) {
        case kEpiFilm | kEpiIn: return launch<C, NT, P, kEpiFilm | kEpiIn>(d, s);
        case kEpiFilm | kEpiSc | kEpiHead: return launch<C, NT, P, kEpiFilm | kEpiSc | kEpiHead>(d, s);
        case kEpiIn: return launch<C, NT, P, kEpiIn>(d, s);
        case kEpiHead: return launch<C, NT, P, kEpiHead>(d, s);
        }
    }
    return ou_fail(-1, "block: unsupported epilogue combination %d at %d channels", epi, C);
}

// 32-frame N tiles per workgroup, per channel count
template <int C>
constexpr int nt_for()
{
    return C == 32 ? OU_BLOCK_NT32 : C == 64 ? OU_BLOCK_NT64 : C == 128 ? OU_BLOCK_NT128
         : C == 48 ? OU_BLOCK_NT48 : C == 96 ? OU_BLOCK_NT96 : C == 192 ? OU_BLOCK_NT192 : 1;
}

template <int P>
int launch_p(const ou_block_desc& d, hipStream_t s)
{
    switch (d.channels) {
    case 32: return launch_epi<32, nt_for<32>(), P>(d, s);
    case 64: return launch_epi<64, nt_for<64>(), P>(d, s);
    case 128: return launch_epi<128, nt_for<128>(), P>(d, s);
    case 48: return launch_epi<48, nt_for<48>(), P>(d, s);
    case 96: return launch_epi<96, nt_for<96>(), P>(d, s);
    case 192: return launch_epi<192, nt_for<192>(), P>(d, s);
    case 256: return launch_epi<256, 1, P>(d, s);
    }
    return ou_fail(-1, "block: unsupported channel count %d", d.channels);
}

}  // namespace

// C = 256 (and the 512-channel bottleneck) stay on ou_conv: with one
// workgroup owning every channel, the fused form re-streams the whole
// 256 x 256 x 11 weight set for every 28 frames and is weight-bandwidth bound
// (53 us with 4 waves, 64 us with 8, against 52 us for the three ou_conv
// launches at 4005 frames, tools/block_bench.py); at 32 / 64 / 128 channels
// it is 2.0x / 1.4x / 1.2x faster than the unfused launches.
extern "C" int ou_block_supported(int channels, int prec)
{
    return (prec == 0 || prec == 1 || prec == 2) &&
           (channels == 32 || channels == 64 || channels == 128 || channels == 48 || channels == 96 ||
            channels == 192);
}

extern "C" int ou_block_down_supported(int channels, int rate, int kt, int prec)
{
    return prec != 0 && ou_block_supported(channels, prec) && down_ok(channels, rate, kt);
}

extern "C" int ou_block_frames(int channels)
{
    switch (channels) {
    case 32: return BCfg<32, nt_for<32>(), 1>::F;
    case 64: return BCfg<64, nt_for<64>(), 1>::F;
    case 128: return BCfg<128, nt_for<128>(), 1>::F;
    case 48: return BCfg<48, nt_for<48>(), 1>::F;
    case 96: return BCfg<96, nt_for<96>(), 1>::F;
    case 192: return BCfg<192, nt_for<192>(), 1>::F;
    case 256: return BCfg<256, 1, 1>::F;
    }
    return 0;
}

extern "C" int64_t ou_block_packed_halves(int channels, int kt)
{
    return (int64_t)(channels + 31) / 32 * 32 * channels * kt * 2;   // rows padded to 32
}

extern "C" int ou_block_pack(const float* w, int channels, int kt, void* out, float* w_unscale)
{
    if (channels % 32 == 0 || !w || channels <= 0 || kt <= 0)
        return ou_block_pack_rect(w, channels, channels, kt, out, w_unscale);
    // 48 channels: zero rows up to the next 32 (ou_block computes, never stores, them)
    const int m = (channels + 31) / 32 * 32;
    std::vector<float> wp((size_t)m * channels * kt, 0.f);
    std::copy(w, w + (size_t)channels * channels * kt, wp.begin());
    return ou_block_pack_rect(wp.data(), m, channels, kt, out, w_unscale);
}

extern "C" int ou_block_pack_rect(const float* w, int m, int channels, int kt, void* out, float* w_unscale)
{
    if (!w || !out || !w_unscale || m <= 0 || m % 32 || channels <= 0 || channels % 16 || kt <= 0)
        return ou_fail(-1, "block_pack: bad arguments");
    const int C = channels, KS = C / 16, MT = m / 32;
    const int64_t n = (int64_t)m * C * kt;
    float mx = 0.f;
    for (int64_t i = 0; i < n; ++i) {
        if (!std::isfinite(w[i])) return ou_fail(-1, "block_pack: non-finite weight at %lld", (long long)i);
        mx = std::fmax(mx, std::fabs(w[i]));
    }
    int e = 0;
    if (mx > 0.f) {
        int ex = 0;
        std::frexp(mx, &ex);                       // mx in [2^(ex-1), 2^ex)
        e = std::min(100, std::max(-100, 10 - ex));   // max|a| in [2^9, 2^10)
    }
    const float sc = std::ldexp(1.f, e);
    _Float16* o = (_Float16*)out;
    for (int mt = 0; mt < MT; ++mt)
        for (int k = 0; k < kt; ++k)
            for (int ks = 0; ks < KS; ++ks)
                for (int plane = 0; plane < 2; ++plane)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int i = 0; i < 8; ++i) {
                            const int row = mt * 32 + (lane & 31);
                            const int c = ks * 16 + 8 * (lane >> 5) + i;
                            const float a = w[((int64_t)row * C + c) * kt + k] * sc;
                            const _Float16 hi = (_Float16)a;
                            *o++ = plane == 0 ? hi : (_Float16)((a - (float)hi) * 2048.f);
                        }
    *w_unscale = std::ldexp(1.f, kStageShift - e);
    return 0;
}

extern "C" int64_t ou_block_packed_f32(int channels, int kt)
{
    return (int64_t)(channels + 31) / 32 * 32 * channels * kt;
}

// f32 operands (prec 0): [mt][tap][s4][lane][4] of w[row][2 (4 s4 + j) + (lane >> 5)][tap],
// row = 32 mt + (lane & 31) (zero past `channels`); *w_unscale = 2^kStageShift
// (the kernel stages activations as x * 2^-kStageShift, as the split form)
extern "C" int ou_block_pack_f32(const float* w, int channels, int kt, float* out, float* w_unscale)
{
    if (!w || !out || !w_unscale || channels <= 0 || channels % 16 || kt <= 0)
        return ou_fail(-1, "block_pack_f32: bad arguments");
    const int C = channels, MT = (C + 31) / 32, S4 = C / 8;
    for (int mt = 0; mt < MT; ++mt)
        for (int k = 0; k < kt; ++k)
            for (int s4 = 0; s4 < S4; ++s4)
                for (int lane = 0; lane < 64; ++lane)
                    for (int j = 0; j < 4; ++j) {
                        const int row = mt * 32 + (lane & 31);
                        const int c = 2 * (4 * s4 + j) + (lane >> 5);
                        *out++ = row < C ? w[((int64_t)row * C + c) * kt + k] : 0.f;
                    }
    *w_unscale = (float)(1 << kStageShift);
    return 0;
}

extern "C" int ou_block(const ou_block_desc* dp, void* stream)
{
    if (!dp) return ou_fail(-1, "block: null descriptor");
    const ou_block_desc& d = *dp;
    if (!d.h || !d.y || !d.w[0] || !d.w[1] || !d.w[2] || d.length <= 0 || d.batch <= 0 || d.batch > 65535)
        return ou_fail(-1, "block: invalid descriptor");
    if (!ou_block_supported(d.channels, d.prec))
        return ou_fail(-1, "block: channels %d / prec %d not supported", d.channels, d.prec);
    // buffer resources take 32-bit offsets with a sentinel for "outside":
    // every per-item tensor must stay below it
    const int64_t lim = kBlkSentinel;
    if ((int64_t)d.channels * d.h_cstride * 4 >= lim || (int64_t)d.channels * d.y_cstride * 4 >= lim ||
        (d.res2 && (int64_t)d.channels * d.r2_cstride * 4 >= lim) ||
        (d.sc && (int64_t)d.channels * d.sc_cstride * 4 >= lim) ||
        (d.cond_out && (int64_t)d.channels * d.co_cstride * 4 >= lim) ||
        (d.e && (int64_t)2 * d.channels * d.e_cstride * 4 >= lim))
        return ou_fail(-1, "block: a per-item tensor of %d x %lld floats exceeds the 32-bit buffer range", d.channels,
                       (long long)d.h_cstride);
    if (d.sy && (d.prec != 1 || d.channels % 32 || d.head.w || d.sy_rows < d.length || d.sy_shift < -100 ||
                 d.sy_shift > 100 || (int64_t)(d.channels / 32) * d.sy_rows * 128 >= lim))
        return ou_fail(-1, "block: a split-image output needs prec 1, channels %% 32 == 0, no head, sy_rows >= length");
    if (d.xs && (d.prec != 1 || d.channels % 32 || d.x || d.f0 || d.f1 || d.h0 || d.h1 || d.xs_rows < d.length ||
                 (int64_t)(d.channels / 32) * d.xs_rows * 128 >= lim))
        return ou_fail(-1, "block: a split-image input needs prec 1, channels %% 32 == 0, the whole signal, no input "
                           "conv, xs_rows >= length");
    hipStream_t s = (hipStream_t)stream;
    return d.prec == 1 ? launch_p<1>(d, s) : d.prec == 2 ? launch_p<2>(d, s) : launch_p<0>(d, s);
}
