// ou_conv.hip -- fused implicit-GEMM 1-D convolution for gfx950 (MI355X).
//
// One kernel covers every dense contraction of the UNIVERSE(++) hot path
// (SURVEY.md section 2.3, K1/K2/K3/K5/K8):
//   * PReLU_Conv k5/k3 'same' convs           (networks/universe/blocks.py:203-231)
//   * strided down-sampling conv + binomial FIR (blocks.py:268-275,123-134) with
//     the FIR folded into a 3-frame polyphase kernel (host, at load time)
//   * ConvTranspose1d up-sampling + FIR         (blocks.py:277-287), polyphase
//   * 1x1 convs (signal_cond_proj, GRU input projection, mel filterbank)
//   * st_convs (condition.py:33-65) and the STFT as a framed GEMM
//
// GEMM view: M = output rows (rout * cout), N = frames, K = channels x taps.
// The input is read through a "frame view" x'[c'][t] = x[c'/R][t*R + c'%R]
// so strided convs and the STFT become plain convolutions over frames.
//
// MI355X mapping
//   * fp32 operands => v_mfma_f32_32x32x2_f32 (exact f32 FMA chain; 157 TF/s
//     dense peak, 64 cycles per instruction per SIMD).
//   * workgroup = 4 waves arranged WM x WN x WK: WM x WN output sub-tiles of
//     32 x (32*NR), and WK waves splitting the K range of the same sub-tile
//     (intra-workgroup split-K, reduced through LDS).  Small-N deep levels
//     (512 channels x 801 frames at batch 1) need WK > 1 to put >= 1 wave on
//     every SIMD; the high-rate levels use WK = 1 and wide N tiles.
//   * K is walked in chunks of CC frame-view channels x KT taps.  Both
//     operands of a chunk are staged through LDS, double-buffered: the global
//     loads of chunk q+1 are issued into registers before the MFMAs of chunk q
//     and written to the other LDS buffer after them, so one barrier per chunk
//     separates staging from compute and HBM/L2 latency hides under MFMA.
//   * The PReLU (and the optional per-item input scale) is applied while
//     staging the input window, so the KT-tap re-reads of a sample hit LDS.
//   * Lane half h = lane>>5 owns channel 2*cp + h of the chunk at the same
//     tap, so every B-fragment read is 32 consecutive floats of one LDS row
//     (conflict-free ds_read_b32) and no per-step index decode is needed.  The
//     weights are packed once on the host in exactly that per-lane order
//     (ou_conv_pack), so A-fragment reads are lane-linear too.
//   * Epilogue (bias, zero-fill, residual, FiLM, residual) on the accumulator
//     registers; each 32-lane half stores one contiguous 128-B row segment.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "../../include/ouhip.h"
#include "ou_common.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int kCinAlign = 64;   // packed weights pad the channel axis to this

// Tile: 4 waves as WM x WN x WK; each wave owns MR x NR MFMA tiles of 32 x 32
// (register blocking) over its share (1/WK) of every K chunk.
// P = 0: f32 operands (v_mfma_f32_32x32x2_f32).  P = 1: split-f16 operands
// (v_mfma_f32_32x32x16_f16, three passes per k-step, see conv_kernel).
// P = 2: plain f16 operands (the hi halves only, one pass; f32 accumulation).
template <int KT, int CC, int WM, int WN, int WK, int MR, int NR, int P = 0>
struct Cfg {
    static constexpr int BM = 32 * WM * MR;
    static constexpr int BN = 32 * NR * WN;
    static constexpr int W = BN + KT - 1;            // staged frames per chunk
    static constexpr int HALF = CC / 2;              // channel pairs per chunk
    static constexpr int HQ = HALF / 4;              // 4-pair groups per chunk
    static constexpr int CPW = HQ / WK;              // 4-pair groups per wave
    static constexpr int HQ8 = HALF / 8;             // P: 8-pair groups per chunk (one f16 k-step)
    static constexpr int CPW8 = P ? HQ8 / WK : 0;     // P: 8-pair groups per wave
    // X row stride in elements: f32 CC + 4 (SX/4 odd), f16 CC + 8 (SX/8 odd);
    // the f16 image holds two planes (hi, lo) of W * SX halves = W * SX floats
    static constexpr int SX = P ? CC + 8 : CC + 4;
    static constexpr int XG = W * CC / 4;            // float4 groups of X per chunk
    static constexpr int XE = (XG + 255) / 256;      // per thread
    static constexpr int AG = WM * MR * HQ * KT * 64;  // float4 of A per chunk
    static constexpr int AGL = P == 2 ? AG / 2 : AG;  // float4 of A staged (f16: hi halves only)
    static constexpr int AE = (AGL + 255) / 256;
    static constexpr int XBUF = W * SX;
    static constexpr int STAGE = XBUF + AG * 4;
    static constexpr int RED = (WK - 1) * WM * WN * MR * NR * 16 * 64;
    static constexpr int LDS1 = STAGE > RED ? STAGE : RED;            // one chunk
    static constexpr int LDS2 = 2 * STAGE > RED ? 2 * STAGE : RED;    // double-buffered
};

constexpr int kSentinel = 0x7ffffff0;   // byte offset past any buffer: loads return 0
// tile bit 16: m-groups fastest in the workgroup order (ou_xcd_block_m), for
// inputs much larger than the weights; the one-tile and register-streamed kernels
constexpr int kMajBit = 1 << 16;

// Diagnostic build only (-DOU_CONV_STAMPS, tools/conv_bench.py --stamps):
// thread 0 of each of the first kStampWGs workgroups sums s_memtime deltas
// per phase: prologue, load issue, MFMA, staging stores, barrier, split-K
// reduce + epilogue.
#ifdef OU_CONV_STAMPS
constexpr int kStampWGs = 4096;
constexpr int kStampPhases = 8;
__device__ uint64_t g_conv_stamps[kStampWGs * kStampPhases];
#define OU_CSTAMP_INIT uint64_t cst_[kStampPhases] = {}; uint64_t ctp_ = __builtin_amdgcn_s_memtime(); \
    cst_[6] = __builtin_amdgcn_s_memrealtime();
#define OU_CSTAMP(i) do { const uint64_t n_ = __builtin_amdgcn_s_memtime(); cst_[i] += n_ - ctp_; ctp_ = n_; } while (0)
#define OU_CSTAMP_SAVE                                                                         \
    do {                                                                                       \
        const int wg_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);        \
        cst_[7] = __builtin_amdgcn_s_memrealtime();                                            \
        if (threadIdx.x == 0 && wg_ < kStampWGs)                                               \
            for (int i_ = 0; i_ < kStampPhases; ++i_) g_conv_stamps[wg_ * kStampPhases + i_] = cst_[i_]; \
    } while (0)
// warp-specialised kernel: MFMA wave 0 -> slots 0-7 (0 prefetch/setup, 1 MFMA,
// 2 epilogue, 3 tick barrier, 4 first barrier, 6/7 start/end realtime), staging
// wave 0 -> slots 8-15 (8 DMA issue, 9 vmcnt wait, 10 barrier, 14/15 realtime)
#define OU_WSTAMP_INIT uint64_t wst_[8] = {}; uint64_t wtp_ = __builtin_amdgcn_s_memtime(); \
    wst_[6] = __builtin_amdgcn_s_memrealtime();
#define OU_WSTAMP(i) do { const uint64_t n_ = __builtin_amdgcn_s_memtime(); wst_[i] += n_ - wtp_; wtp_ = n_; } while (0)
#define OU_WSTAMP_SAVE(cond, base)                                                              \
    do {                                                                                        \
        wst_[7] = __builtin_amdgcn_s_memrealtime();                                             \
        if ((cond) && blockIdx.x < kStampWGs / 2)                                               \
            for (int i_ = 0; i_ < 8; ++i_) g_conv_stamps[blockIdx.x * 16 + (base) + i_] = wst_[i_]; \
    } while (0)
#else
#define OU_CSTAMP_INIT
#define OU_CSTAMP(i) do { } while (0)
#define OU_CSTAMP_SAVE do { } while (0)
#define OU_WSTAMP_INIT
#define OU_WSTAMP(i) do { } while (0)
#define OU_WSTAMP_SAVE(cond, base) do { } while (0)
#endif

// LDS images of one K chunk (CC frame-view channels x KT taps):
//   X  [frame w][h * HALF + p]  = PReLU(x'[2 p + h][t0 + w])     row stride SX
//   A  [m-tile][p / 4][tap][lane][p % 4]  (the packed global order, copied)
// so one ds_read_b128 gives a lane the operands of 4 consecutive k-steps
// (channel pairs p .. p+3 at one tap) for both A and B, conflict-free.
//
// Split-f16 form (P = 1).  Every operand is split as v = hi + lo * 2^-11 with
// hi = f16(v) and lo = f16((v - hi) * 2^11) (the weights on the host, the
// PReLU'd input while it is staged), and the product is taken as
//   a b ~= ha hb + (ha lb + la hb) * 2^-11        (la lb ~ 2^-22 |a b| dropped)
// on v_mfma_f32_32x32x16_f16: exact f16 products, f32 accumulation, the main
// and the cross terms in two accumulators that are combined (exact powers of
// two) before the epilogue.  Representation error ~2^-22 relative, i.e. f32
// class (the f32 MFMA rounds at 2^-24), at 3 x 32 instead of 8 x 64 MFMA
// cycles per 16 k-steps.  The weights carry a per-layer power-of-two scale
// (d.w_unscale undoes it) that keeps them in f16's normal range; the staged
// activations must stay below 2^15 in magnitude (the engine keeps the f32
// form for the STFT and mel layers, whose inputs are unbounded powers).
// LDS planes: X [frame][h * HALF + p] of hi, then of lo (halves); A the packed
// global order [m-tile][8-pair group][hi | lo][tap][lane][8 halves].
// Input exponent.  The input is staged as x * 2^-s (exact), s = the layer's
// d.xs_shift (the engine's default 6 = kSplitShift: |x| < 2^21 stays in f16's
// range, |x| >= 2^-8 keeps the full 2^-22 relative precision and smaller
// values an absolute error <= 2^-29).  A staged finite |x| 2^-s >= 2^15 sets
// range code 1 in *d.status (ou_range_flag): the host widens that layer's s
// and reruns the enhance.  ou_conv_pack_split's w_unscale assumes s = 6; a
// kernel scales its result by 2^(s - 6) more.
constexpr int kSplitShift = 6;
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef uint32_t ou_u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t ou_u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));

// Output row m -> (channel co, phase ph) of a transposed conv's pixel
// shuffle.  rout > 0: phase-major rows (m = ph cout + co); rout < 0:
// channel-major rows (m = co |rout| + ph), so a lane's 4 consecutive
// accumulator rows hold consecutive output samples of one or two channels
// (the epilogue then moves them with one 16-B / two 8-B accesses).
__device__ __forceinline__ void ou_row_map(int m, int rout, int cout, int& co, int& ph)
{
    if (rout < 0) {
        co = m / -rout;
        ph = m - co * -rout;
    } else {
        ph = rout > 1 ? m / cout : 0;
        co = m - ph * cout;
    }
}

// Epilogue of one wave's MR x NR accumulator tiles (scaled, K complete):
// bias, zero-fill past valid_len, residual 1, FiLM, residual 2, the rout
// pixel shuffle and the store.  mtb: the wave's first 32-row m-tile; ub: the
// first output frame of its columns.
//
// Two phases: conv_epi_load issues every load the tile's epilogue needs (bias,
// FiLM, both residuals) into registers, conv_epi_store finishes and stores.
// Branch-free: every out-of-range element gets a sentinel offset, so its
// buffer load returns 0 and its buffer store is dropped.  A kernel with work
// between the two (conv_rkernel's K-split reduction through LDS) issues the
// loads first, so their latency overlaps that work; conv_epilogue runs both.
// Split-image output (ou_conv_desc.sy): the next conv's operand, PReLU'd,
// scaled by 2^-sy_shift and split into f16 hi / lo, in the blocked layout
// [c / 32][t][hi | lo][c % 32] (one 128-B row per 32-channel block and sample).
struct SplitOut {
    __amdgpu_buffer_rsrc_t rs;
    int rows;
    float scale, slope;
};

__device__ __forceinline__ SplitOut split_ctx(const ou_conv_desc& d, int b, int cout)
{
    SplitOut s;
    const bool on = d.sy != nullptr;
    s.rs = ou_rsrc(on ? (const char*)d.sy + (int64_t)b * d.sy_bstride : (const char*)d.y,
                   on ? (int64_t)((cout + 31) / 32) * d.sy_rows * 128 : 0);
    s.rows = d.sy_rows;
    s.scale = ou_exp2i(-d.sy_shift);
    s.slope = d.sy_slope;
    return s;
}

// 4 consecutive channels co0 .. co0 + 3 (co0 % 4 == 0) of sample t: 8 B of
// hi and 8 B of lo (the two lane halves of an accumulator register group
// hold channels co0 and co0 + 4: one 16-B piece of the row per instruction)
__device__ __forceinline__ void split_store4(const SplitOut& s, int co0, int t, bool ok, float v0, float v1,
                                             float v2, float v3, float& omax)
{
    const int off = ok ? ((co0 >> 5) * s.rows + t) * 128 + (co0 & 31) * 2 : kSentinel;
    ou_split_store4(s.rs, off, ok, v0, v1, v2, v3, s.scale, s.slope, omax);
}

struct EpiCtx {
    int M, rout, cout, ylen;
    __amdgpu_buffer_rsrc_t ys, r1s, r2s, bs, fs;
    bool has_r1, has_r2, has_fm, vec, has_sy;
    float s1e, s2e, fadd;
    SplitOut so;
};

__device__ __forceinline__ EpiCtx epi_ctx(const ou_conv_desc& d, int b)
{
    EpiCtx c;
    c.M = d.m;
    c.rout = d.rout < 0 ? -d.rout : d.rout;   // output samples per frame
    c.cout = c.M / c.rout;
    const int yrows = c.cout;
    c.ylen = d.out_len;
    c.ys = ou_rsrc(d.y + (int64_t)b * d.y_bstride, (int64_t)yrows * d.y_cstride * 4);
    c.r1s = ou_rsrc(d.res1 ? d.res1 + (int64_t)b * d.r1_bstride : d.y, d.res1 ? (int64_t)yrows * d.r1_cstride * 4 : 0);
    c.r2s = ou_rsrc(d.res2 ? d.res2 + (int64_t)b * d.r2_bstride : d.y, d.res2 ? (int64_t)yrows * d.r2_cstride * 4 : 0);
    // absent operands get zero-size resources (their loads return 0): every
    // load is unconditional -- a per-element `ptr ? load : default` makes hipcc
    // branch around each load and drain vmcnt(0) per element
    c.has_r1 = d.res1 != nullptr, c.has_r2 = d.res2 != nullptr, c.has_fm = d.film != nullptr;
    // branch-free epilogue: an absent operand loads 0 and meets a unit scale
    c.s1e = c.has_r1 ? d.s1 : 1.f, c.s2e = c.has_r2 ? d.s2 : 1.f, c.fadd = c.has_fm ? 0.f : 1.f;
    c.bs = ou_rsrc(d.bias, d.bias ? (int64_t)c.cout * 4 : 0);
    c.fs = ou_rsrc(c.has_fm ? d.film + (int64_t)b * d.film_bstride : d.y, c.has_fm ? (int64_t)c.cout * 8 : 0);
    // vector path: channel-major rows at rout 2 or a multiple of 4, with every
    // row start 8-B / 16-B aligned (uniform over the launch)
    const int rout = c.rout;
    auto al = [&](const float* p, int64_t bst, int64_t cst) {
        const int A = rout == 2 ? 2 : 4;   // 8-B (rout 2) / 16-B accesses
        return !p || (((uintptr_t)p % (4 * A)) == 0 && bst % A == 0 && cst % A == 0);
    };
    c.vec = d.rout < 0 && (rout == 2 || rout % 4 == 0) && c.M % 4 == 0 && al(d.y, d.y_bstride, d.y_cstride) &&
            al(d.res1, d.r1_bstride, d.r1_cstride) && al(d.res2, d.r2_bstride, d.r2_cstride);
    c.has_sy = d.sy != nullptr;   // host-checked: rout 1, m % 32 == 0
    c.so = split_ctx(d, b, c.cout);
    return c;
}

template <int MR, int NR>
struct EpiPre {
    float bias[MR][16], fa[MR][16], fb[MR][16];
    float v1[MR][NR][16], v2[MR][NR][16];
    bool vec[MR][NR];   // this (m-tile, frame tile) takes the vector path
};

template <int MR, int NR>
__device__ __forceinline__ void conv_epi_load(const ou_conv_desc& d, const EpiCtx& c, int mtb, int ub, int lane,
                                              EpiPre<MR, NR>& e)
{
    const int h = lane >> 5, l32 = lane & 31;
    const int M = c.M, rout = c.rout, cout = c.cout, ylen = c.ylen;
#pragma unroll
    for (int mr = 0; mr < MR; ++mr) {
        const int mt = mtb + mr;
        int co[16], ph[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = min(mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, M - 1);
            ou_row_map(m, d.rout, cout, co[r], ph[r]);
        }
        // absent operands: one uniform branch around the whole group of loads
        // (never a per-element select between a load and a default)
        if (d.bias) {
#pragma unroll
            for (int r = 0; r < 16; ++r) e.bias[mr][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(c.bs, co[r] * 4, 0, 0));
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) e.bias[mr][r] = 0.f;
        }
        if (c.has_fm) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                e.fa[mr][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(c.fs, co[r] * 4, 0, 0));
                e.fb[mr][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(c.fs, (cout + co[r]) * 4, 0, 0));
            }
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) e.fa[mr][r] = 0.f, e.fb[mr][r] = 0.f;
        }
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
            const int u = ub + nr * 32 + l32;
            e.vec[mr][nr] = false;
            if (c.vec) {
                // channel-major rows at rout 2 or 4 k: register group g (rows
                // m0 = 8 g + 4 h + j, j < 4) holds 4 consecutive samples
                // u rout + ph(m0) .. of one channel (rout 4 k) or 2 + 2 of two
                // channels (rout 2) -- one 16-B or two 8-B accesses per group
                // and tensor, consecutive lanes on consecutive frames
                const int t0 = u * rout;
                const bool uok = u < d.f0 + d.n_frames && t0 < ylen;
                if (__all(!uok || t0 + rout <= ylen)) {
                    e.vec[mr][nr] = true;
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const bool ok = uok && mt * 32 + 8 * g + 4 * h < M;
#pragma unroll
                        for (int sv = 0; sv < 4 / 4 + (rout == 2); ++sv) {
                            const int cc = co[4 * g + 2 * sv];
                            const int o1 = ok ? (cc * (int)d.r1_cstride + t0 + ph[4 * g + 2 * sv]) * 4 : kSentinel;
                            const int o2 = ok ? (cc * (int)d.r2_cstride + t0 + ph[4 * g + 2 * sv]) * 4 : kSentinel;
                            if (rout != 2) {
                                const auto a1 = __builtin_amdgcn_raw_buffer_load_b128(c.r1s, o1, 0, 0);
                                const auto a2 = __builtin_amdgcn_raw_buffer_load_b128(c.r2s, o2, 0, 0);
#pragma unroll
                                for (int j = 0; j < 4; ++j)
                                    e.v1[mr][nr][4 * g + j] = __uint_as_float(a1[j]), e.v2[mr][nr][4 * g + j] = __uint_as_float(a2[j]);
                            } else {
                                const auto a1 = __builtin_amdgcn_raw_buffer_load_b64(c.r1s, o1, 0, 0);
                                const auto a2 = __builtin_amdgcn_raw_buffer_load_b64(c.r2s, o2, 0, 0);
#pragma unroll
                                for (int j = 0; j < 2; ++j)
                                    e.v1[mr][nr][4 * g + 2 * sv + j] = __uint_as_float(a1[j]),
                                    e.v2[mr][nr][4 * g + 2 * sv + j] = __uint_as_float(a2[j]);
                            }
                        }
                    }
                    continue;
                }
            }
            int off[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int t = u * rout + ph[r];
                const bool ok = m < M && u < d.f0 + d.n_frames && t < ylen;
                off[r] = ok ? t : -1;   // column; row offsets differ per tensor
            }
            if (c.has_r1) {
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    e.v1[mr][nr][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                        c.r1s, off[r] >= 0 ? (co[r] * (int)d.r1_cstride + off[r]) * 4 : kSentinel, 0, 0));
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) e.v1[mr][nr][r] = 0.f;
            }
            if (c.has_r2) {
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    e.v2[mr][nr][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                        c.r2s, off[r] >= 0 ? (co[r] * (int)d.r2_cstride + off[r]) * 4 : kSentinel, 0, 0));
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) e.v2[mr][nr][r] = 0.f;
            }
        }
    }
}

template <int MR, int NR>
__device__ __forceinline__ void conv_epi_store(const ou_conv_desc& d, const EpiCtx& c, int mtb, int ub,
                                               floatx16 (&acc)[MR][NR], const EpiPre<MR, NR>& e, int lane)
{
    const int h = lane >> 5, l32 = lane & 31;
    const int M = c.M, rout = c.rout, cout = c.cout, ylen = c.ylen;
    float somax = 0.f;  // max |split-image value| (range flag)
#pragma unroll
    for (int mr = 0; mr < MR; ++mr) {
        const int mt = mtb + mr;
        int co[16], ph[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = min(mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, M - 1);
            ou_row_map(m, d.rout, cout, co[r], ph[r]);
        }
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
            const int u = ub + nr * 32 + l32;
            if (e.vec[mr][nr]) {
                const int t0 = u * rout;
                const bool uok = u < d.f0 + d.n_frames && t0 < ylen;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const bool ok = uok && mt * 32 + 8 * g + 4 * h < M;
                    float val[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = 4 * g + j;
                        float v = acc[mr][nr][r] + e.bias[mr][r];
                        if (t0 + ph[r] >= d.valid_len) v = 0.f;
                        v = (v + e.v1[mr][nr][r]) * c.s1e;
                        v = (e.fa[mr][r] + c.fadd) * v + e.fb[mr][r];
                        v = (v + e.v2[mr][nr][r]) * c.s2e;
                        val[j] = v;
                    }
#pragma unroll
                    for (int sv = 0; sv < 4 / 4 + (rout == 2); ++sv) {
                        const int cc = co[4 * g + 2 * sv];
                        const int oy = ok ? (cc * (int)d.y_cstride + t0 + ph[4 * g + 2 * sv]) * 4 : kSentinel;
                        if (rout != 2)
                            __builtin_amdgcn_raw_buffer_store_b128(
                                ou_u32x4{__float_as_uint(val[0]), __float_as_uint(val[1]), __float_as_uint(val[2]),
                                         __float_as_uint(val[3])},
                                c.ys, oy, 0, 0);
                        else
                            __builtin_amdgcn_raw_buffer_store_b64(
                                ou_u32x2{__float_as_uint(val[2 * sv]), __float_as_uint(val[2 * sv + 1])}, c.ys, oy, 0, 0);
                    }
                }
                continue;
            }
            float sv[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int t = u * rout + ph[r];
                const bool ok = m < M && u < d.f0 + d.n_frames && t < ylen;
                float v = acc[mr][nr][r] + e.bias[mr][r];
                if ((ok ? t : -1) >= d.valid_len) v = 0.f;
                v = (v + e.v1[mr][nr][r]) * c.s1e;
                v = (e.fa[mr][r] + c.fadd) * v + e.fb[mr][r];
                v = (v + e.v2[mr][nr][r]) * c.s2e;
                sv[r] = v;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), c.ys,
                                                      ok ? (co[r] * (int)d.y_cstride + t) * 4 : kSentinel, 0, 0);
            }
            if (c.has_sy) {   // rout 1: row m = channel, sample u
                const bool ok = mt * 32 < M && u < d.f0 + d.n_frames && u < ylen;
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    split_store4(c.so, mt * 32 + 8 * g + 4 * h, u, ok, sv[4 * g], sv[4 * g + 1], sv[4 * g + 2],
                                 sv[4 * g + 3], somax);
            }
        }
    }
    if (c.has_sy) ou_range_flag(d.status, somax, 2, lane);
}

// The one-phase epilogue of the chunked / persistent kernels: per m-tile
// and frame tile, its loads then its stores (live ranges stay one tile's
// worth -- those kernels hold MR x NR tiles).
// col: the lane's frame within its 32-frame tile (default lane & 31; the FIR
// down kernel's B rows are a permutation of the frames, conv_fdkernel)
template <int MR, int NR>
__device__ __forceinline__ void conv_epilogue(const ou_conv_desc& d, int b, int mtb, int ub,
                                              floatx16 (&acc)[MR][NR], int lane, int col = -1)
{
    const int h = lane >> 5, l32 = col >= 0 ? col : lane & 31;
    // Branch-free: every out-of-range element gets a sentinel offset, so its
    // buffer load returns 0 and its buffer store is dropped.  All residual
    // loads of the tile are issued before any arithmetic, so their latency is
    // paid once, not once per row.
    const int M = d.m;
    const int rout = d.rout < 0 ? -d.rout : d.rout;   // output samples per frame
    const int cout = M / rout;
    const int yrows = cout;
    const int ylen = d.out_len;
    const __amdgpu_buffer_rsrc_t ys = ou_rsrc(d.y + (int64_t)b * d.y_bstride, (int64_t)yrows * d.y_cstride * 4);
    const __amdgpu_buffer_rsrc_t r1s = ou_rsrc(d.res1 ? d.res1 + (int64_t)b * d.r1_bstride : d.y, d.res1 ? (int64_t)yrows * d.r1_cstride * 4 : 0);
    const __amdgpu_buffer_rsrc_t r2s = ou_rsrc(d.res2 ? d.res2 + (int64_t)b * d.r2_bstride : d.y, d.res2 ? (int64_t)yrows * d.r2_cstride * 4 : 0);
    // absent operands get zero-size resources (their loads return 0): every
    // load is unconditional -- a per-element `ptr ? load : default` makes hipcc
    // branch around each load and drain vmcnt(0) per element
    const bool has_r1 = d.res1 != nullptr, has_r2 = d.res2 != nullptr, has_fm = d.film != nullptr;
    // branch-free epilogue: an absent operand loads 0 and meets a unit scale
    const float s1e = has_r1 ? d.s1 : 1.f, s2e = has_r2 ? d.s2 : 1.f, fadd = has_fm ? 0.f : 1.f;
    const __amdgpu_buffer_rsrc_t bs = ou_rsrc(d.bias, d.bias ? (int64_t)cout * 4 : 0);
    const __amdgpu_buffer_rsrc_t fs = ou_rsrc(has_fm ? d.film + (int64_t)b * d.film_bstride : d.y,
                                              has_fm ? (int64_t)cout * 8 : 0);
    // vector path: channel-major rows at rout 2 or a multiple of 4, with every
    // row start 8-B / 16-B aligned (uniform over the launch)
    auto al = [&](const float* p, int64_t bst, int64_t cst) {
        const int A = rout == 2 ? 2 : 4;   // 8-B (rout 2) / 16-B accesses
        return !p || (((uintptr_t)p % (4 * A)) == 0 && bst % A == 0 && cst % A == 0);
    };
    const bool vec = d.rout < 0 && (rout == 2 || rout % 4 == 0) && M % 4 == 0 && al(d.y, d.y_bstride, d.y_cstride) &&
                     al(d.res1, d.r1_bstride, d.r1_cstride) && al(d.res2, d.r2_bstride, d.r2_cstride);
    const SplitOut so = split_ctx(d, b, cout);
    float somax = 0.f;
#pragma unroll
    for (int mr = 0; mr < MR; ++mr) {
        const int mt = mtb + mr;
        int co[16], ph[16];
        float bias[16], fa[16], fb[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = min(mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, M - 1);
            ou_row_map(m, d.rout, cout, co[r], ph[r]);
        }
        // absent operands: one uniform branch around the whole group of loads
        // (never a per-element select between a load and a default)
        if (d.bias) {
#pragma unroll
            for (int r = 0; r < 16; ++r) bias[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bs, co[r] * 4, 0, 0));
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) bias[r] = 0.f;
        }
        if (has_fm) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                fa[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(fs, co[r] * 4, 0, 0));
                fb[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(fs, (cout + co[r]) * 4, 0, 0));
            }
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                fa[r] = 0.f;
                fb[r] = 0.f;
            }
        }
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
            const int u = ub + nr * 32 + l32;
            if (vec) {
                // channel-major rows at rout 2 or 4 k: register group g (rows
                // m0 = 8 g + 4 h + j, j < 4) holds 4 consecutive samples
                // u rout + ph(m0) .. of one channel (rout 4 k) or 2 + 2 of two
                // channels (rout 2) -- one 16-B or two 8-B accesses per group
                // and tensor, consecutive lanes on consecutive frames
                const int t0 = u * rout;
                const bool uok = u < d.f0 + d.n_frames && t0 < ylen;
                if (__all(!uok || t0 + rout <= ylen)) {
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const bool ok = uok && mt * 32 + 8 * g + 4 * h < M;
                        float v1[4], v2[4], val[4];
#pragma unroll
                        for (int sv = 0; sv < 4 / 4 + (rout == 2); ++sv) {
                            const int c = co[4 * g + 2 * sv];
                            const int o1 = ok ? (c * (int)d.r1_cstride + t0 + ph[4 * g + 2 * sv]) * 4 : kSentinel;
                            const int o2 = ok ? (c * (int)d.r2_cstride + t0 + ph[4 * g + 2 * sv]) * 4 : kSentinel;
                            if (rout != 2) {
                                const auto a1 = __builtin_amdgcn_raw_buffer_load_b128(r1s, o1, 0, 0);
                                const auto a2 = __builtin_amdgcn_raw_buffer_load_b128(r2s, o2, 0, 0);
#pragma unroll
                                for (int j = 0; j < 4; ++j) v1[j] = __uint_as_float(a1[j]), v2[j] = __uint_as_float(a2[j]);
                            } else {
                                const auto a1 = __builtin_amdgcn_raw_buffer_load_b64(r1s, o1, 0, 0);
                                const auto a2 = __builtin_amdgcn_raw_buffer_load_b64(r2s, o2, 0, 0);
#pragma unroll
                                for (int j = 0; j < 2; ++j)
                                    v1[2 * sv + j] = __uint_as_float(a1[j]), v2[2 * sv + j] = __uint_as_float(a2[j]);
                            }
                        }
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int r = 4 * g + j;
                            float v = acc[mr][nr][r] + bias[r];
                            if (t0 + ph[r] >= d.valid_len) v = 0.f;
                            v = (v + v1[j]) * s1e;
                            v = (fa[r] + fadd) * v + fb[r];
                            v = (v + v2[j]) * s2e;
                                val[j] = v;
                        }
#pragma unroll
                        for (int sv = 0; sv < 4 / 4 + (rout == 2); ++sv) {
                            const int c = co[4 * g + 2 * sv];
                            const int oy = ok ? (c * (int)d.y_cstride + t0 + ph[4 * g + 2 * sv]) * 4 : kSentinel;
                            if (rout != 2)
                                __builtin_amdgcn_raw_buffer_store_b128(
                                    ou_u32x4{__float_as_uint(val[0]), __float_as_uint(val[1]), __float_as_uint(val[2]),
                                             __float_as_uint(val[3])},
                                    ys, oy, 0, 0);
                            else
                                __builtin_amdgcn_raw_buffer_store_b64(
                                    ou_u32x2{__float_as_uint(val[2 * sv]), __float_as_uint(val[2 * sv + 1])}, ys, oy, 0, 0);
                        }
                    }
                    continue;
                }
            }
            int off[16];
            float v1[16], v2[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int t = u * rout + ph[r];
                const bool ok = m < M && u < d.f0 + d.n_frames && t < ylen;
                off[r] = ok ? t : -1;   // column; row offsets differ per tensor
            }
            if (has_r1) {
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    v1[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                        r1s, off[r] >= 0 ? (co[r] * (int)d.r1_cstride + off[r]) * 4 : kSentinel, 0, 0));
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) v1[r] = 0.f;
            }
            if (has_r2) {
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    v2[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                        r2s, off[r] >= 0 ? (co[r] * (int)d.r2_cstride + off[r]) * 4 : kSentinel, 0, 0));
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) v2[r] = 0.f;
            }
            float sv[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float v = acc[mr][nr][r] + bias[r];
                if (off[r] >= d.valid_len) v = 0.f;
                v = (v + v1[r]) * s1e;
                v = (fa[r] + fadd) * v + fb[r];
                v = (v + v2[r]) * s2e;
                sv[r] = v;
                __builtin_amdgcn_raw_buffer_store_b32(
                    __float_as_uint(v), ys, off[r] >= 0 ? (co[r] * (int)d.y_cstride + off[r]) * 4 : kSentinel, 0, 0);
            }
            if (d.sy) {   // split image of the next conv's operand (rout 1: row m = channel, sample u)
                const bool ok = mt * 32 < M && u < d.f0 + d.n_frames && u < ylen;
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    split_store4(so, mt * 32 + 8 * g + 4 * h, u, ok, sv[4 * g], sv[4 * g + 1], sv[4 * g + 2],
                                 sv[4 * g + 3], somax);
            }
        }
    }
    if (d.sy) ou_range_flag(d.status, somax, 2, lane);
}

//
// K slices (tile bits 12-13, S = 2..8; for grids too small to fill the chip):
// ksmode 1 runs the workgroups of slice ks = blockIdx.z % S over chunks
// [ks n / S, (ks + 1) n / S) and stores their sums to d.ks_ws; ksmode 2 (a
// second launch, so the kernel boundary orders the two) adds the S partial
// sums in slice order -- deterministic -- and runs the epilogue.
template <int KT, int CC, int WM, int WN, int WK, int MR, int NR, int P = 0>
__global__ __launch_bounds__(256) void conv_kernel(ou_conv_desc d, int nchunks, int mtiles,
                                                   int64_t a_mt_stride, int ksmode)
{
    using C = Cfg<KT, CC, WM, WN, WK, MR, NR, P>;
    static_assert(CC % 8 == 0 && C::HQ % WK == 0, "chunk must split into 4-pair groups per wave");
    static_assert(WM * WN * WK == 4, "4 waves per workgroup");
    ou_kernarg_prefetch6();
    static_assert(P || (C::SX / 4) % 2 == 1, "X row stride must be an odd number of 16-B slots");
    static_assert(!P || (CC % 16 == 0 && C::HQ8 % WK == 0 && (C::SX / 8) % 2 == 1),
                  "split-f16: chunk must split into 8-pair groups per wave, odd 16-B row stride");
    OU_DYNAMIC_LDS(float4, lds4);
    float* lds = (float*)lds4;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wn = wave % WN;
    const int wm = (wave / WN) % WM;
    const int wk = wave / (WN * WM);
    const int nks = ksmode ? 1 << ((d.tile >> 12) & 3) : 1;   // K slices per output tile
    int bx, by, bz;
    if (d.tile & kMajBit) ou_xcd_block_m(bx, by, bz); else ou_xcd_block(bx, by, bz);
    const int b = ksmode == 1 ? bz / nks : bz;
    const int ks = ksmode == 1 ? bz - b * nks : 0;
    const int q0 = ksmode == 1 ? ks * nchunks / nks : 0;
    const int q1 = ksmode == 1 ? (ks + 1) * nchunks / nks : nchunks;
    const int n0 = bx * C::BN + d.f0;     // first output frame (global)
    const int mt0 = by * (WM * MR);       // first m-tile of the workgroup
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int R = d.frame;
    const int cin = d.cin;
    const int in_len = d.in_len;
    const int xc = (int)d.x_cstride;
    const float* xb = d.x + (int64_t)b * d.x_bstride;
    const float scale = d.in_scale ? d.in_scale[b] : 1.0f;
    // split-f16 staging / result scales: the layer's staging exponent
    const float xsc = ou_exp2i(-d.xs_shift), su = d.w_unscale * ou_exp2i(d.xs_shift - kSplitShift);
    const float slope = d.slope;
    const float sxs = scale * xsc;   // xsc is a power of two: x (scale xsc) == (x scale) xsc exactly
    const int t0 = n0 - d.pad;

    // ---- staging geometry, fixed for the whole K loop ----------------------
    // X group g -> frame w = g % W, lane half hh, 4-pair group cq; its four
    // elements are chunk channels 8 cq + 2 j + hh (j = 0..3) at frame w.
    int xdst[C::XE];
    int xsrc[C::XE];   // R == 1: byte offset of element j = 0 (or kSentinel); R > 1: sample of phase 0
    int xcl[C::XE];    // chunk channel of element j = 0
#pragma unroll
    for (int e = 0; e < C::XE; ++e) {
        const int g = tid + e * 256;
        const int w = g % C::W;
        const int r = g / C::W;
        const int hh = r & 1, cq = r >> 1;
        const bool valid = g < C::XG;
        xdst[e] = valid ? w * C::SX + hh * C::HALF + 4 * cq : -1;
        xcl[e] = 8 * cq + hh;
        if (R == 1) {
            const int pos = t0 + w + d.shift;
            xsrc[e] = (valid && pos >= 0 && pos < in_len) ? (xcl[e] * xc + pos) * 4 : kSentinel;
        } else {
            xsrc[e] = (t0 + w) * R + d.shift;
        }
    }
    // packed weights: (mtiles * a_mt_stride) floats; one buffer resource
    const __amdgpu_buffer_rsrc_t wrs = ou_rsrc(d.w, (int64_t)mtiles * a_mt_stride * 4);
    int aoff[C::AE], adst[C::AE];   // global float offset and LDS float4 slot of each staged float4
#pragma unroll
    for (int e = 0; e < C::AE; ++e) {
        const int f = min(tid + e * 256, C::AGL - 1);
        int ml, r;
        if constexpr (P == 2) {   // hi blocks only: [g8][hi][tap][lane] of each m-tile
            ml = f / (C::HQ8 * KT * 64);
            const int rh = f - ml * (C::HQ8 * KT * 64);
            const int g8 = rh / (KT * 64);
            r = g8 * 2 * KT * 64 + (rh - g8 * KT * 64);
        } else {
            ml = f / (C::HQ * KT * 64);
            r = f - ml * (C::HQ * KT * 64);
        }
        const int mtg = min(mt0 + ml, mtiles - 1);   // rows past M are computed, never stored
        aoff[e] = (int)(mtg * a_mt_stride) + r * 4;
        adst[e] = ml * (C::HQ * KT * 64) + r;
    }

    float xr[4 * C::XE];   // plain float arrays: float4 arrays end up in scratch
    float ar[4 * C::AE];

#define OU_LOAD_CHUNK(q)                                                                       \
    {                                                                                          \
        const int q_ = (q);                                                                    \
        if (R == 1) {                                                                          \
            const int nch = cin - q_ * CC;                                                     \
            const __amdgpu_buffer_rsrc_t rs =                                                  \
                ou_rsrc(xb + (int64_t)q_ * CC * xc, nch > 0 ? (int64_t)nch * xc * 4 : 0);      \
            _Pragma("unroll") for (int e = 0; e < C::XE; ++e) {                                \
                const unsigned o = (unsigned)xsrc[e];                                          \
                const unsigned st = 8u * (unsigned)xc;                                         \
                _Pragma("unroll") for (int j = 0; j < 4; ++j) xr[4 * e + j] =                  \
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o + j * st, 0, 0));   \
            }                                                                                  \
        } else if (cin % CC == 0) {                                                            \
            /* phase-major frame view: the chunk is one phase ph of channels */                \
            /* ci0 .. ci0+CC-1: x'[ci0 + cl][t] = x[ci0 + cl][t*R + ph + shift] */              \
            const int ph = (q_ * CC) / cin;                                                    \
            const int ci0 = q_ * CC - ph * cin;                                                \
            const __amdgpu_buffer_rsrc_t rs =                                                  \
                ou_rsrc(xb + (int64_t)ci0 * xc, (int64_t)(cin - ci0) * xc * 4);                \
            _Pragma("unroll") for (int e = 0; e < C::XE; ++e) {                                \
                const int pos = xsrc[e] + ph;                                                  \
                const bool ok = xdst[e] >= 0 && pos >= 0 && pos < in_len;                      \
                _Pragma("unroll") for (int j = 0; j < 4; ++j) xr[4 * e + j] =                  \
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(                      \
                        rs, ok ? ((xcl[e] + 2 * j) * xc + pos) * 4 : kSentinel, 0, 0));        \
            }                                                                                  \
        } else {                                                                               \
            const __amdgpu_buffer_rsrc_t rs =                                                  \
                ou_rsrc(xb, (int64_t)cin * xc * 4);                                            \
            _Pragma("unroll") for (int e = 0; e < C::XE; ++e) {                                \
                _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                \
                    const int cq = q_ * CC + xcl[e] + 2 * j;                                   \
                    const int ph = cq / cin;                                                   \
                    const int ci = cq - ph * cin;                                              \
                    const int pos = xsrc[e] + ph;                                              \
                    const int off = (xdst[e] >= 0 && ph < R && pos >= 0 && pos < in_len)       \
                                        ? (ci * xc + pos) * 4                                  \
                                        : kSentinel;                                           \
                    xr[4 * e + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0)); \
                }                                                                              \
            }                                                                                  \
        }                                                                                      \
        _Pragma("unroll") for (int e = 0; e < C::AE; ++e) {                                    \
            /* voffset fixed per lane, chunk offset in the scalar soffset: no */                \
            /* per-chunk VGPR address math (which made the compiler drain vmcnt) */            \
            const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(                             \
                wrs, aoff[e] * 4, q_ * (C::HQ * KT * 256 * 4), 0);                            \
            ar[4 * e] = __uint_as_float(v4[0]);                                                \
            ar[4 * e + 1] = __uint_as_float(v4[1]);                                            \
            ar[4 * e + 2] = __uint_as_float(v4[2]);                                            \
            ar[4 * e + 3] = __uint_as_float(v4[3]);                                            \
        }                                                                                      \
    }

#define OU_PRELU(v) ((v) * scale >= 0.f ? (v) * scale : (v) * scale * slope)

#define OU_STORE_CHUNK(buf)                                                                    \
    {                                                                                          \
        float* xs_ = lds + (buf) * C::STAGE;                                                   \
        if constexpr (P) {                                                                     \
            _Float16* xh_ = (_Float16*)xs_;                                                    \
            _Pragma("unroll") for (int e = 0; e < C::XE; ++e) if (xdst[e] >= 0) {              \
                half4_t hi_, lo_;                                                              \
                float v_[4];                                                                   \
                _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                \
                    const float q_ = xr[4 * e + j] * sxs;   /* == PReLU(x scale) xsc: 2^k */   \
                    v_[j] = q_ >= 0.f ? q_ : q_ * slope;                                       \
                }                                                                              \
                omax = fmaxf(omax, fmaxf(fmaxf(__builtin_fabsf(v_[0]), __builtin_fabsf(v_[1])),    \
                                         fmaxf(__builtin_fabsf(v_[2]), __builtin_fabsf(v_[3]))));   \
                _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                \
                    hi_[j] = (_Float16)v_[j];                                                  \
                    lo_[j] = (_Float16)((v_[j] - (float)hi_[j]) * 2048.f);                     \
                }                                                                              \
                *(half4_t*)(xh_ + xdst[e]) = hi_;                                              \
                if constexpr (P == 1) *(half4_t*)(xh_ + C::W * C::SX + xdst[e]) = lo_;         \
            }                                                                                  \
        } else {                                                                               \
            _Pragma("unroll") for (int e = 0; e < C::XE; ++e) if (xdst[e] >= 0)                \
                *(float4*)(xs_ + xdst[e]) = make_float4(OU_PRELU(xr[4 * e]), OU_PRELU(xr[4 * e + 1]), \
                                                        OU_PRELU(xr[4 * e + 2]), OU_PRELU(xr[4 * e + 3])); \
        }                                                                                      \
        float4* as_ = (float4*)(xs_ + C::XBUF);                                                \
        _Pragma("unroll") for (int e = 0; e < C::AE; ++e) if (C::AGL % 256 == 0 || tid + e * 256 < C::AGL) \
            as_[adst[e]] = make_float4(ar[4 * e], ar[4 * e + 1], ar[4 * e + 2], ar[4 * e + 3]); \
    }

    floatx16 acc[MR][NR];
    floatx16 accx[P == 1 ? MR : 1][P == 1 ? NR : 1];   // split-f16 cross terms
    float omax = 0.f;                        // split-f16: max |staged input| (range flag)
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    if constexpr (P == 1) {
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
            for (int j = 0; j < NR; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) accx[i][j][r] = 0.f;
    }

    OU_CSTAMP_INIT
    // phase-major frame views (one phase of CC channels per chunk): walk the
    // chunks phase-fastest, so the R chunks that read the same input lines
    // (every R-th sample, each phase in turn) run back to back and hit the
    // caches, instead of R passes over the whole window
    const int cpb = cin / CC;   // channel blocks per phase
    auto qperm = [&](int k) { return (R > 1 && cin % CC == 0) ? (k % R) * cpb + k / R : k; };
    if (ksmode != 2) {
    OU_LOAD_CHUNK(qperm(q0));
    OU_STORE_CHUNK(0);
    __syncthreads();
    OU_CSTAMP(0);
    for (int q = q0; q < q1; ++q) {
        const int cur = (q - q0) & 1;
        if (q + 1 < q1) OU_LOAD_CHUNK(qperm(q + 1));
        OU_CSTAMP(1);
        if constexpr (P) {
            // one step = 8 channel pairs (16 k) at one tap: 3 f16 MFMAs per
            // (mr, nr); fragments of step s + 1 are read during step s
            const _Float16* xh = (const _Float16*)(lds + cur * C::STAGE);
            const half8_t* ap = (const half8_t*)(lds + cur * C::STAGE + C::XBUF) +
                                ((wm * MR) * C::HQ + wk * C::CPW8 * 2) * KT * 64 + lane;
            const _Float16* xp = xh + (wn * 32 * NR + l32) * C::SX + h * C::HALF + 8 * wk * C::CPW8;
            constexpr int NS = C::CPW8 * KT;
            half8_t fa[2][MR], fal[2][MR], fb[2][NR], fbl[2][NR];
            auto frag = [&](int st, half8_t* a, half8_t* al, half8_t* bq, half8_t* bl) {
                const int c8 = st / KT, k = st - (st / KT) * KT;
#pragma unroll
                for (int mr = 0; mr < MR; ++mr) {
                    a[mr] = ap[(mr * C::HQ * KT + (c8 * 2) * KT + k) * 64];
                    if constexpr (P == 1) al[mr] = ap[(mr * C::HQ * KT + (c8 * 2 + 1) * KT + k) * 64];
                }
#pragma unroll
                for (int nr = 0; nr < NR; ++nr) {
                    bq[nr] = *(const half8_t*)(xp + (nr * 32 + k) * C::SX + 8 * c8);
                    if constexpr (P == 1)
                        bl[nr] = *(const half8_t*)(xp + C::W * C::SX + (nr * 32 + k) * C::SX + 8 * c8);
                }
            };
            frag(0, fa[0], fal[0], fb[0], fbl[0]);
#pragma unroll
            for (int st = 0; st < NS; ++st) {
                const int c = st & 1, n = c ^ 1;
                if (st + 1 < NS) frag(st + 1, fa[n], fal[n], fb[n], fbl[n]);
#pragma unroll
                for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                    for (int nr = 0; nr < NR; ++nr) {
                        acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[c][mr], fb[c][nr], acc[mr][nr], 0, 0, 0);
                        if constexpr (P == 1) {
                            accx[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[c][mr], fbl[c][nr], accx[mr][nr], 0, 0, 0);
                            accx[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal[c][mr], fb[c][nr], accx[mr][nr], 0, 0, 0);
                        }
                    }
            }
        } else {
            const float* xs = lds + cur * C::STAGE;
            const float4* ap = (const float4*)(xs + C::XBUF) +
                               ((wm * MR) * C::HQ + wk * C::CPW) * KT * 64 + lane;
            const float* xp = xs + (wn * 32 * NR + l32) * C::SX + h * C::HALF + 4 * wk * C::CPW;
            // software-pipelined: the fragments of step s + 1 are read while
            // the MFMAs of step s run (step = 4 channel pairs at one tap)
            constexpr int NS = C::CPW * KT;
            float4 fa[2][MR], fb[2][NR];
            auto frag = [&](int st, float4* a, float4* bq) {
                const int cpq = st / KT, k = st - (st / KT) * KT;
#pragma unroll
                for (int mr = 0; mr < MR; ++mr) a[mr] = ap[((mr * C::HQ + cpq) * KT + k) * 64];
#pragma unroll
                for (int nr = 0; nr < NR; ++nr)
                    bq[nr] = *(const float4*)(xp + (nr * 32 + k) * C::SX + 4 * cpq);
            };
            frag(0, fa[0], fb[0]);
#pragma unroll
            for (int st = 0; st < NS; ++st) {
                if (st + 1 < NS) frag(st + 1, fa[(st + 1) & 1], fb[(st + 1) & 1]);
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                        for (int nr = 0; nr < NR; ++nr)
                            acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                                fa[st & 1][mr][j], fb[st & 1][nr][j], acc[mr][nr], 0, 0, 0);
            }
        }
        OU_CSTAMP(2);
        if (q + 1 < q1) OU_STORE_CHUNK(cur ^ 1);
        OU_CSTAMP(3);
        __syncthreads();
        OU_CSTAMP(4);
    }
#undef OU_LOAD_CHUNK
#undef OU_STORE_CHUNK
#undef OU_PRELU
    if constexpr (P) {   // range flag, then combine the split-f16 terms (exact powers of two)
        ou_range_flag(d.status, omax, 1, lane);
        const float sx = su * (1.f / 2048.f);
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
            for (int j = 0; j < NR; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    acc[i][j][r] = P == 1 ? fmaf(accx[i][j][r], sx, acc[i][j][r] * su) : acc[i][j][r] * su;
    }

    // ---- intra-workgroup split-K reduction (fixed order: deterministic) ----
    if (WK > 1) {
        float* red = lds;
        const int sub = wm * WN + wn;
        if (wk > 0) {
#pragma unroll
            for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                for (int nr = 0; nr < NR; ++nr)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        red[(((((wk - 1) * WM * WN + sub) * MR + mr) * NR + nr) * 16 + r) * 64 + lane] =
                            acc[mr][nr][r];
        }
        __syncthreads();
        if (wk > 0) return;
#pragma unroll
        for (int j = 1; j < WK; ++j)
#pragma unroll
            for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                for (int nr = 0; nr < NR; ++nr)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        acc[mr][nr][r] +=
                            red[(((((j - 1) * WM * WN + sub) * MR + mr) * NR + nr) * 16 + r) * 64 + lane];
    }

    if (ksmode == 1) {   // this slice's sums -> d.ks_ws, [tile][slice][sub-tile][acc][lane]
        const int64_t tl = ((int64_t)b * gridDim.y + by) * gridDim.x + bx;
        float* pw = d.ks_ws + ((tl * nks + ks) * (WM * WN) + wm * WN + wn) * (MR * NR * 16 * 64) + lane;
#pragma unroll
        for (int mr = 0; mr < MR; ++mr)
#pragma unroll
            for (int nr = 0; nr < NR; ++nr)
#pragma unroll
                for (int r = 0; r < 16; ++r) pw[((mr * NR + nr) * 16 + r) * 64] = acc[mr][nr][r];
        return;
    }
    } else {   // ksmode 2: add the slices' sums in slice order
        if (wk > 0) return;
        const int S = 1 << ((d.tile >> 12) & 3);
        const int64_t tl = ((int64_t)b * gridDim.y + by) * gridDim.x + bx;
        const float* pr = d.ks_ws + (tl * S * (WM * WN) + wm * WN + wn) * (MR * NR * 16 * 64) + lane;
        for (int k = 0; k < S; ++k) {
            const float* pk = pr + (int64_t)k * (WM * WN) * (MR * NR * 16 * 64);
#pragma unroll
            for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                for (int nr = 0; nr < NR; ++nr)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float v = pk[((mr * NR + nr) * 16 + r) * 64];
                        acc[mr][nr][r] = k == 0 ? v : acc[mr][nr][r] + v;
                    }
        }
    }

    // ---- epilogue ----
    conv_epilogue<MR, NR>(d, b, mt0 + wm * MR, n0 + wn * (32 * NR), acc, lane);
    OU_CSTAMP(5);
    OU_CSTAMP_SAVE;
}

// ---------------------------------------------------------------------------
// Register-streamed variant (tile bit 14; split-f16 / f16, cin a multiple
// of 16, any frame view R whose window fits LDS): for the deep, short levels (256 / 512 channels at 4005 /
// 801 frames), where the chunked kernel above pays one L2 round trip per
// 16-64-channel chunk and, to fill the chip, a K-slice pass plus a second
// launch.  Here a workgroup stages its whole input window -- every input
// channel x (32 NR + KT - 1) frames, PReLU'd and split -- into LDS once, and
// the weights stream straight from L2 into a register ring (each A fragment
// is read by exactly one wave: the packed ou_conv_pack_split order is already
// lane-linear, no LDS copy).  4 waves as WM (32-row m-tiles) x WK (K halves or
// quarters of every tap x 16-channel step), reduced through LDS in a fixed
// order; the epilogue is conv_kernel's.
//   X image: [frame w][h * CE/2 + p] = split(PReLU(x'[2p + h][t0 + w]) 2^-6)
//   over the CE = cin * R frame-view channels, row stride CE + 8 halves (an
//   odd number of 16-B slots), lo plane after; staged from consecutive
//   samples, so the loads are coalesced whatever R is.
template <int P>
__device__ __forceinline__ void split4r(float x0, float x1, float x2, float x3, half4_t& hi, half4_t& lo, float& omax)
{
    hi = half4_t{(_Float16)x0, (_Float16)x1, (_Float16)x2, (_Float16)x3};
    if constexpr (P == 1)
        lo = half4_t{(_Float16)((x0 - (float)hi[0]) * 2048.f), (_Float16)((x1 - (float)hi[1]) * 2048.f),
                     (_Float16)((x2 - (float)hi[2]) * 2048.f), (_Float16)((x3 - (float)hi[3]) * 2048.f)};
    omax = fmaxf(omax, fmaxf(fmaxf(fabsf(x0), fabsf(x1)), fmaxf(fabsf(x2), fabsf(x3))));
}

constexpr int kStageItems = 9;   // conv_rkernel: staging items (8 channels x 1 frame) per thread per round trip

#ifndef OU_RS_RING
#define OU_RS_RING 12
#endif
template <int KT, int WM, int WK, int NR>
struct RCfg {
    static constexpr int BM = 32 * WM, BN = 32 * NR, W = BN + KT - 1;
    static constexpr int RING = OU_RS_RING;   // weight-fragment ring depth (steps): RING - 1 steps of MFMA hide the L2 latency
    static constexpr int DR = KT == 5 ? (RING / 5 > 1 ? RING / 5 : 2) * 5 : (KT == 3 ? RING / 3 * 3 : RING);   // a multiple of KT
    static constexpr int RED = (WK - 1) * WM * NR * 16 * 64;   // floats of the K-split reduction
    static_assert(WM * WK == 4, "4 waves per workgroup");
};

// LDS bytes of the register-streamed kernel for chunks of cec K channels
template <int KT, int WM, int WK, int NR, int P>
int rlds_bytes(int cec)
{
    using R = RCfg<KT, WM, WK, NR>;
    const int x = R::W * (cec + 8) * (P == 1 ? 2 : 1) * 2;
    return std::max(x, R::RED * 4);
}


template <int KT, int WM, int WK, int NR, int P>
__global__ __launch_bounds__(256) void conv_rkernel(ou_conv_desc d, int mtiles, int64_t a_mt_stride, int PC, int CCH,
                                                    int S)
{
    using R = RCfg<KT, WM, WK, NR>;
    constexpr int W = R::W;
    OU_CSTAMP_INIT
    ou_kernarg_prefetch6();
    OU_DYNAMIC_LDS(float4, lds4);
    _Float16* xs = (_Float16*)lds4;
    // K channels: the frame view's cin * R (phase-major: ph * cin + ci), in
    // chunks of PC phases x CCH channels (PC == 1 or CCH == cin, so a chunk is
    // the contiguous K range [p0 cin + c0, + CEC)); one chunk when the whole
    // window fits LDS
    const int cin = d.cin, RF = d.frame, CEC = PC * CCH, SX = CEC + 8, HALF = CEC / 2, plane = W * SX;
    const int nchc = cin / CCH, nchunks = (RF / PC) * nchc;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar step math
    const int wm = wave % WM, wk = wave / WM;
    const int h = lane >> 5, l32 = lane & 31;
    int bx, by, bz;
    if (d.tile & kMajBit) ou_xcd_block_m(bx, by, bz); else ou_xcd_block(bx, by, bz);
    // K slices (S > 1, tile bits 12-13): grid z = batch x S, slice ks walks
    // chunks [ks nchunks / S, (ks + 1) nchunks / S) and stores its partial
    // sums to d.ks_ws; conv_rreduce adds them in slice order (deterministic)
    const int b = bz / S, ks = bz - (bz / S) * S;
    const int n0 = bx * R::BN + d.f0;   // first output frame (global)
    const int mtu = by * WM + wm;       // this wave's m-tile (rows past M: computed, not stored)
    const int mt = min(mtu, mtiles - 1);
    const int diag = (d.tile >> 8) & 3;   // diagnostics (tools/conv_bench.py --rdiag): 1 no input loads, 2 no K loop

    floatx16 acc[1][NR], accx[NR];
#pragma unroll
    for (int nr = 0; nr < NR; ++nr)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[0][nr][r] = 0.f, accx[nr][r] = 0.f;
    // ---- per chunk, steps s = (16-channel group g of the chunk, tap k),
    // s = g * KT + k; wave wk owns steps [s0, s1).  A fragments (hi | lo)
    // stream from the packed global order [m-tile][G][hi | lo][tap][lane][8]
    // (G = the chunk's first 16-group + g) through a D-deep ring whose first
    // D - 1 steps are issued before the chunk's staging, so their L2 latency
    // overlaps it.
    // K steps of a chunk: i = (16-channel group g of the chunk, tap k) with
    // i = (g - g0) KT + k; wave wk owns groups [g0, g1).  A fragments (hi |
    // lo) stream from the packed order [m-tile][G][hi | lo][tap][lane][8]
    // (G = the chunk's first 16-group + g) through a DR-deep register ring
    // (DR a multiple of KT), DR - 1 steps ahead; the ring's first steps are
    // issued before the chunk's staging, so their L2 latency overlaps it.
    // Every step index, offset and bound is wave-uniform (the wave index
    // goes through readfirstlane), so the step loop's address arithmetic runs
    // on the scalar unit: buffer loads with a lane-constant voffset and a
    // scalar soffset, LDS reads at per-(frame tile, tap) row bases advanced
    // once per DR steps, and uniform branches for the ragged last block --
    // the MFMA gaps carry no per-step VALU index math.
    constexpr int DR = R::DR;
    const int G = CEC / 16;
    const int g0 = wk * G / WK, g1 = (wk + 1) * G / WK, n = (g1 - g0) * KT;
    const __amdgpu_buffer_rsrc_t ars = ou_rsrc((const char*)d.w + (int64_t)mt * a_mt_stride * 4, a_mt_stride * 4);
    const unsigned avoff = (unsigned)lane * 16u;
    half8_t ra[DR][2];
    const int64_t xc = d.x_cstride;
    // the batch item's input (cin rows of x_cstride floats)
    const __amdgpu_buffer_rsrc_t xrs = ou_rsrc(d.x + (int64_t)b * d.x_bstride, (int64_t)cin * xc * 4);
    const float scale = d.in_scale ? d.in_scale[b] : 1.f, slope = d.slope;
    const float xsc = ou_exp2i(-d.xs_shift);   // the layer's staging exponent
    const int in_len = d.in_len;
    const int WS = W * PC;                                 // window samples of one chunk, per channel
    const int NI = (CCH / 8) * WS;
    float omax = 0.f;   // max |staged input| (range flag)
    // LDS row bases of this lane's B fragments, per (frame tile, tap), at group g0
    const _Float16* xrow[NR][KT];
#pragma unroll
    for (int nr = 0; nr < NR; ++nr)
#pragma unroll
        for (int k = 0; k < KT; ++k) xrow[nr][k] = xs + (l32 + nr * 32 + k) * SX + h * HALF + 8 * g0;
    const int qa = ks * nchunks / S, qb = (ks + 1) * nchunks / S;
    for (int q = qa; q < qb; ++q) {
        const int p0 = (q / nchc) * PC, c0 = (q - (q / nchc) * nchc) * CCH;
        // byte offset of the chunk's group g0 in the m-tile's panel
        const unsigned abase = (unsigned)(((p0 * cin + c0) / 16 + g0) * 2 * KT) * 1024u;
        auto load_a = [&](int i, half8_t (&dst)[2]) {   // i: uniform step index
            const unsigned so = abase + (unsigned)(2 * (i / KT) * KT + i % KT) * 1024u;
            dst[0] = __builtin_bit_cast(half8_t, __builtin_amdgcn_raw_buffer_load_b128(ars, avoff, so, 0));
            if constexpr (P == 1)
                dst[1] = __builtin_bit_cast(half8_t,
                                            __builtin_amdgcn_raw_buffer_load_b128(ars, avoff, so + KT * 1024u, 0));
        };
        if (n > 0) {   // uniform; clamped (unconditional) loads keep the vmcnt counting exact
#pragma unroll
            for (int j = 0; j < DR - 1; ++j) load_a(min(j, n - 1), ra[j]);
        }
        OU_CSTAMP(0);
        if (q > qa) __syncthreads();   // every wave is done reading the previous chunk
        // ---- stage the chunk: item = (8 channels c0 + 8 g .., sample j of the
        // chunk's window): consecutive lanes load consecutive samples of PC
        // phases (the whole frame when PC = R); sample j is frame j / PC, phase
        // p0 + j % PC, i.e. chunk K channels (j % PC) cin + 8 g .. + 7 of row j / PC.
        // Buffer loads at one per-item voffset (the 8 channels are scalar
        // soffsets i * xc; a sample outside [0, in_len) gets the sentinel
        // voffset and loads 0), items advanced incrementally (no per-item
        // integer division), PC > 1 frames by a float reciprocal (exact for
        // the sample counts a window has), packed f16 conversion.
        const int t0 = (n0 - d.pad) * RF + d.shift + p0;   // first sample of frame 0, phase p0
        constexpr int IPT = kStageItems;
        const int dq = 256 / WS, dr = 256 - dq * WS;          // item += 256: g += dq, sm += dr (carry)
        int g_it = tid / WS, sm_it = tid - g_it * WS;
        const float rpc = 1.f / (float)PC;
        const int xoff0 = c0 * (int)xc * 4;
        for (int base = 0; base < NI; base += IPT * 256) {
            float v[IPT][8];
            int dsto[IPT];
#pragma unroll
            for (int it = 0; it < IPT; ++it) {
                const int item = base + tid + 256 * it;
                const int g = g_it, sm = sm_it;
                sm_it += dr, g_it += dq;
                if (sm_it >= WS) sm_it -= WS, ++g_it;
                const int w = PC == 1 ? sm : (int)(((float)sm + 0.5f) * rpc);
                const int pl = sm - w * PC;
                const int t = t0 + __mul24(w, RF) + pl;
                const bool ok = item < NI && (unsigned)t < (unsigned)in_len && !(diag & 1);
                const int vo = ok ? xoff0 + (__mul24(8 * g, (int)xc) + t) * 4 : kSentinel;   // 24-bit products: full rate
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    v[it][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, vo, i * (int)xc * 4, 0));
                dsto[it] = item < NI ? __mul24(w, SX) + ((__mul24(pl, cin) + 8 * g) >> 1) : -1;
            }
#pragma unroll
            for (int it = 0; it < IPT; ++it) {
                if (dsto[it] < 0) break;   // items run in order: the rest are past NI too
                float x[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float qv = v[it][i] * scale;
                    x[i] = (qv >= 0.f ? qv : qv * slope) * xsc;
                }
                half4_t he, le, ho, lo;
                split4r<P>(x[0], x[2], x[4], x[6], he, le, omax);
                split4r<P>(x[1], x[3], x[5], x[7], ho, lo, omax);
                _Float16* dst = xs + dsto[it];
                *(half4_t*)dst = he;
                *(half4_t*)(dst + HALF) = ho;
                if constexpr (P == 1) {
                    *(half4_t*)(dst + plane) = le;
                    *(half4_t*)(dst + plane + HALF) = lo;
                }
            }
        }
        OU_CSTAMP(1);
        __syncthreads();
        OU_CSTAMP(2);

        // step j of a block: B fragments from LDS, three MFMAs (split-f16)
        auto step = [&](int gj, int j) {
            const int k = j % KT;   // static: blocks start at multiples of KT
            half8_t bq[NR], bl[NR];
#pragma unroll
            for (int nr = 0; nr < NR; ++nr) {
                const _Float16* qq = xrow[nr][k] + 8 * gj;
                bq[nr] = *(const half8_t*)qq;
                if constexpr (P == 1) bl[nr] = *(const half8_t*)(qq + plane);
            }
#pragma unroll
            for (int nr = 0; nr < NR; ++nr) {
                acc[0][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[j][0], bq[nr], acc[0][nr], 0, 0, 0);
                if constexpr (P == 1) {
                    accx[nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[j][0], bl[nr], accx[nr], 0, 0, 0);
                    accx[nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[j][1], bq[nr], accx[nr], 0, 0, 0);
                }
            }
        };
        const int nn = (diag & 2) ? 0 : n;
        // whole blocks: branch-free, every load unconditional (step index
        // clamped to the last one: a few redundant loads at the end), so the
        // compiler counts vmcnt exactly and waits only for the slot in use
        int ib = 0;
        for (; ib + DR <= nn; ib += DR) {
            const int gb = ib / KT;
#pragma unroll
            for (int j = 0; j < DR; ++j) {
                load_a(min(ib + j + DR - 1, nn - 1), ra[(j + DR - 1) % DR]);
                step(gb + j / KT, j);
            }
        }
        // ragged last block (n % DR steps; none when DR divides n): its
        // fragments are already in the ring
        if (ib < nn) {
            const int gb = ib / KT;
#pragma unroll
            for (int j = 0; j < DR - 1; ++j)
                if (ib + j < nn) step(gb + j / KT, j);
        }
        OU_CSTAMP(3);
    }
    ou_range_flag(d.status, omax, 1, lane);
    const float su = d.w_unscale * ou_exp2i(d.xs_shift - kSplitShift), sx = su * (1.f / 2048.f);
#pragma unroll
    for (int nr = 0; nr < NR; ++nr)
#pragma unroll
        for (int r = 0; r < 16; ++r)
            acc[0][nr][r] = P == 1 ? fmaf(accx[nr][r], sx, acc[0][nr][r] * su) : acc[0][nr][r] * su;

    // the epilogue's loads (bias, FiLM, residuals) go out before the K-split
    // reduction, so their latency overlaps it (wave wk = 0 finishes the tile)
    const EpiCtx ec = epi_ctx(d, b);
    EpiPre<1, NR> ep;
    if (S == 1 && wk == 0) conv_epi_load<1, NR>(d, ec, mtu, n0, lane, ep);
    // ---- K-split reduction in wave order (deterministic)
    if constexpr (WK > 1) {
        float* red = (float*)lds4;
        __syncthreads();   // every wave is done reading the X image
        if (wk > 0) {
#pragma unroll
            for (int nr = 0; nr < NR; ++nr)
#pragma unroll
                for (int r = 0; r < 16; ++r) red[((((wk - 1) * WM + wm) * NR + nr) * 16 + r) * 64 + lane] = acc[0][nr][r];
        }
        __syncthreads();
        OU_CSTAMP(4);
        if (wk > 0) return;
        for (int j = 1; j < WK; ++j)
#pragma unroll
            for (int nr = 0; nr < NR; ++nr)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[0][nr][r] += red[((((j - 1) * WM + wm) * NR + nr) * 16 + r) * 64 + lane];
    }
    if (S > 1) {   // this slice's sums -> d.ks_ws [tile][slice][wm][nr][16][lane]
        const int64_t tl = ((int64_t)b * gridDim.y + by) * gridDim.x + bx;
        float* pw = d.ks_ws + (((tl * S + ks) * WM + wm) * NR) * 16 * 64 + lane;
#pragma unroll
        for (int nr = 0; nr < NR; ++nr)
#pragma unroll
            for (int r = 0; r < 16; ++r) pw[(nr * 16 + r) * 64] = acc[0][nr][r];
        return;
    }
    OU_CSTAMP(4);
    conv_epi_store<1, NR>(d, ec, mtu, n0, acc, ep, lane);
    OU_CSTAMP(5);
    OU_CSTAMP_SAVE;
}

// Second launch of a K-sliced register-streamed conv: one wave per m-tile of
// a (frame tile, m-group) adds the S partial sums in slice order and runs the
// epilogue.  grid (frame tiles, m-groups, batch) as conv_rkernel's without
// the slices; 64 WM threads.
template <int NR>
__global__ __launch_bounds__(256) void conv_rreduce(ou_conv_desc d, int S, int WM)
{
    int bx, by, bz;
    ou_xcd_block(bx, by, bz);
    const int lane = threadIdx.x & 63, wm = threadIdx.x >> 6;
    const int b = bz, n0 = bx * 32 * NR + d.f0, mtu = by * WM + wm;
    const int64_t tl = ((int64_t)b * gridDim.y + by) * gridDim.x + bx;
    floatx16 acc[1][NR];
#pragma unroll
    for (int nr = 0; nr < NR; ++nr)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[0][nr][r] = 0.f;
    for (int k = 0; k < S; ++k) {
        const float* pr = d.ks_ws + (((tl * S + k) * WM + wm) * NR) * 16 * 64 + lane;
#pragma unroll
        for (int nr = 0; nr < NR; ++nr)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float v = pr[(nr * 16 + r) * 64];
                acc[0][nr][r] = k == 0 ? v : acc[0][nr][r] + v;
            }
    }
    conv_epilogue<1, NR>(d, b, mtu, n0, acc, lane);
}

// ---------------------------------------------------------------------------
// Split-image kernel (tile bit 15; split-f16, cin a multiple of 32).  The
// input is not the f32 signal but its split image (ou_conv_desc.xs): the
// producing conv's epilogue has already applied this conv's PReLU and staging
// exponent and split the result into f16 hi / lo halves, in the blocked
// layout [c / 32][t][hi | lo][c % 32] (one 128-B row per 32-channel block and
// sample).  Staging is a copy -- 16-B loads of whole rows, 16-B LDS stores,
// no conversion VALU -- so it can run beside the MFMAs:
//   * K is walked in chunks of one (phase, 32-channel block) x every tap;
//     chunk c belongs to wave c % 4, which stages and consumes it through
//     its own two LDS slots (no workgroup barrier before the final
//     reduction);
//   * the next chunk's loads are issued before the current chunk's MFMAs
//     and stored to the other slot halfway through them;
//   * the weights stream from L2 into a DR-deep register ring across chunk
//     boundaries (lane-linear ou_conv_pack_split_nat order: lane l holds row
//     l & 31, channels 16 G + 8 (l >> 5) + j, so the matching B fragment is
//     8 consecutive channels of one LDS row: one ds_read_b128 per plane);
//   * the four waves' partial sums are added through LDS in wave order
//     (deterministic), each wave finishing a quarter of the rows, so the
//     epilogue is spread over the whole workgroup.
// One workgroup = one 32-row m-tile x 32 NR frames.  Waves whose chunk
// count falls short of the unrolled body run zero chunks (their B rows read
// 0, their A steps are clamped to real ones: +0 exactly).
#ifndef OU_SK_BPREF   // B fragments read one step ahead of their MFMAs
#define OU_SK_BPREF 1
#endif
#ifndef OU_SK_EPIPRE  // the epilogue's loads issued before the cross-wave reduction
#define OU_SK_EPIPRE 1
#endif
// Diagnostic build (-DOU_SK_STAMPS, tools/conv_bench.py --sstamps): lane 0 of
// every wave of the first 1024 workgroups sums s_memtime deltas per phase
// (prologue, main loop, reduction, epilogue; 6/7 realtime) into d.ks_ws as
// uint64 [workgroup][wave][8] -- the split-image kernel takes no K slices.
#ifdef OU_SK_STAMPS
#define OU_SSTAMP_INIT uint64_t sst_[8] = {}; uint64_t stp_ = __builtin_amdgcn_s_memtime(); \
    sst_[6] = __builtin_amdgcn_s_memrealtime();
#define OU_SSTAMP(i) do { const uint64_t n_ = __builtin_amdgcn_s_memtime(); sst_[i] += n_ - stp_; stp_ = n_; } while (0)
#define OU_SSTAMP_SAVE                                                                          \
    do {                                                                                        \
        sst_[7] = __builtin_amdgcn_s_memrealtime();                                             \
        const int wg_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);         \
        if (lane == 0 && d.ks_ws && wg_ < 1024)                                                 \
            for (int i_ = 0; i_ < 8; ++i_) ((uint64_t*)d.ks_ws)[(wg_ * 4 + wave) * 8 + i_] = sst_[i_]; \
    } while (0)
#else
#define OU_SSTAMP_INIT
#define OU_SSTAMP(i) do { } while (0)
#define OU_SSTAMP_SAVE do { } while (0)
#endif

template <int KT, int NR, int DEEP = 0>
struct SCfg {
    static constexpr int W = 32 * NR + KT - 1;      // window frames (LDS rows) of a chunk
    static constexpr int NL = (W * 8 + 63) / 64;   // 16-B loads per lane per chunk (8 lanes per row)
    static constexpr int RS = 144;                 // LDS row stride: 128 B + 16 (9 slots: odd, conflict-free)
    static constexpr int SLOT = W * RS;
    static constexpr int STEPS = 2 * KT;           // K steps per chunk: 2 groups of 16 channels x taps
    static constexpr int U = KT == 1 ? 4 : 2;      // chunks per unrolled body
    // register sets for rows in flight: 1 = the next chunk's rows loaded at a
    // chunk's start and stored halfway through it; DEEP: U sets, loaded
    // SETS - 0.5 chunks ahead (more VGPRs: at 64-frame tiles two waves per
    // SIMD no longer fit, slower on the 4005-frame levels, faster at 801)
    static constexpr int SETS = DEEP ? U : 1;
    static constexpr int DR = KT == 5 ? 10 : U * STEPS;   // weight ring depth (divides U * STEPS)
    static constexpr int RED = 4 * NR * 16 * 64 * 4;       // the reduction image (bytes)
    static constexpr int LDS = 8 * SLOT > RED ? 8 * SLOT : RED;
    static_assert((U * STEPS) % DR == 0, "ring depth must divide the unrolled body");
    static_assert(U % SETS == 0, "register sets must divide the unrolled body");
};

// The split-image kernel's epilogue: wave q finishes rows 8 q + 4 h .. + 3
// (accumulator registers 4 q .. 4 q + 3) of its m-tile.  Two phases: every
// load (bias, FiLM, residuals) is issued before the cross-wave reduction,
// which then hides their latency.
template <int NR>
struct EpiQ {
    int m0, co[4], ph[4], off[NR][4];
    float bias[4], fa[4], fb[4], v1[NR][4], v2[NR][4];
};

template <int NR>
__device__ __forceinline__ void conv_epi_q_load(const ou_conv_desc& d, const EpiCtx& c, int mt, int ub, int q, int lane,
                                                EpiQ<NR>& e)
{
    const int h = lane >> 5, l32 = lane & 31;
    const int M = c.M, rout = c.rout, cout = c.cout, ylen = c.ylen;
    e.m0 = mt * 32 + 8 * q + 4 * h;
#pragma unroll
    for (int j = 0; j < 4; ++j) ou_row_map(min(e.m0 + j, M - 1), d.rout, cout, e.co[j], e.ph[j]);
    if (d.bias) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            e.bias[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(c.bs, e.co[j] * 4, 0, 0));
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) e.bias[j] = 0.f;
    }
    if (c.has_fm) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            e.fa[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(c.fs, e.co[j] * 4, 0, 0));
            e.fb[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(c.fs, (cout + e.co[j]) * 4, 0, 0));
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) e.fa[j] = 0.f, e.fb[j] = 0.f;
    }
#pragma unroll
    for (int nr = 0; nr < NR; ++nr) {
        const int u = ub + nr * 32 + l32;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = u * rout + e.ph[j];
            e.off[nr][j] = (e.m0 + j < M && u < d.f0 + d.n_frames && t < ylen) ? t : -1;
            e.v1[nr][j] = e.v2[nr][j] = 0.f;
        }
        if (c.has_r1) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                e.v1[nr][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                    c.r1s, e.off[nr][j] >= 0 ? (e.co[j] * (int)d.r1_cstride + e.off[nr][j]) * 4 : kSentinel, 0, 0));
        }
        if (c.has_r2) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                e.v2[nr][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                    c.r2s, e.off[nr][j] >= 0 ? (e.co[j] * (int)d.r2_cstride + e.off[nr][j]) * 4 : kSentinel, 0, 0));
        }
    }
}

template <int NR>
__device__ __forceinline__ void conv_epi_q_store(const ou_conv_desc& d, const EpiCtx& c, int ub, const EpiQ<NR>& e,
                                                 const float (&v)[NR][4], int lane, float& somax)
{
    const int l32 = lane & 31;
#pragma unroll
    for (int nr = 0; nr < NR; ++nr) {
        float sv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float x = v[nr][j] + e.bias[j];
            if (e.off[nr][j] >= d.valid_len) x = 0.f;
            x = (x + e.v1[nr][j]) * c.s1e;
            x = (e.fa[j] + c.fadd) * x + e.fb[j];
            x = (x + e.v2[nr][j]) * c.s2e;
            sv[j] = x;
            __builtin_amdgcn_raw_buffer_store_b32(
                __float_as_uint(x), c.ys, e.off[nr][j] >= 0 ? (e.co[j] * (int)d.y_cstride + e.off[nr][j]) * 4 : kSentinel,
                0, 0);
        }
        if (c.has_sy) {   // rout 1 (host-checked): rows are channels m0 .. m0 + 3, sample u
            const int u = ub + nr * 32 + l32;
            split_store4(c.so, e.m0, u, e.off[nr][0] >= 0, sv[0], sv[1], sv[2], sv[3], somax);
        }
    }
}

template <int KT, int NR, int DEEP>
__global__ __launch_bounds__(256) void conv_skernel(ou_conv_desc d, int mtiles, int64_t a_mt_stride)
{
    using S = SCfg<KT, NR, DEEP>;
    ou_kernarg_prefetch8();
    OU_DYNAMIC_LDS(float4, lds4);
    char* lds = (char*)lds4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar chunk / step math
    const int h = lane >> 5, l32 = lane & 31;
    int bx, by, bz;
    if (d.tile & kMajBit) ou_xcd_block_m(bx, by, bz); else ou_xcd_block(bx, by, bz);
    const int b = bz;
    const int n0 = bx * 32 * NR + d.f0;   // first output frame (global)
    const int mt = min(by, mtiles - 1);
    const int cin = d.cin, RF = d.frame;
    const int ncb = cin / 32, nch = ncb * RF;   // chunks c = ph * ncb + cb (phase-major K)
    // every wave walks the same number of chunks (a multiple of U): chunk
    // c = wave + 4 j, zero chunks past nch
    const int njb = (nch + 4 * S::U - 1) / (4 * S::U);   // unrolled bodies
    const int nj = njb * S::U;
    const int n = nj * S::STEPS;                         // K steps of this wave

    // ---- weights: step i = (chunk j, group gg, tap k) -> 16-channel group
    // G = 2 c + gg of the phase-major K; byte offset in the m-tile's panel
    const __amdgpu_buffer_rsrc_t ars = ou_rsrc((const char*)d.w + (int64_t)mt * a_mt_stride * 4, a_mt_stride * 4);
    const unsigned avoff = (unsigned)lane * 16u;
    half8_t ra[S::DR][2];
    auto load_a = [&](int i, half8_t (&dst)[2]) {   // i uniform
        i = min(i, n - 1);
        const int j = i / S::STEPS, s = i - (i / S::STEPS) * S::STEPS;
        const int c = min(wave + 4 * j, nch - 1);   // zero chunks: any real step (times B = 0)
        const int gg = s / KT, k = s - (s / KT) * KT;
        const unsigned so = (unsigned)(((2 * c + gg) * 2 * KT + k) * 1024);
        dst[0] = __builtin_bit_cast(half8_t, __builtin_amdgcn_raw_buffer_load_b128(ars, avoff, so, 0));
        dst[1] = __builtin_bit_cast(half8_t, __builtin_amdgcn_raw_buffer_load_b128(ars, avoff, so + KT * 1024u, 0));
    };

    // ---- input rows: load l of a lane covers item 64 l + lane = (window
    // row w = item / 8, 16-B piece ls = item % 8) -- 8 lanes per 128-B row
    const __amdgpu_buffer_rsrc_t xrs =
        ou_rsrc((const char*)d.xs + (int64_t)b * d.xs_bstride, (int64_t)ncb * d.xs_rows * 128);
    const int t0 = (n0 - d.pad) * RF + d.shift;   // sample of window row 0 at phase 0
    const int in_len = d.in_len;
    char* myslots = lds + wave * 2 * S::SLOT;
    const int wr0 = lane >> 3, ls = lane & 7;
    ou_u32x4 xr[S::SETS][S::NL];   // a chunk's rows are loaded SETS - 0.5 chunks before they are stored
    auto stage_load = [&](int j, int set) {   // j uniform (j >= nj or a zero chunk: every load reads 0)
        const int c = wave + 4 * j;
        const bool real = c < nch;
        const int ph = real ? c / ncb : 0, cb = real ? c - (c / ncb) * ncb : 0;
        const unsigned so = (unsigned)(cb * d.xs_rows) * 128u;
#pragma unroll
        for (int l = 0; l < S::NL; ++l) {
            const int w = 8 * l + wr0;
            const int t = t0 + w * RF + ph;
            const bool ok = real && w < S::W && (unsigned)t < (unsigned)in_len;
            xr[set][l] = __builtin_amdgcn_raw_buffer_load_b128(xrs, ok ? t * 128 + ls * 16 : kSentinel, so, 0);
        }
    };
    auto stage_store = [&](int slot, int set) {   // slot, set static
        char* base = myslots + slot * S::SLOT + wr0 * S::RS + ls * 16;
#pragma unroll
        for (int l = 0; l < S::NL; ++l)
            if (8 * (S::NL - 1) + 7 < S::W || l < S::NL - 1 || 8 * l + wr0 < S::W)
                *(ou_u32x4*)(base + l * 8 * S::RS) = xr[set][l];
        OU_WAVE_SYNC();
    };

    floatx16 acc[NR], accx[NR];
#pragma unroll
    for (int nr = 0; nr < NR; ++nr)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[nr][r] = 0.f, accx[nr][r] = 0.f;

    // B fragments of (slot, group gg, tap k): LDS row nr * 32 + l32 + k,
    // 16-B piece 2 gg + h (hi) and + 4 (lo)
    const char* bbase = myslots + l32 * S::RS + h * 16;
    half8_t bq[2][NR], bl[2][NR];   // B fragments, double-buffered by step parity
    auto read_b = [&](int slot, int gg, int k, half8_t (&q)[NR], half8_t (&l)[NR]) {
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
            const char* p = bbase + slot * S::SLOT + (nr * 32 + k) * S::RS + gg * 32;
            q[nr] = *(const half8_t*)p;
            l[nr] = *(const half8_t*)(p + 64);
        }
    };
    auto mfmas = [&](const half8_t (&a)[2], const half8_t (&q)[NR], const half8_t (&l)[NR]) {
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
            acc[nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], q[nr], acc[nr], 0, 0, 0);
            accx[nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], l[nr], accx[nr], 0, 0, 0);
            accx[nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], q[nr], accx[nr], 0, 0, 0);
        }
    };

    // Schedule of chunk j (LDS slot j & 1):
    //   SETS == 1: chunk j + 1's rows are loaded at chunk j's start and stored
    //     to slot (j + 1) & 1 halfway through it;
    //   SETS > 1: at chunk j's half, chunk j + SETS's rows are loaded into set
    //     j % SETS (whose rows, chunk j's, are in LDS already), and at step
    //     STEPS - 2 set (j + 1) % SETS is stored to slot (j + 1) & 1, one step
    //     before chunk j + 1 reads it.
    //   Slot (j + 1) & 1's last reader, chunk j - 1, is done by then.  With
    //   OU_SK_BPREF the B fragments of step s + 1 are read before step s's
    //   MFMAs (the next chunk's first ones from the other slot).
    OU_SSTAMP_INIT
    stage_load(0, 0);   // the first rows first: chunk 0 waits for them, not for the ring
#pragma unroll
    for (int i = 0; i < S::DR - 1; ++i) load_a(i, ra[i]);
    stage_store(0, 0);
#pragma unroll
    for (int q = 1; q < S::SETS; ++q) stage_load(q, q);
    if (OU_SK_BPREF) read_b(0, 0, 0, bq[0], bl[0]);
    OU_SSTAMP(0);
    for (int jb = 0; jb < njb; ++jb) {
#pragma unroll
        for (int u = 0; u < S::U; ++u) {
            const int j = jb * S::U + u;
            if (S::SETS == 1) stage_load(j + 1, 0);
#pragma unroll
            for (int s = 0; s < S::STEPS; ++s) {
                const int ib = (u * S::STEPS + s) % S::DR;   // ring slot of step j * STEPS + s (static)
                const int par = (u * S::STEPS + s) & 1;      // B buffer of this step
                if (S::SETS > 1 && s == S::STEPS / 2) stage_load(j + S::SETS, u % S::SETS);
                load_a(j * S::STEPS + s + S::DR - 1, ra[(ib + S::DR - 1) % S::DR]);
                if (OU_SK_BPREF) {
                    // the next step's fragments (the next chunk's first: the other slot)
                    if (s + 1 < S::STEPS) read_b(u & 1, (s + 1) / KT, (s + 1) % KT, bq[par ^ 1], bl[par ^ 1]);
                    else read_b((u + 1) & 1, 0, 0, bq[par ^ 1], bl[par ^ 1]);
                } else {
                    read_b(u & 1, s / KT, s % KT, bq[par], bl[par]);
                }
                mfmas(ra[ib], bq[par], bl[par]);
                if (S::SETS == 1 ? s == S::STEPS / 2 - 1 : (s == S::STEPS - 2 || (S::STEPS < 2 && s == 0)))
                    stage_store((u + 1) & 1, S::SETS == 1 ? 0 : (u + 1) % S::SETS);
            }
        }
    }
    OU_SSTAMP(1);

    // ---- combine the split-f16 terms, then the four waves' partial sums
    const float su = d.w_unscale * ou_exp2i(d.xs_shift - kSplitShift), sx = su * (1.f / 2048.f);
#pragma unroll
    for (int nr = 0; nr < NR; ++nr)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[nr][r] = fmaf(accx[nr][r], sx, acc[nr][r] * su);
    const EpiCtx ec = epi_ctx(d, b);
    EpiQ<NR> eq;
    if (OU_SK_EPIPRE) conv_epi_q_load<NR>(d, ec, by, n0, wave, lane, eq);   // latency hidden by the reduction
    __syncthreads();   // every wave is done with its slots
    ou_u32x4* red = (ou_u32x4*)lds;   // [wave][nr][register quad][lane]
#pragma unroll
    for (int nr = 0; nr < NR; ++nr)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
            red[((wave * NR + nr) * 4 + qq) * 64 + lane] =
                ou_u32x4{__float_as_uint(acc[nr][4 * qq]), __float_as_uint(acc[nr][4 * qq + 1]),
                         __float_as_uint(acc[nr][4 * qq + 2]), __float_as_uint(acc[nr][4 * qq + 3])};
    __syncthreads();
    float v[NR][4];
#pragma unroll
    for (int nr = 0; nr < NR; ++nr) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[nr][j] = 0.f;
#pragma unroll
        for (int p = 0; p < 4; ++p) {   // wave order: deterministic
            const ou_u32x4 x = red[((p * NR + nr) * 4 + wave) * 64 + lane];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[nr][j] = p == 0 ? __uint_as_float(x[j]) : v[nr][j] + __uint_as_float(x[j]);
        }
    }
    if (!OU_SK_EPIPRE) conv_epi_q_load<NR>(d, ec, by, n0, wave, lane, eq);
    OU_SSTAMP(2);
    float somax = 0.f;
    conv_epi_q_store<NR>(d, ec, n0, eq, v, lane, somax);
    if (ec.has_sy) ou_range_flag(d.status, somax, 2, lane);
    OU_SSTAMP(3);
    OU_SSTAMP_SAVE;
}

// ---------------------------------------------------------------------------
// Persistent variant (tiles-per-workgroup >= 2, shapes without split-K).
//
// All workgroups of the one-tile kernel above run in lockstep, so the whole
// grid loads X, then computes, then writes its outputs at the same moment:
// the HBM bursts and the MFMA phases add up.  Here a workgroup walks output
// tiles blockIdx.x, +gridDim.x, ...; its (tile, chunk) work items form one
// stream whose next item -- the next tile's first chunk included -- is loaded
// while the current item's MFMAs run, and the residual + bias of a tile's
// epilogue are loaded at the start of its last chunk.  The epilogue's stores
// then drain while the next tile computes.
// ---------------------------------------------------------------------------
template <int KT, int CC, int WM, int WN, int MR, int NR>
__global__ __launch_bounds__(256) void conv_pkernel(ou_conv_desc d, int nchunks, int mtiles,
                                                    int64_t a_mt_stride, int ntn, int mgroups, int ntiles)
{
    constexpr int WK = 1;
    using C = Cfg<KT, CC, WM, WN, WK, MR, NR>;
    static_assert(CC % 8 == 0 && WM * WN == 4, "4 waves, no split-K");
    static_assert((C::SX / 4) % 2 == 1, "X row stride must be an odd number of 16-B slots");
    OU_DYNAMIC_LDS(float4, lds4);
    float* lds = (float*)lds4;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wn = wave % WN;
    const int wm = wave / WN;
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int R = d.frame;
    const int cin = d.cin;
    const int in_len = d.in_len;
    const int xc = (int)d.x_cstride;
    const float slope = d.slope;

    // staging geometry independent of the tile
    int xdst[C::XE], xw[C::XE], xcl[C::XE];
#pragma unroll
    for (int e = 0; e < C::XE; ++e) {
        const int g = tid + e * 256;
        const int w = g % C::W;
        const int r = g / C::W;
        xdst[e] = g < C::XG ? w * C::SX + (r & 1) * C::HALF + 4 * (r >> 1) : -1;
        xw[e] = w;
        xcl[e] = 8 * (r >> 1) + (r & 1);
    }
    const __amdgpu_buffer_rsrc_t wrs = ou_rsrc(d.w, (int64_t)mtiles * a_mt_stride * 4);
    int aoff[C::AE], aml[C::AE];
#pragma unroll
    for (int e = 0; e < C::AE; ++e) {
        const int f = min(tid + e * 256, C::AG - 1);
        const int ml = f / (C::HQ * KT * 64);
        aml[e] = ml;
        aoff[e] = (int)((ml * a_mt_stride + (f - ml * (C::HQ * KT * 64)) * 4) * 4);
    }

    float xr[4 * C::XE];
    float ar[4 * C::AE];
    float xscale = 1.f;   // in_scale of the item held in xr

#define OU_DECODE(tile_, b_, n0_, mt0_)                                                        \
    const int b_ = (tile_) / ntn / mgroups;                                                    \
    const int n0_ = ((tile_) % ntn) * C::BN;                                                   \
    const int mt0_ = (((tile_) / ntn) % mgroups) * (WM * MR);

    auto load_item = [&](int tile, int q) {
        OU_DECODE(tile, b, n0, mt0)
        const int t0 = n0 - d.pad;
        const float* xb = d.x + (int64_t)b * d.x_bstride;
        xscale = d.in_scale ? d.in_scale[b] : 1.0f;
        if (R == 1) {
            const int nch = cin - q * CC;
            const __amdgpu_buffer_rsrc_t rs = ou_rsrc(xb + (int64_t)q * CC * xc, nch > 0 ? (int64_t)nch * xc * 4 : 0);
#pragma unroll
            for (int e = 0; e < C::XE; ++e) {
                const int pos = t0 + xw[e] + d.shift;
                const bool ok = xdst[e] >= 0 && pos >= 0 && pos < in_len;
                const unsigned o = ok ? (unsigned)((xcl[e] * xc + pos) * 4) : (unsigned)kSentinel;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    xr[4 * e + j] = __uint_as_float(
                        __builtin_amdgcn_raw_buffer_load_b32(rs, o + j * 8u * (unsigned)xc, 0, 0));
            }
        } else if (cin % CC == 0) {
            const int ph = (q * CC) / cin;
            const int ci0 = q * CC - ph * cin;
            const __amdgpu_buffer_rsrc_t rs = ou_rsrc(xb + (int64_t)ci0 * xc, (int64_t)(cin - ci0) * xc * 4);
#pragma unroll
            for (int e = 0; e < C::XE; ++e) {
                const int pos = (t0 + xw[e]) * R + d.shift + ph;
                const bool ok = xdst[e] >= 0 && pos >= 0 && pos < in_len;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    xr[4 * e + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                        rs, ok ? ((xcl[e] + 2 * j) * xc + pos) * 4 : kSentinel, 0, 0));
            }
        } else {
            const __amdgpu_buffer_rsrc_t rs = ou_rsrc(xb, (int64_t)cin * xc * 4);
#pragma unroll
            for (int e = 0; e < C::XE; ++e) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int cq = q * CC + xcl[e] + 2 * j;
                    const int ph = cq / cin;
                    const int ci = cq - ph * cin;
                    const int pos = (t0 + xw[e]) * R + d.shift + ph;
                    const int off = (xdst[e] >= 0 && ph < R && pos >= 0 && pos < in_len) ? (ci * xc + pos) * 4
                                                                                         : kSentinel;
                    xr[4 * e + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
                }
            }
        }
        // the range check covers the voffset only: m-tiles past the weights
        // get the sentinel voffset (the tile offset travels in soffset)
        const int soff = (int)((mt0 * a_mt_stride + (int64_t)q * (C::HQ * KT * 256)) * 4);
#pragma unroll
        for (int e = 0; e < C::AE; ++e) {
            const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(wrs, mt0 + aml[e] < mtiles ? aoff[e] : kSentinel,
                                                                   soff, 0);
            ar[4 * e] = __uint_as_float(v4[0]);
            ar[4 * e + 1] = __uint_as_float(v4[1]);
            ar[4 * e + 2] = __uint_as_float(v4[2]);
            ar[4 * e + 3] = __uint_as_float(v4[3]);
        }
    };

    auto store_item = [&](int buf) {
        float* xs = lds + buf * C::STAGE;
        const float sc = xscale;
#define OU_PRELU(v) ((v) * sc >= 0.f ? (v) * sc : (v) * sc * slope)
#pragma unroll
        for (int e = 0; e < C::XE; ++e)
            if (xdst[e] >= 0)
                *(float4*)(xs + xdst[e]) = make_float4(OU_PRELU(xr[4 * e]), OU_PRELU(xr[4 * e + 1]),
                                                       OU_PRELU(xr[4 * e + 2]), OU_PRELU(xr[4 * e + 3]));
#undef OU_PRELU
        float4* as = (float4*)(xs + C::XBUF);
#pragma unroll
        for (int e = 0; e < C::AE; ++e)
            if (C::AG % 256 == 0 || tid + e * 256 < C::AG)
                as[tid + e * 256] = make_float4(ar[4 * e], ar[4 * e + 1], ar[4 * e + 2], ar[4 * e + 3]);
    };

    const int M = d.m;
    const int rout = d.rout < 0 ? -d.rout : d.rout;
    const int cout = M / rout;
    const bool has_r1 = d.res1 != nullptr, has_r2 = d.res2 != nullptr;
    float ev1[MR][NR][16];
    float ebias[MR][16];
    auto row_of = [&](int mt, int r, int& co, int& ph) {
        const int m = min(mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, M - 1);
        ou_row_map(m, d.rout, cout, co, ph);
    };
    // residual 1 and bias of a tile's epilogue, issued one chunk ahead
    const __amdgpu_buffer_rsrc_t bs = ou_rsrc(d.bias, d.bias ? (int64_t)cout * 4 : 0);
    auto load_epilogue = [&](int tile) {
        OU_DECODE(tile, b, n0, mt0)
        const __amdgpu_buffer_rsrc_t r1s = ou_rsrc(has_r1 ? d.res1 + (int64_t)b * d.r1_bstride : d.y,
                                                   has_r1 ? (int64_t)cout * d.r1_cstride * 4 : 0);
#pragma unroll
        for (int mr = 0; mr < MR; ++mr) {
            const int mt = mt0 + wm * MR + mr;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                int co, ph;
                row_of(mt, r, co, ph);
                ebias[mr][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bs, co * 4, 0, 0));
                const int m = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
                for (int nr = 0; nr < NR; ++nr) {
                    const int u = n0 + wn * (32 * NR) + nr * 32 + l32;
                    const int t = u * rout + ph;
                    const bool ok = has_r1 && m < M && u < d.n_frames && t < d.out_len;
                    ev1[mr][nr][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                        r1s, ok ? (co * (int)d.r1_cstride + t) * 4 : kSentinel, 0, 0));
                }
            }
        }
    };

    floatx16 acc[MR][NR];
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    int tile = blockIdx.x;
    if (tile >= ntiles) return;
    load_item(tile, 0);
    store_item(0);
    __syncthreads();
    int buf = 0;
    while (true) {
        for (int q = 0; q < nchunks; ++q) {
            const int ntile = q + 1 < nchunks ? tile : tile + (int)gridDim.x;
            const int nq = q + 1 < nchunks ? q + 1 : 0;
            const bool has_next = ntile < ntiles;
            if (q + 1 == nchunks) load_epilogue(tile);
            if (has_next) load_item(ntile, nq);
            {
                const float* xs = lds + buf * C::STAGE;
                const float4* ap = (const float4*)(xs + C::XBUF) + (wm * MR) * C::HQ * KT * 64 + lane;
                const float* xp = xs + (wn * 32 * NR + l32) * C::SX + h * C::HALF;
                constexpr int NS = C::CPW * KT;
                float4 fa[2][MR], fb[2][NR];
                auto frag = [&](int st, float4* a, float4* bq) {
                    const int cpq = st / KT, k = st - (st / KT) * KT;
#pragma unroll
                    for (int mr = 0; mr < MR; ++mr) a[mr] = ap[((mr * C::HQ + cpq) * KT + k) * 64];
#pragma unroll
                    for (int nr = 0; nr < NR; ++nr)
                        bq[nr] = *(const float4*)(xp + (nr * 32 + k) * C::SX + 4 * cpq);
                };
                frag(0, fa[0], fb[0]);
#pragma unroll
                for (int st = 0; st < NS; ++st) {
                    if (st + 1 < NS) frag(st + 1, fa[(st + 1) & 1], fb[(st + 1) & 1]);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                            for (int nr = 0; nr < NR; ++nr)
                                acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                                    fa[st & 1][mr][j], fb[st & 1][nr][j], acc[mr][nr], 0, 0, 0);
                }
            }
            if (has_next) store_item(buf ^ 1);
            __syncthreads();
            buf ^= 1;
        }

        // epilogue of `tile`: branch-free, out-of-range elements dropped
        {
            OU_DECODE(tile, b, n0, mt0)
            const __amdgpu_buffer_rsrc_t ys = ou_rsrc(d.y + (int64_t)b * d.y_bstride, (int64_t)cout * d.y_cstride * 4);
            const __amdgpu_buffer_rsrc_t r2s = ou_rsrc(has_r2 ? d.res2 + (int64_t)b * d.r2_bstride : d.y,
                                                       has_r2 ? (int64_t)cout * d.r2_cstride * 4 : 0);
            const bool has_fm = d.film != nullptr;
            const float s1e = has_r1 ? d.s1 : 1.f, s2e = has_r2 ? d.s2 : 1.f, fadd = has_fm ? 0.f : 1.f;
            const __amdgpu_buffer_rsrc_t fs = ou_rsrc(has_fm ? d.film + (int64_t)b * d.film_bstride : d.y,
                                                      has_fm ? (int64_t)cout * 8 : 0);
#pragma unroll
            for (int mr = 0; mr < MR; ++mr) {
                const int mt = mt0 + wm * MR + mr;
#pragma unroll
                for (int nr = 0; nr < NR; ++nr) {
                    const int u = n0 + wn * (32 * NR) + nr * 32 + l32;
                    int off[16];
                    float v2[16];
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        int co, ph;
                        row_of(mt, r, co, ph);
                        const int m = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        const int t = u * rout + ph;
                        const bool ok = m < M && u < d.n_frames && t < d.out_len;
                        off[r] = ok ? t : -1;
                        v2[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                            r2s, (has_r2 && ok) ? (co * (int)d.r2_cstride + t) * 4 : kSentinel, 0, 0));
                    }
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        int co, ph;
                        row_of(mt, r, co, ph);
                        float v = acc[mr][nr][r] + ebias[mr][r];
                        if (off[r] >= d.valid_len) v = 0.f;
                        v = (v + ev1[mr][nr][r]) * s1e;
                        v = (__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(fs, co * 4, 0, 0)) + fadd) * v +
                            __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(fs, (cout + co) * 4, 0, 0));
                        v = (v + v2[r]) * s2e;
                        __builtin_amdgcn_raw_buffer_store_b32(
                            __float_as_uint(v), ys, off[r] >= 0 ? (co * (int)d.y_cstride + off[r]) * 4 : kSentinel,
                            0, 0);
                        acc[mr][nr][r] = 0.f;
                    }
                }
            }
        }
        tile += gridDim.x;
        if (tile >= ntiles) break;
    }
#undef OU_DECODE
}

// ---------------------------------------------------------------------------
// Warp-specialised persistent variant (tile bit 10): 512 threads = 4 MFMA
// waves (WM x WN x WK) + 4 staging waves, one of each per SIMD.  The MFMA
// waves only read LDS, issue MFMAs and write their accumulators back to LDS;
// every global memory access belongs to the staging waves.
//
// Staging waves, per K chunk t ("tick", one workgroup barrier each):
//   1. LDS-DMA (buffer_load ... lds) of chunk t + 2 into a 3-stage ring: the X
//      window as [channel][frame] rows (64-frame dword pieces, coalesced) and
//      the chunk's packed weights (16-B pieces, lane-linear);
//   2. when chunk t is a tile's last: LDS-DMA of that tile's residual in
//      row-major 16-B groups, each lane the groups it will itself finish;
//   3. vmcnt: chunk t + 1 and the residual have landed (chunk t + 2 stays in
//      flight across the barrier);
//   4. PReLU(x * in_scale) in place on the X rows the wave DMA'd itself;
//   5. the epilogue of the tile whose last chunk the MFMA waves finished in the
//      previous tick: accumulator image (+ split-K partials, fixed order)
//      + bias, zero past valid_len, residual 1, FiLM (bias / gamma / beta by
//      scalar loads), residual 2 -> buffer_store_dwordx4.
// A workgroup walks output tiles blockIdx.x, +gridDim.x, ... and its chunk
// stream runs across tile boundaries, so staging, MFMA and the stores of
// consecutive tiles overlap.  Tiles of one K chunk are refused (host): the
// single accumulator image needs a tick between two tiles' last chunks.
//
// LDS: ring of 3 stages {X [CC][SW] (SW = 64 NI + 32: channels 2p and 2p+1 in
// opposite bank halves), A [AG float4]}, the accumulator image
// [WK][BM][BN + 8] (+8: conflict-free MFMA-order writes), the residual tile
// [BM][BN].  B fragment of k-step (pair p, tap k): lane l reads
// X[2p + l/32][n + l%32 + k].
// ---------------------------------------------------------------------------
constexpr int kWsLoaders = 8;   // staging waves per workgroup (4 MFMA waves)

template <int KT, int CC, int WM, int WN, int WK, int MR, int NR, int S>
struct WCfg {
    static constexpr int NL = kWsLoaders;
    static constexpr int BM = 32 * WM * MR;
    static constexpr int BN = 32 * NR * WN;
    static constexpr int W = BN + KT - 1;                 // frames per chunk row
    static constexpr int NI = (W + 63) / 64;              // 64-frame DMA pieces per row
    static constexpr int SW = 64 * NI + 32;               // row stride (floats)
    static constexpr int XBUF = CC * SW;
    static constexpr int HQ = CC / 8;                     // 4-pair groups per chunk
    static constexpr int CPW = HQ / WK;                   // ... per MFMA wave
    static constexpr int AG = WM * MR * HQ * KT * 64;     // float4 of weights per chunk
    static constexpr int STAGE = XBUF + AG * 4;           // floats
    static constexpr int XPW = (CC / NL) * NI;            // X dword pieces per staging wave per chunk
    static constexpr int PQ = XBUF / 256;                 // X 16-B pieces per chunk (quad path)
    static constexpr int XPWQ = (PQ + NL - 1) / NL;       // ... per staging wave
    static constexpr int APW = (AG / 64 + NL - 1) / NL;   // A pieces per staging wave per chunk
    static constexpr int NPI = XPW + APW;                 // DMAs per staging wave per chunk
    static constexpr int NPIQ = XPWQ + APW;               // ... on the quad path
    static constexpr int OS = BN + 8;                     // accumulator image row stride
    static constexpr int OUT = S * STAGE;                 // accumulator image offset
    static constexpr int RES = OUT + WK * BM * OS;        // residual tile offset
    static constexpr int DUMMY = RES + BM * BN;           // sink of padding A pieces (never read)
    static constexpr int LDS = DUMMY + 256;               // floats
    static constexpr int G4 = BM * BN / 4;                // 16-B epilogue groups per tile
    static constexpr int GPT = G4 / (64 * NL);            // ... per staging thread
    static constexpr int RPP = 256 / BN;                  // rows per 64-group piece
    static_assert(G4 % (64 * NL) == 0 && 256 % BN == 0 && BN % 4 == 0 && CC % NL == 0, "staging mapping");
};

template <int KT, int CC, int WM, int WN, int WK, int MR, int NR, int S>
__global__ __launch_bounds__(256 + 64 * kWsLoaders) void conv_wkernel(ou_conv_desc d, int nchunks, int mtiles,
                                                    int64_t a_mt_stride, int ntn, int mgroups, int ntiles)
{
    using WC = WCfg<KT, CC, WM, WN, WK, MR, NR, S>;
    static_assert(CC % 8 == 0 && WC::HQ % WK == 0, "chunk must split into 4-pair groups per wave");
    static_assert(WM * WN * WK == 4, "4 MFMA waves");
    static_assert(S == 3, "3-stage ring (DMA two chunks ahead)");
    static_assert(WC::NPI <= 63 && WC::NPIQ <= 63, "vmcnt range");
    static_assert(WC::XBUF % 256 == 0 && WC::SW >= WC::BN + 8, "quad X pieces tile the window");
    // X staging path: "quad" (16-B DMA groups of 4 frames, lane-private
    // activation) when the frame view is the plain signal and 4-frame groups
    // align with sample 0; LDS column 0 is frame n0 - 4 there, n0 - pad on the
    // dword path
    const bool quad = d.frame == 1 && (d.shift & 3) == 0;
    const int xoff = quad ? 4 - d.pad : 0;
    OU_DYNAMIC_LDS(float4, lds4);
    float* lds = (float*)lds4;

    const int bx = (int)blockIdx.x, gx = (int)gridDim.x;
    const int nt_wg = bx < ntiles ? (ntiles - 1 - bx) / gx + 1 : 0;
    const int items = nt_wg * nchunks;   // (tile, chunk) work items of this workgroup
    const int M = d.m;

    // tile i of this workgroup -> (batch item, first frame, first m-tile)
    auto decode = [&](int i, int& b, int& n0, int& mt0) {
        const int tile = bx + i * gx;
        b = tile / (ntn * mgroups);
        const int r = tile - b * (ntn * mgroups);
        mt0 = (r / ntn) * (WM * MR);
        n0 = (r - (r / ntn) * ntn) * WC::BN;
    };

    if (threadIdx.x >= 256) {
        // ======================= staging waves ==============================
        const int tid = threadIdx.x - 256;
        const int lane = tid & 63;
        const int sw = __builtin_amdgcn_readfirstlane(tid >> 6);   // X rows [sw CC/NL, (sw+1) CC/NL)
        const int R = d.frame;
        const int cin = d.cin;
        const int in_len = d.in_len;
        const int xc = (int)d.x_cstride;
        const float slope = d.slope;
        const ou_ldsa_t lds0 = OU_LDS_ADDR(lds);
        const __amdgpu_buffer_rsrc_t wrs = ou_rsrc(d.w, (int64_t)mtiles * a_mt_stride * 4);
        const bool has_r1 = d.res1 != nullptr, has_r2 = d.res2 != nullptr, has_fm = d.film != nullptr;
        const float s1e = has_r1 ? d.s1 : 1.f, s2e = has_r2 ? d.s2 : 1.f, fadd = has_fm ? 0.f : 1.f;
        const int ulim = min(d.n_frames, d.out_len);
        const int r1c = (int)d.r1_cstride, r2c = (int)d.r2_cstride, yc = (int)d.y_cstride;

        auto issue_item = [&](int t) {
            const int i = t / nchunks;
            const int q = t - i * nchunks;
            int b, n0, mt0;
            decode(i, b, n0, mt0);
            const ou_ldsa_t st = lds0 + (unsigned)((t % S) * WC::STAGE * 4);
            const __amdgpu_buffer_rsrc_t xrs = ou_rsrc(d.x + (int64_t)b * d.x_bstride, (int64_t)cin * xc * 4);
            if (quad) {
                // 16-B piece p = 64 lanes x 4 frames of the [channel][frame] image
#pragma unroll
                for (int kk = 0; kk < WC::XPWQ; ++kk) {
                    const int p = sw * WC::XPWQ + kk;
                    const int e = 256 * p + 4 * lane;
                    const int row = e / WC::SW, col = e - (e / WC::SW) * WC::SW;
                    const int cq = q * CC + row;
                    const int smp = n0 - 4 + col + d.shift;
                    const bool ok = (int)(p < WC::PQ) & (int)(cq < cin) & (int)(smp >= 0) & (int)(smp + 3 < in_len);
                    ou_blds16(xrs, ok ? (unsigned)(cq * xc + smp) * 4u : (unsigned)kSentinel, 0u,
                              p < WC::PQ ? st + (unsigned)(256 * p * 4) : lds0 + (unsigned)(WC::DUMMY * 4));
                }
            } else {
            int fw[WC::NI];   // lane sample of each 64-frame piece (frame f -> sample f R + ph + shift)
#pragma unroll
            for (int pi = 0; pi < WC::NI; ++pi) fw[pi] = (n0 - d.pad + pi * 64 + lane) * R + d.shift;
            const int cq0 = q * CC + sw * (CC / WC::NL);
            int ph = cq0 / cin;
            int ci = cq0 - ph * cin;
#pragma unroll
            for (int c = 0; c < CC / WC::NL; ++c) {
                const bool chan_ok = ph < R;
                const unsigned soff = (unsigned)(chan_ok ? ci : 0) * (unsigned)xc * 4u;
                const ou_ldsa_t row = st + (unsigned)((sw * (CC / WC::NL) + c) * WC::SW * 4);
#pragma unroll
                for (int pi = 0; pi < WC::NI; ++pi) {
                    const int pos = fw[pi] + ph;
                    const bool ok = chan_ok & ((unsigned)pos < (unsigned)in_len);
                    ou_blds4(xrs, ok ? (unsigned)pos * 4u : (unsigned)kSentinel, soff, row + pi * 256);
                }
                if (++ci == cin) { ci = 0; ++ph; }
            }
            }
            const unsigned wbase = (unsigned)((mt0 * a_mt_stride + (int64_t)q * (WC::HQ * KT * 256)) * 4);
#pragma unroll
            for (int jj = 0; jj < WC::APW; ++jj) {
                const int j = sw * WC::APW + jj;            // piece = 64 float4
                if (j * 64 < WC::AG) {
                    const int ml = j / (WC::HQ * KT);        // m-tile of the piece
                    const unsigned soff = wbase + (unsigned)(ml * a_mt_stride * 4) +
                                          (unsigned)((j - ml * (WC::HQ * KT)) * 1024);
                    ou_blds16(wrs, mt0 + ml < mtiles ? (unsigned)lane * 16u : (unsigned)kSentinel, soff,
                              st + (unsigned)((WC::XBUF + j * 256) * 4));
                } else {   // same DMA count in every staging wave
                    ou_blds16(wrs, (unsigned)kSentinel, 0u, lds0 + (unsigned)(WC::DUMMY * 4));
                }
            }
        };
        // epilogue group k of this thread: piece (sw + NL k) of the row-major tile, lane's group in it
        auto group_of = [&](int k, int& row, int& c4) {
            const int g = (sw + WC::NL * k) * 64 + lane;
            row = g / (WC::BN / 4);
            c4 = g - row * (WC::BN / 4);
        };
        // residual 1 of tile i: full groups by LDS-DMA into this lane's slots of the residual tile
        auto issue_res = [&](int i) {
            int b, n0, mt0;
            decode(i, b, n0, mt0);
            const __amdgpu_buffer_rsrc_t r1s = ou_rsrc(has_r1 ? d.res1 + (int64_t)b * d.r1_bstride : d.y,
                                                       has_r1 ? (int64_t)M * r1c * 4 : 0);
#pragma unroll
            for (int k = 0; k < WC::GPT; ++k) {
                int row, c4;
                group_of(k, row, c4);
                const int m = mt0 * 32 + row, u = n0 + 4 * c4;
                const bool full = (int)(m < M) & (int)(u + 3 < ulim);
                ou_blds16(r1s, full ? (unsigned)(m * r1c + u) * 4u : (unsigned)kSentinel, 0u,
                          lds0 + (unsigned)((WC::RES + (sw + WC::NL * k) * 256) * 4));
            }
        };
        // PReLU(x * in_scale) in place on this wave's X rows of item t
        auto prelu_item = [&](int t) {
            const int i = t / nchunks;
            int b, n0, mt0;
            decode(i, b, n0, mt0);
            const float sc = d.in_scale ? d.in_scale[b] : 1.0f;
            if (quad) {   // the groups this lane DMA'd itself; the right edge's partial group by plain loads
                const int q = t - i * nchunks;
                float4* x4 = (float4*)(lds + (t % S) * WC::STAGE);
#pragma unroll
                for (int kk = 0; kk < WC::XPWQ; ++kk) {
                    const int p = sw * WC::XPWQ + kk;
                    if (p < WC::PQ) {
                        float4 v = x4[64 * p + lane];
                        const int e = 256 * p + 4 * lane;
                        const int row = e / WC::SW, col = e - (e / WC::SW) * WC::SW;
                        const int cq = q * CC + row;
                        const int smp = n0 - 4 + col + d.shift;
                        if (cq < cin && smp < in_len && smp + 3 >= in_len && smp >= 0) {
                            const float* xr = d.x + (int64_t)b * d.x_bstride + (int64_t)cq * xc + smp;
                            v.x = xr[0];
                            v.y = smp + 1 < in_len ? xr[1] : 0.f;
                            v.z = smp + 2 < in_len ? xr[2] : 0.f;
                            v.w = 0.f;
                        }
                        v.x *= sc; v.y *= sc; v.z *= sc; v.w *= sc;
                        v.x = v.x >= 0.f ? v.x : v.x * slope;
                        v.y = v.y >= 0.f ? v.y : v.y * slope;
                        v.z = v.z >= 0.f ? v.z : v.z * slope;
                        v.w = v.w >= 0.f ? v.w : v.w * slope;
                        x4[64 * p + lane] = v;
                    }
                }
                return;
            }
            float4* xs = (float4*)(lds + (t % S) * WC::STAGE + sw * (CC / WC::NL) * WC::SW);
            constexpr int N4 = (CC / WC::NL) * WC::SW / 4;
#pragma unroll
            for (int k = 0; k < (N4 + 63) / 64; ++k) {
                const int f = lane + 64 * k;
                if (N4 % 64 == 0 || f < N4) {
                    float4 v = xs[f];
                    v.x *= sc; v.y *= sc; v.z *= sc; v.w *= sc;
                    v.x = v.x >= 0.f ? v.x : v.x * slope;
                    v.y = v.y >= 0.f ? v.y : v.y * slope;
                    v.z = v.z >= 0.f ? v.z : v.z * slope;
                    v.w = v.w >= 0.f ? v.w : v.w * slope;
                    xs[f] = v;
                }
            }
        };
        auto epilogue = [&](int i) {
            int b, n0, mt0;
            decode(i, b, n0, mt0);
            const __amdgpu_buffer_rsrc_t ys = ou_rsrc(d.y + (int64_t)b * d.y_bstride, (int64_t)M * yc * 4);
            const __amdgpu_buffer_rsrc_t r1s = ou_rsrc(has_r1 ? d.res1 + (int64_t)b * d.r1_bstride : d.y,
                                                       has_r1 ? (int64_t)M * r1c * 4 : 0);
            const __amdgpu_buffer_rsrc_t r2s = ou_rsrc(has_r2 ? d.res2 + (int64_t)b * d.r2_bstride : d.y,
                                                       has_r2 ? (int64_t)M * r2c * 4 : 0);
            const float* fmb = has_fm ? d.film + (int64_t)b * d.film_bstride : nullptr;
            const float* out = lds + WC::OUT;
#pragma unroll
            for (int k = 0; k < WC::GPT; ++k) {
                int row, c4;
                group_of(k, row, c4);
                const int m = mt0 * 32 + row, u = n0 + 4 * c4;
                const bool mok = m < M;
                const bool full = mok & (u + 3 < ulim);
                // per-row operands by scalar loads: the piece spans rows
                // row0 .. row0 + RPP - 1 (wave-uniform row0)
                const int row0 = ((sw + WC::NL * k) * 64) / (WC::BN / 4);
                float pb = 0.f, pa = 0.f, pf = 0.f;
#pragma unroll
                for (int rr = 0; rr < WC::RPP; ++rr) {
                    const int mm = min(mt0 * 32 + row0 + rr, M - 1);
                    const float bb = d.bias ? d.bias[mm] : 0.f;
                    const float aa = fmb ? fmb[mm] : 0.f;
                    const float ff = fmb ? fmb[M + mm] : 0.f;
                    if (row == row0 + rr) { pb = bb; pa = aa; pf = ff; }
                }
                float4 a = *(const float4*)(out + row * WC::OS + 4 * c4);
#pragma unroll
                for (int j = 1; j < WK; ++j) {   // split-K partials, fixed order
                    const float4 p = *(const float4*)(out + (j * WC::BM + row) * WC::OS + 4 * c4);
                    a.x += p.x; a.y += p.y; a.z += p.z; a.w += p.w;
                }
                float4 r1 = *(const float4*)(lds + WC::RES + ((sw + WC::NL * k) * 64 + lane) * 4);
                float r2v[4] = {0.f, 0.f, 0.f, 0.f};
                if (!full) {   // tile edge: per-element residual 1 (the DMA skipped the group)
                    float t1[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        t1[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                            r1s, (mok & (u + e < ulim)) ? (m * r1c + u + e) * 4 : kSentinel, 0, 0));
                    r1 = make_float4(t1[0], t1[1], t1[2], t1[3]);
                }
                if (has_r2) {   // rare: plain loads
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        r2v[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                            r2s, (mok & (u + e < ulim)) ? (m * r2c + u + e) * 4 : kSentinel, 0, 0));
                }
                float v[4] = {a.x, a.y, a.z, a.w};
                const float r1v[4] = {r1.x, r1.y, r1.z, r1.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float x = v[e] + pb;
                    if (u + e >= d.valid_len) x = 0.f;
                    x = (x + r1v[e]) * s1e;
                    x = (pa + fadd) * x + pf;
                    x = (x + r2v[e]) * s2e;
                    v[e] = x;
                }
                if (full) {
                    __builtin_amdgcn_raw_buffer_store_b128(
                        (__attribute__((ext_vector_type(4))) unsigned){__float_as_uint(v[0]), __float_as_uint(v[1]),
                                                                        __float_as_uint(v[2]), __float_as_uint(v[3])},
                        ys, (m * yc + u) * 4, 0, 0);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        __builtin_amdgcn_raw_buffer_store_b32(
                            __float_as_uint(v[e]), ys, (mok & (u + e < ulim)) ? (m * yc + u + e) * 4 : kSentinel, 0, 0);
                }
            }
        };

        // prologue: chunks 0, 1 in flight; chunk 0 landed and activated
        OU_WSTAMP_INIT
        for (int t = 0; t < 2 && t < items; ++t) issue_item(t);
        if (items >= 2) {
            if (quad) OU_WAIT_VMCNT(WC::NPIQ);
            else OU_WAIT_VMCNT(WC::NPI);
        } else {
            OU_WAIT_VMCNT0();
        }
        if (items > 0) prelu_item(0);
        __syncthreads();
        for (int t = 0; t < items; ++t) {
            const int q = t % nchunks;
            // the tile the MFMA waves finished last tick (its image is complete)
            const int fin = (t > 0 && q == 0) ? t / nchunks - 1 : -1;
            OU_WSTAMP(5);
            if (t + 2 < items) issue_item(t + 2);
            OU_WSTAMP(0);
            // chunk t + 1 (and everything older) landed; chunk t + 2 stays in flight
            if (t + 2 < items) {
                if (quad) OU_WAIT_VMCNT(WC::NPIQ);
                else OU_WAIT_VMCNT(WC::NPI);
            } else {
                OU_WAIT_VMCNT0();
            }
            OU_WSTAMP(1);
            if (t + 1 < items) prelu_item(t + 1);
            OU_WSTAMP(3);
            if (fin >= 0) epilogue(fin);
            OU_WSTAMP(4);
            if (q == nchunks - 1) {
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this lane's RES reads are done
                issue_res(t / nchunks);
            }
            OU_WSTAMP(5);
            __syncthreads();
            OU_WSTAMP(2);
        }
        // the last tile: its chunk finished before the final barrier
        if (items > 0) {
            OU_WAIT_VMCNT0();
            epilogue(items / nchunks - 1);
        }
        OU_WSTAMP(4);
        OU_WSTAMP_SAVE(threadIdx.x == 256, 8);
        return;
    }

    // ========================= MFMA waves ===================================
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave % WN;
    const int wm = (wave / WN) % WM;
    const int wk = wave / (WN * WM);
    const int h = lane >> 5;
    const int l32 = lane & 31;

    floatx16 acc[MR][NR];
    OU_WSTAMP_INIT
    __syncthreads();
    OU_WSTAMP(4);
    for (int t = 0; t < items; ++t) {
        const int q = t % nchunks;
        if (q == 0) {
#pragma unroll
            for (int a = 0; a < MR; ++a)
#pragma unroll
                for (int c = 0; c < NR; ++c)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;
        }
        {
            const float* xs = lds + (t % S) * WC::STAGE;
            const float4* ap = (const float4*)(xs + WC::XBUF) + ((wm * MR) * WC::HQ + wk * WC::CPW) * KT * 64 + lane;
            // lane's B column: row 2p + h, frame wn*32*NR + nr*32 + l32 + tap
            const float* xp = xs + (8 * wk * WC::CPW + h) * WC::SW + wn * 32 * NR + l32 + xoff;
            constexpr int NS = WC::CPW * KT;
            float4 fa[2][MR];
            float fb[2][4][NR];
            auto frag = [&](int st, float4* a, float (*bq)[NR]) {
                const int cpq = st / KT, k = st - (st / KT) * KT;
#pragma unroll
                for (int mr = 0; mr < MR; ++mr) a[mr] = ap[((mr * WC::HQ + cpq) * KT + k) * 64];
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int nr = 0; nr < NR; ++nr) bq[j][nr] = xp[(2 * (4 * cpq + j)) * WC::SW + nr * 32 + k];
            };
            frag(0, fa[0], fb[0]);
#pragma unroll
            for (int st = 0; st < NS; ++st) {
                if (st + 1 < NS) frag(st + 1, fa[(st + 1) & 1], fb[(st + 1) & 1]);
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                        for (int nr = 0; nr < NR; ++nr)
                            acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                                fa[st & 1][mr][j], fb[st & 1][j][nr], acc[mr][nr], 0, 0, 0);
            }
        }
        OU_WSTAMP(1);
        if (q == nchunks - 1) {   // accumulator image: [wk][row][col]
            float* out = lds + WC::OUT + wk * WC::BM * WC::OS;
#pragma unroll
            for (int mr = 0; mr < MR; ++mr)
#pragma unroll
                for (int nr = 0; nr < NR; ++nr)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        out[((wm * MR + mr) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * WC::OS + wn * 32 * NR + nr * 32 +
                            l32] = acc[mr][nr][r];
        }
        OU_WSTAMP(2);
        __syncthreads();
        OU_WSTAMP(3);
    }
    OU_WSTAMP_SAVE(threadIdx.x == 0, 0);
}

// ---------------------------------------------------------------------------
// Anti-aliased rate-change convolutions with the FIR applied (tile bit 17,
// ou_conv_desc.fir).
//
// PReLU_Conv with use_antialiasing runs a (2R+1)-tap binomial FIR
// (blocks.py:66-72, 123-134) before a strided conv (down, blocks.py:214-218)
// or after a transposed one (up, blocks.py:221-225).  Folded into the weights
// (engine.spec_down / spec_up, the kernels above) that is a 3-frame polyphase
// kernel: three times the reference's dense MACs.  These two kernels keep the
// reference's factorisation -- the GEMM has one tap and K = cin R (down) or
// cin (up) -- and run the FIR on the VALU:
//   conv_fdkernel (down): while a K chunk (16 channels x R phases) is staged,
//     thread (channel c, frame group g) holds F R + 2 R consecutive PReLU'd
//     samples of its channel in registers, slides the FIR over them and
//     writes the F R results, split into f16 hi / lo, into the B image
//     [frame][16 channels][phase] (channel-major K: a frame's R phases are one
//     16 / 8 / 4-B store; row stride 16 R + 8 halves, an odd number of 16-B
//     slots, so the ds_read_b128 fragment reads are conflict-free);
//   conv_fukernel (up): the workgroup computes the transposed conv over BN
//     frames (one frame of halo each side: BN - 2 output frames), keeping
//     P = 32 / R whole channels per 32-row m-tile (packed rows 32 (co / P) +
//     (co % P) R + ph), writes the results to LDS as sample rows, and each
//     thread runs the FIR over 4 consecutive output samples of a channel
//     before bias, residuals and the store.
// The weights (ou_conv_pack_split_nat order, include/ouhip.h) stream from L2
// through a register ring one K chunk deep (the slot a step's MFMAs used is
// refilled with the next chunk's same step); B is double-buffered in LDS, one
// barrier per chunk.  Split-f16 (P 1: three MFMAs per k-step) or f16 (P 2).
//
// conv_fdkernel<..., ST = 1> (ou_conv_desc.fir 3) is the same kernel without
// the FIR for the conditioner's wide strided st_convs (condition.py:53-59:
// kernel = stride = Rt of 20 .. 240): K = cin Rt in the same channel-block
// order, walked as chunks of 16 channels x R phases (R = 4 or 8 dividing Rt),
// the R phases of every frame being one contiguous run of samples -- so a
// workgroup reads each input sample once (the frame-view kernels' phase-major
// chunks re-read every line once per chunk of phases).
// ---------------------------------------------------------------------------
[[maybe_unused]] constexpr int kFirBit = 1 << 17;
// tile bit 9 (down fir 1 without residuals / FiLM, up without bit 8): two
// input chunks in flight per thread (PD = 2) -- the raw x window of chunk
// q + 2 is requested while chunk q's MFMAs run, for the layers whose chunks
// are too short to cover an HBM round trip; costs 10-60 VGPRs
[[maybe_unused]] constexpr int kFirDeep = 1 << 9;
[[maybe_unused]] constexpr int kFirEarly = 1 << 8;   // up (fir 2): epilogue loads before the main loop

template <int R, int WM, int WN, int MR, int NR>
struct FCfg {
    static_assert(WM * WN == 4, "4 waves per workgroup");
    static constexpr int BM = 32 * WM * MR;
    static constexpr int BN = 32 * WN * NR;
    static constexpr int NT = 2 * R + 1;            // FIR taps
    // down: K chunk = 16 channels x R phases (R k-steps); B row (frame) [ph][16 ch]
    static constexpr int DRS = 16 * R + 8;          // halves (DRS / 8 = 2 R + 1 slots: odd)
    static constexpr int DF = BN / 16;              // frames per staging thread (16 per channel)
    static constexpr int DWIN = (DF + 2) * R;       // window samples per staging thread
    static constexpr int DPLANE = BN * DRS;         // halves per plane
    static constexpr int DLDS = 2 * 2 * DPLANE * 2; // bytes: 2 buffers x (hi, lo)
    // up: K chunk = 32 channels (2 k-steps); B row (frame) [32 ch]
    static constexpr int URS = 32 + 8;
    static constexpr int UPLANE = BN * URS;
    static constexpr int UIT = 4 * BN;              // staging items: 8 channels x 1 frame
    static constexpr int UIE = (UIT + 255) / 256;
    static constexpr int CPT = 32 / R;              // up: whole channels per 32-row m-tile
    static constexpr int UCH = WM * MR * CPT;       // up: channels per workgroup
    static constexpr int YRS = BN * R + 8;          // up: sample-row stride of the Y image (floats)
    static constexpr int ULDS_B = 2 * 2 * UPLANE * 2;
    static constexpr int ULDS_Y = UCH * YRS * 4;
    static constexpr int ULDS = ULDS_B > ULDS_Y ? ULDS_B : ULDS_Y;
};

// FIR taps of one launch (uniform addresses: scalar loads)
template <int NT>
__device__ __forceinline__ void fir_taps(const ou_conv_desc& d, float (&tap)[NT])
{
#pragma unroll
    for (int j = 0; j < NT; ++j) tap[j] = d.fir_taps[j];
}

// The down / st_conv epilogue when the layer has no residuals and no FiLM (the
// rate-change convs of the encoders and the st_convs): bias, zero-fill past
// valid_len, the store and the optional split image -- a fraction of
// conv_epilogue's registers, so more workgroups stay resident per CU.
template <int MR, int NR>
__device__ __forceinline__ void conv_epilogue_lean(const ou_conv_desc& d, int b, int mtb, int ub,
                                                   floatx16 (&acc)[MR][NR], int lane, int col)
{
    const int h = lane >> 5, l32 = col;
    const int M = d.m;
    const __amdgpu_buffer_rsrc_t ys = ou_rsrc(d.y + (int64_t)b * d.y_bstride, (int64_t)M * d.y_cstride * 4);
    const __amdgpu_buffer_rsrc_t bs = ou_rsrc(d.bias, d.bias ? (int64_t)M * 4 : 0);
    const SplitOut so = split_ctx(d, b, M);
    const int uend = min(d.f0 + d.n_frames, d.out_len);
    float somax = 0.f;
#pragma unroll
    for (int mr = 0; mr < MR; ++mr) {
        const int m0 = (mtb + mr) * 32 + 4 * h;   // rows m0 + (r & 3) + 8 (r >> 2)
        float bias[16];
#pragma unroll
        for (int r = 0; r < 16; ++r)
            bias[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bs, min(m0 + (r & 3) + 8 * (r >> 2), M - 1) * 4, 0, 0));
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
            const int u = ub + nr * 32 + l32;
            const bool uok = u < uend;
            const bool zero = u >= d.valid_len;
            float sv[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + (r & 3) + 8 * (r >> 2);
                const float v = zero ? 0.f : acc[mr][nr][r] + bias[r];
                sv[r] = v;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ys,
                                                      (uok && m < M) ? (m * (int)d.y_cstride + u) * 4 : kSentinel, 0, 0);
            }
            if (d.sy) {
                const bool ok = (mtb + mr) * 32 < M && uok;
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    split_store4(so, m0 + 8 * g, u, ok, sv[4 * g], sv[4 * g + 1], sv[4 * g + 2], sv[4 * g + 3], somax);
            }
        }
    }
    if (d.sy) ou_range_flag(d.status, somax, 2, lane);
}

template <int R, int WM, int WN, int MR, int NR, int P, int ST = 0, int LEAN = 0, int PD = 1>
__global__ __launch_bounds__(256) void conv_fdkernel(ou_conv_desc d, int mtiles, int64_t a_mt_stride)
{
    using F = FCfg<R, WM, WN, MR, NR>;
    constexpr int WIN = ST ? F::DF * R : F::DWIN;   // window samples per staging thread
    ou_kernarg_prefetch8();
    OU_DYNAMIC_LDS(float4, lds4);
    _Float16* ldsh = (_Float16*)lds4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave % WN, wm = wave / WN;
    const int h = lane >> 5, l32 = lane & 31;
    int bx, by, bz;
    if (d.tile & kMajBit) ou_xcd_block_m(bx, by, bz); else ou_xcd_block(bx, by, bz);
    const int b = bz;
    const int n0 = bx * F::BN + d.f0;     // first output frame (global)
    const int mt0 = by * (WM * MR);
    const int in_len = d.in_len;
    const int Rt = ST ? d.frame : R;      // samples per frame
    const int nsub = Rt / R;              // chunks (of R phases) per 16-channel block
    const int nch = d.cin / 16 * nsub;    // K chunks: block cb = q / nsub, phases (q % nsub) R ..
    const float xsc = ou_exp2i(-d.xs_shift), su = d.w_unscale * ou_exp2i(d.xs_shift - kSplitShift);
    const float slope = d.slope;
    float tap[F::NT];
    if constexpr (!ST) fir_taps<F::NT>(d, tap);

    // ---- weights: chunk q (16 channels x R phases, channel-major), step s =
    // its K values 16 s .. 16 s + 15
    const __amdgpu_buffer_rsrc_t ars = ou_rsrc(d.w, (int64_t)mtiles * a_mt_stride * 4);
    half8_t ra[R][MR][2];
    auto load_a = [&](int q, int s) {   // q uniform, clamped (a reload past the end is never used)
        q = min(q, nch - 1);
#pragma unroll
        for (int mr = 0; mr < MR; ++mr) {
            const int mt = min(mt0 + wm * MR + mr, mtiles - 1);
            const unsigned so = (unsigned)(mt * a_mt_stride * 4 + (int64_t)(q * R + s) * 2048);
            ra[s][mr][0] = __builtin_bit_cast(half8_t, __builtin_amdgcn_raw_buffer_load_b128(ars, lane * 16, so, 0));
            if constexpr (P == 1)
                ra[s][mr][1] = __builtin_bit_cast(half8_t, __builtin_amdgcn_raw_buffer_load_b128(ars, lane * 16, so + 1024, 0));
        }
    };

    // ---- staging: thread (channel sc of the chunk, frame group sg) owns
    // frames n0 + sg F .. + F - 1; its window is samples [s0, s0 + (F + 2) R)
    // (ST: the R-sample runs (n0 + sg F + f) Rt + sub R .. of its F frames f).
    // Frame groups fastest (neighbouring lanes read neighbouring windows); a
    // frame's R phases are R consecutive halves sc R .. of its B row
    // (channel-major K: one 16 / 8 / 4-B store), and the rows interleave the
    // groups inside each 32-frame tile -- frame 32 t + g F + f (group g of the
    // S = 32 / F groups of tile t) at row 32 t + f S + g -- so the lanes of a
    // store hit consecutive rows (odd 16-B-slot stride: <= 2-way conflicts).
    // The MFMA column of B row 32 t + j is frame 32 t + FCOL(j) (epilogue).
    const int sg = tid & 15, sc = tid >> 4;
    constexpr int SG = 32 / F::DF;   // frame groups per 32-frame tile
    const int srow = (sg / SG) * 32 + sg % SG;
    const int64_t xc = d.x_cstride;
    const __amdgpu_buffer_rsrc_t xrs = ou_rsrc(d.x + (int64_t)b * d.x_bstride, (int64_t)d.cin * xc * 4);
    const int s0 = ST ? (n0 + sg * F::DF) * Rt : (n0 + sg * F::DF - 1) * R;
    // 16-B (R % 4 == 0) / 8-B (R == 2) loads where every row start is aligned
    constexpr int V = R % 4 == 0 ? 4 : (R == 2 ? 2 : 1);
    const bool vec = V > 1 && ((uintptr_t)d.x % (4 * V)) == 0 && d.x_bstride % V == 0 && xc % V == 0;
    float xws[PD][WIN];   // PD raw windows in flight
    auto stage_load = [&](int q, float (&xw)[WIN]) {   // q uniform, clamped (the extra load is never stored)
        q = min(q, nch - 1);
        const int cb = ST ? q / nsub : q;
        const int row = (cb * 16 + sc) * (int)xc;
        const int sb = ST ? s0 + (q - cb * nsub) * R : s0;   // the chunk's first sample
        if (vec) {
#pragma unroll
            for (int e = 0; e < WIN; e += V) {
                // a multiple of V: a group lies wholly left of 0 or right of it
                const int smp = sb + (ST ? (e / R) * Rt + e % R : e);
                const int off = (smp >= 0 && smp < in_len) ? (row + smp) * 4 : kSentinel;
                if constexpr (V == 4) {
                    const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0);
#pragma unroll
                    for (int j = 0; j < 4; ++j) xw[e + j] = smp + j < in_len ? __uint_as_float(v4[j]) : 0.f;
                } else {
                    const auto v2 = __builtin_amdgcn_raw_buffer_load_b64(xrs, off, 0, 0);
#pragma unroll
                    for (int j = 0; j < 2; ++j) xw[e + j] = smp + j < in_len ? __uint_as_float(v2[j]) : 0.f;
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < WIN; ++e) {
                const int smp = sb + (ST ? (e / R) * Rt + e % R : e);
                xw[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                    xrs, (smp >= 0 && smp < in_len) ? (row + smp) * 4 : kSentinel, 0, 0));
            }
        }
    };
    float omax = 0.f;
    // stores of VW consecutive halves (a frame's phases): 16 / 8 / 4 / 2 B
    constexpr int VW = R % 8 == 0 ? 8 : R % 4 == 0 ? 4 : R % 2 == 0 ? 2 : 1;
    auto store_h = [](_Float16* p, const _Float16 (&v)[VW]) {
        if constexpr (VW == 8) {
            *(half8_t*)p = half8_t{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
        } else if constexpr (VW == 4) {
            *(ou_h4_t*)p = ou_h4_t{v[0], v[1], v[2], v[3]};
        } else if constexpr (VW == 2) {
            *(uint32_t*)p = (uint32_t)__builtin_bit_cast(uint16_t, v[0]) |
                            ((uint32_t)__builtin_bit_cast(uint16_t, v[1]) << 16);
        } else {
            *p = v[0];
        }
    };
    auto stage_store = [&](int buf, float (&xw)[WIN]) {
        _Float16* bh = ldsh + buf * 2 * F::DPLANE + srow * F::DRS + sc * R;
#pragma unroll
        for (int e = 0; e < WIN; ++e) {
            const float v = xw[e] * xsc;   // 2^-s: exact
            xw[e] = v >= 0.f ? v : v * slope;
        }
#pragma unroll
        for (int f = 0; f < F::DF; ++f)
#pragma unroll
            for (int p0 = 0; p0 < R; p0 += VW) {
                _Float16 hv[VW], lv[VW];
#pragma unroll
                for (int j = 0; j < VW; ++j) {
                    const int i = f * R + p0 + j;
                    float v = 0.f;
                    if constexpr (ST) {
                        v = xw[i];
                    } else {
#pragma unroll
                        for (int t = 0; t < F::NT; ++t) v = fmaf(tap[t], xw[i + t], v);
                    }
                    omax = fmaxf(omax, __builtin_fabsf(v));
                    hv[j] = (_Float16)v;
                    lv[j] = (_Float16)((v - (float)hv[j]) * 2048.f);
                }
                _Float16* o = bh + f * SG * F::DRS + p0;
                store_h(o, hv);
                if constexpr (P == 1) store_h(o + F::DPLANE, lv);
            }
    };

    floatx16 acc[MR][NR];
    floatx16 accx[P == 1 ? MR : 1][P == 1 ? NR : 1];
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    if constexpr (P == 1) {
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
            for (int j = 0; j < NR; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) accx[i][j][r] = 0.f;
    }
    // B fragments of (buffer, step s): row wn 32 NR + nr 32 + l32, halves s 16 + 8 h
    const _Float16* bb = ldsh + (wn * 32 * NR + l32) * F::DRS + 8 * h;
    auto mfma_step = [&](int buf, int s) {
        half8_t bq[NR], bl[NR];
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
            const _Float16* p = bb + buf * 2 * F::DPLANE + nr * 32 * F::DRS + s * 16;
            bq[nr] = *(const half8_t*)p;
            if constexpr (P == 1) bl[nr] = *(const half8_t*)(p + F::DPLANE);
        }
#pragma unroll
        for (int mr = 0; mr < MR; ++mr)
#pragma unroll
            for (int nr = 0; nr < NR; ++nr) {
                acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s][mr][0], bq[nr], acc[mr][nr], 0, 0, 0);
                if constexpr (P == 1) {
                    accx[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s][mr][0], bl[nr], accx[mr][nr], 0, 0, 0);
                    accx[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s][mr][1], bq[nr], accx[mr][nr], 0, 0, 0);
                }
            }
    };

#pragma unroll
    for (int j = 0; j < PD; ++j) stage_load(j, xws[j]);
#pragma unroll
    for (int s = 0; s < R; ++s) load_a(0, s);
    stage_store(0, xws[0]);
    __syncthreads();
    if constexpr (PD == 1) {   // (kept as its own loop: the generic one measured slower at PD 1)
        for (int q = 0; q < nch; ++q) {
            const int cur = q & 1;
            stage_load(q + 1, xws[0]);   // the next chunk's window, in flight under this chunk's MFMAs
#pragma unroll
            for (int s = 0; s < R; ++s) {
                mfma_step(cur, s);
                load_a(q + 1, s);   // refill the slot just used
            }
            if (q + 1 < nch) stage_store(cur ^ 1, xws[0]);
            __syncthreads();
        }
    } else {
        for (int q0 = 0; q0 < nch; q0 += PD) {
#pragma unroll
            for (int j = 0; j < PD; ++j) {   // chunk q: window set j (stored), set j + 1 holds chunk q + 1
                const int q = q0 + j;
                if (q >= nch) break;
                const int cur = q & 1;
                stage_load(q + PD, xws[j]);   // in flight under the next PD chunks' MFMAs (clamped)
#pragma unroll
                for (int s = 0; s < R; ++s) {
                    mfma_step(cur, s);
                    load_a(q + 1, s);   // refill the slot just used
                }
                if (q + 1 < nch) stage_store(cur ^ 1, xws[(j + 1) % PD]);
                __syncthreads();
            }
        }
    }
    if constexpr (P != 0) ou_range_flag(d.status, omax, 1, lane);
    const float sx = su * (1.f / 2048.f);
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                acc[i][j][r] = P == 1 ? fmaf(accx[i][j][r], sx, acc[i][j][r] * su) : acc[i][j][r] * su;
    const int col = (l32 % SG) * F::DF + l32 / SG;   // FCOL: this lane's frame in its 32-frame tile
    if constexpr (LEAN)
        conv_epilogue_lean<MR, NR>(d, b, mt0 + wm * MR, n0 + wn * (32 * NR), acc, lane, col);
    else
        conv_epilogue<MR, NR>(d, b, mt0 + wm * MR, n0 + wn * (32 * NR), acc, lane, col);
}

template <int R, int WM, int WN, int MR, int NR, int P, int EARLY = 0, int PD = 1>
__global__ __launch_bounds__(256) void conv_fukernel(ou_conv_desc d, int mtiles, int64_t a_mt_stride)
{
    using F = FCfg<R, WM, WN, MR, NR>;
    constexpr int BNO = F::BN - 2;        // output frames per workgroup (one halo frame each side)
    ou_kernarg_prefetch8();
    OU_DYNAMIC_LDS(float4, lds4);
    _Float16* ldsh = (_Float16*)lds4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave % WN, wm = wave / WN;
    const int h = lane >> 5, l32 = lane & 31;
    int bx, by, bz;
    if (d.tile & kMajBit) ou_xcd_block_m(bx, by, bz); else ou_xcd_block(bx, by, bz);
    const int b = bz;
    const int u0 = bx * BNO + d.f0;       // first output frame
    const int fa = u0 - 1;                // frame of B row 0
    const int mt0 = by * (WM * MR);       // first packed m-tile
    const int in_len = d.in_len;
    const int nch = d.cin / 32;
    const int cout = d.m / R;
    const float xsc = ou_exp2i(-d.xs_shift), su = d.w_unscale * ou_exp2i(d.xs_shift - kSplitShift);
    const float slope = d.slope;

    const __amdgpu_buffer_rsrc_t ars = ou_rsrc(d.w, (int64_t)mtiles * a_mt_stride * 4);
    half8_t ra[2][MR][2];
    auto load_a = [&](int q, int s) {
        q = min(q, nch - 1);
#pragma unroll
        for (int mr = 0; mr < MR; ++mr) {
            const int mt = min(mt0 + wm * MR + mr, mtiles - 1);
            const unsigned so = (unsigned)(mt * a_mt_stride * 4 + (int64_t)(q * 2 + s) * 2048);
            ra[s][mr][0] = __builtin_bit_cast(half8_t, __builtin_amdgcn_raw_buffer_load_b128(ars, lane * 16, so, 0));
            if constexpr (P == 1)
                ra[s][mr][1] = __builtin_bit_cast(half8_t, __builtin_amdgcn_raw_buffer_load_b128(ars, lane * 16, so + 1024, 0));
        }
    };

    // ---- staging: item it = (8-channel group cg = it / BN, row n = it % BN)
    const int64_t xc = d.x_cstride;
    const __amdgpu_buffer_rsrc_t xrs = ou_rsrc(d.x + (int64_t)b * d.x_bstride, (int64_t)d.cin * xc * 4);
    float xvs[PD][F::UIE][8];   // PD chunks in flight
    auto stage_load = [&](int q, float (&xv)[F::UIE][8]) {
        q = min(q, nch - 1);
#pragma unroll
        for (int e = 0; e < F::UIE; ++e) {
            const int it = tid + 256 * e;
            const int n = it % F::BN, cg = it / F::BN;
            const int u = fa + n;
            const bool ok = it < F::UIT && u >= 0 && u < in_len;
            const int base = ok ? ((q * 32 + cg * 8) * (int)xc + u) * 4 : kSentinel;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                xv[e][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, base, ok ? j * (int)xc * 4 : 0, 0));
        }
    };
    float omax = 0.f;
    auto stage_store = [&](int buf, float (&xv)[F::UIE][8]) {
        _Float16* bh = ldsh + buf * 2 * F::UPLANE;
#pragma unroll
        for (int e = 0; e < F::UIE; ++e) {
            const int it = tid + 256 * e;
            if (F::UIT % 256 != 0 && it >= F::UIT) continue;
            const int n = it % F::BN, cg = it / F::BN;
            half8_t hi, lo;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float v = xv[e][j] * xsc;
                v = v >= 0.f ? v : v * slope;
                omax = fmaxf(omax, __builtin_fabsf(v));
                hi[j] = (_Float16)v;
                lo[j] = (_Float16)((v - (float)hi[j]) * 2048.f);
            }
            *(half8_t*)(bh + n * F::URS + cg * 8) = hi;
            if constexpr (P == 1) *(half8_t*)(bh + F::UPLANE + n * F::URS + cg * 8) = lo;
        }
    };

    floatx16 acc[MR][NR];
    floatx16 accx[P == 1 ? MR : 1][P == 1 ? NR : 1];
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    if constexpr (P == 1) {
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
            for (int j = 0; j < NR; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) accx[i][j][r] = 0.f;
    }
    const _Float16* bb = ldsh + (wn * 32 * NR + l32) * F::URS + 8 * h;
    auto mfma_step = [&](int buf, int s) {
        half8_t bq[NR], bl[NR];
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
            const _Float16* p = bb + buf * 2 * F::UPLANE + nr * 32 * F::URS + s * 16;
            bq[nr] = *(const half8_t*)p;
            if constexpr (P == 1) bl[nr] = *(const half8_t*)(p + F::UPLANE);
        }
#pragma unroll
        for (int mr = 0; mr < MR; ++mr)
#pragma unroll
            for (int nr = 0; nr < NR; ++nr) {
                acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s][mr][0], bq[nr], acc[mr][nr], 0, 0, 0);
                if constexpr (P == 1) {
                    accx[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s][mr][0], bl[nr], accx[mr][nr], 0, 0, 0);
                    accx[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s][mr][1], bq[nr], accx[mr][nr], 0, 0, 0);
                }
            }
    };

    // ---- epilogue operands: item it = (channel cw = it / NSG, 4-sample group
    // g).  EARLY (tile bit 8): the skip residual (the up conv's res1) and the
    // bias of every item of this thread are requested before the main loop, so
    // their HBM round trip overlaps the GEMM instead of following the FIR (at
    // the price of 20-60 VGPRs held across it; the tuner times both)
    const int ylen = d.out_len, vlen = d.valid_len;
    const int tend = min((min(u0 + BNO, d.f0 + d.n_frames)) * R, ylen);   // samples [u0 R, tend) are stored
    const int c0 = mt0 * F::CPT;                                           // first channel of the workgroup
    const bool has_r1 = d.res1 != nullptr, has_r2 = d.res2 != nullptr, has_fm = d.film != nullptr;
    const float s1e = has_r1 ? d.s1 : 1.f, s2e = has_r2 ? d.s2 : 1.f, fadd = has_fm ? 0.f : 1.f;
    const __amdgpu_buffer_rsrc_t ys = ou_rsrc(d.y + (int64_t)b * d.y_bstride, (int64_t)cout * d.y_cstride * 4);
    const __amdgpu_buffer_rsrc_t r1s =
        ou_rsrc(has_r1 ? d.res1 + (int64_t)b * d.r1_bstride : d.y, has_r1 ? (int64_t)cout * d.r1_cstride * 4 : 0);
    const __amdgpu_buffer_rsrc_t r2s =
        ou_rsrc(has_r2 ? d.res2 + (int64_t)b * d.r2_bstride : d.y, has_r2 ? (int64_t)cout * d.r2_cstride * 4 : 0);
    const __amdgpu_buffer_rsrc_t bs = ou_rsrc(d.bias, d.bias ? (int64_t)cout * 4 : 0);
    const __amdgpu_buffer_rsrc_t fs =
        ou_rsrc(has_fm ? d.film + (int64_t)b * d.film_bstride : d.y, has_fm ? (int64_t)cout * 8 : 0);
    constexpr int NSG = (BNO * R + 3) / 4;        // 4-sample groups per channel
    constexpr int NIT = F::UCH * NSG;             // epilogue items of the workgroup
    constexpr int UEI = (NIT + 255) / 256;        // per thread
    // 16-B residual loads and stores where the tile's first sample and every
    // row start are 16-B aligned (uniform over the workgroup)
    auto al4 = [&](const float* p, int64_t bst, int64_t cst) {
        return !p || (((uintptr_t)p % 16) == 0 && bst % 4 == 0 && cst % 4 == 0);
    };
    const bool v4 = ((u0 * R) & 3) == 0 && al4(d.y, d.y_bstride, d.y_cstride) &&
                    al4(d.res1, d.r1_bstride, d.r1_cstride) && al4(d.res2, d.r2_bstride, d.r2_cstride);
    auto ep_load = [&](int e, float (&r1)[4], float& bias) {   // item tid + 256 e (clamped)
        const int it = min(tid + 256 * e, NIT - 1);
        const int cw = it / NSG, g = it - (it / NSG) * NSG;
        const int co = c0 + cw, sig = 4 * g, t0 = u0 * R + sig;
        const bool cok = co < cout;
        bias = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bs, cok ? co * 4 : kSentinel, 0, 0));
        if (v4 && cok && sig + 3 < BNO * R && t0 + 3 < tend) {
            const auto a1 = __builtin_amdgcn_raw_buffer_load_b128(r1s, (co * (int)d.r1_cstride + t0) * 4, 0, 0);
#pragma unroll
            for (int k = 0; k < 4; ++k) r1[k] = __uint_as_float(a1[k]);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int t = t0 + k;
                const bool ok = cok && sig + k < BNO * R && t < tend;
                r1[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                    r1s, ok ? (co * (int)d.r1_cstride + t) * 4 : kSentinel, 0, 0));
            }
        }
    };
    float pr1[EARLY ? UEI : 1][4], pbias[EARLY ? UEI : 1];
    if constexpr (EARLY) {
#pragma unroll
        for (int e = 0; e < UEI; ++e) ep_load(e, pr1[e], pbias[e]);
    }

#pragma unroll
    for (int j = 0; j < PD; ++j) stage_load(j, xvs[j]);
    load_a(0, 0);
    load_a(0, 1);
    stage_store(0, xvs[0]);
    __syncthreads();
    if constexpr (PD == 1) {
        for (int q = 0; q < nch; ++q) {
            const int cur = q & 1;
            stage_load(q + 1, xvs[0]);
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                mfma_step(cur, s);
                load_a(q + 1, s);
            }
            if (q + 1 < nch) stage_store(cur ^ 1, xvs[0]);
            __syncthreads();
        }
    } else {
        for (int q0 = 0; q0 < nch; q0 += PD) {
#pragma unroll
            for (int j = 0; j < PD; ++j) {
                const int q = q0 + j;
                if (q >= nch) break;
                const int cur = q & 1;
                stage_load(q + PD, xvs[j]);   // clamped
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    mfma_step(cur, s);
                    load_a(q + 1, s);
                }
                if (q + 1 < nch) stage_store(cur ^ 1, xvs[(j + 1) % PD]);
                __syncthreads();
            }
        }
    }
    if constexpr (P != 0) ou_range_flag(d.status, omax, 1, lane);

    // ---- the transposed conv's outputs -> Y [channel of the workgroup][sample]
    // (sample row index n R + ph for B row n, i.e. global sample (fa + n) R + ph)
    float* Y = (float*)lds4;
    const float sx = su * (1.f / 2048.f);
#pragma unroll
    for (int mr = 0; mr < MR; ++mr)
#pragma unroll
        for (int nr = 0; nr < NR; ++nr)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int ml = (r & 3) + 8 * (r >> 2) + 4 * h;   // row within the m-tile
                const int cl = ml / R, ph = ml - (ml / R) * R;
                const float v = P == 1 ? fmaf(accx[mr][nr][r], sx, acc[mr][nr][r] * su) : acc[mr][nr][r] * su;
                if (cl < F::CPT)
                    Y[((wm * MR + mr) * F::CPT + cl) * F::YRS + (wn * 32 * NR + nr * 32 + l32) * R + ph] = v;
            }
    __syncthreads();

    // ---- FIR over 4 consecutive output samples per item, bias, residuals, store
    float tap[F::NT];
    fir_taps<F::NT>(d, tap);
    constexpr int NW = (4 + 2 * R + 3) / 4 * 4;   // window floats read (16-B reads)
#pragma unroll
    for (int e = 0; e < UEI; ++e) {
        const int it = tid + 256 * e;
        if (NIT % 256 != 0 && it >= NIT) break;
        const int cw = it / NSG, g = it - (it / NSG) * NSG;
        const int co = c0 + cw;
        const int sig = 4 * g;            // output sample u0 R + sig <-> Y index sig + R
        const int t0 = u0 * R + sig;
        float w[NW];
        const float* yr = Y + cw * F::YRS + sig;
#pragma unroll
        for (int k = 0; k < NW; k += 4) {
            const float4 q4 = *(const float4*)(yr + k);
            w[k] = q4.x, w[k + 1] = q4.y, w[k + 2] = q4.z, w[k + 3] = q4.w;
        }
        const bool cok = co < cout;
        float r1v[4], bias;
        if constexpr (EARLY) {
            bias = pbias[e];
#pragma unroll
            for (int k = 0; k < 4; ++k) r1v[k] = pr1[e][k];
        } else {
            ep_load(e, r1v, bias);
        }
        const float ga = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(fs, cok ? co * 4 : kSentinel, 0, 0));
        const float gb = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(fs, cok ? (cout + co) * 4 : kSentinel, 0, 0));
        if (v4 && cok && sig + 3 < BNO * R && t0 + 3 < tend) {   // a whole aligned group: 16-B accesses
            const auto a2 = __builtin_amdgcn_raw_buffer_load_b128(r2s, (co * (int)d.r2_cstride + t0) * 4, 0, 0);
            float o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float f = 0.f;
#pragma unroll
                for (int j = 0; j < F::NT; ++j) f = fmaf(tap[j], w[k + j], f);
                float v = f + bias;
                if (t0 + k >= vlen) v = 0.f;
                v = (v + r1v[k]) * s1e;
                v = (ga + fadd) * v + gb;
                o[k] = (v + __uint_as_float(a2[k])) * s2e;
            }
            __builtin_amdgcn_raw_buffer_store_b128(
                ou_u32x4{__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3])}, ys,
                (co * (int)d.y_cstride + t0) * 4, 0, 0);
            continue;
        }
        int off[4];
        float v2[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int t = t0 + k;
            off[k] = (cok && sig + k < BNO * R && t < tend) ? t : -1;
            v2[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                r2s, off[k] >= 0 ? (co * (int)d.r2_cstride + t) * 4 : kSentinel, 0, 0));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float f = 0.f;
#pragma unroll
            for (int j = 0; j < F::NT; ++j) f = fmaf(tap[j], w[k + j], f);
            float v = f + bias;
            if (off[k] >= vlen) v = 0.f;
            v = (v + r1v[k]) * s1e;
            v = (ga + fadd) * v + gb;
            v = (v + v2[k]) * s2e;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ys,
                                                  off[k] >= 0 ? (co * (int)d.y_cstride + off[k]) * 4 : kSentinel, 0, 0);
        }
    }
}

// ---- tile table ------------------------------------------------------------
struct Tile {
    int wm, wn, wk, mr, nr, big;
};
// BM x BN (split-K): 0 32x256, 1 32x128, 2 32x128/K2, 3 64x128, 4 64x128 (MR2),
// 5 128x128, 6 128x64, 7 256x32, 8 128x32/K2, 9 64x32/K4, 10 64x64/K2, 11 64x64,
// 12 32x64/K4; 13.. the same shapes with chunks sized for one workgroup per CU
// (up to 160 KiB of LDS: twice the MFMA work per chunk, for grids <= 256 WGs)
#define OU_TILES(X)                                                                            \
    X(0, 1, 4, 1, 1, 2, 0) X(1, 1, 4, 1, 1, 1, 0) X(2, 1, 2, 2, 1, 2, 0) X(3, 2, 2, 1, 1, 2, 0) \
    X(4, 1, 4, 1, 2, 1, 0) X(5, 2, 2, 1, 2, 2, 0) X(6, 2, 2, 1, 2, 1, 0) X(7, 4, 1, 1, 2, 1, 0) \
    X(8, 2, 1, 2, 2, 1, 0) X(9, 1, 1, 4, 2, 1, 0) X(10, 1, 2, 2, 2, 1, 0) X(11, 2, 2, 1, 1, 1, 0) \
    X(12, 1, 1, 4, 1, 2, 0) X(13, 1, 1, 4, 1, 2, 1) X(14, 1, 1, 4, 2, 1, 1) X(15, 2, 2, 1, 1, 1, 1) \
    X(16, 2, 1, 2, 2, 1, 1) X(17, 1, 2, 2, 2, 1, 1) X(18, 1, 4, 1, 1, 1, 1)
#define OU_TILE_ENTRY(id, wm, wn, wk, mr, nr, big) {wm, wn, wk, mr, nr, big},
constexpr Tile kTiles[] = {OU_TILES(OU_TILE_ENTRY)};
#undef OU_TILE_ENTRY
[[maybe_unused]] constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

constexpr int kMaxLds = 160 * 1024;     // gfx950: 160 KiB per CU
constexpr int kLdsTwoPerCu = 80 * 1024; // fits two workgroups per CU

// channel chunk: the largest of 64/32/16/8 that splits over the K waves and
// whose double-buffered stage fits two workgroups per CU, else one per CU
template <int KT, int WM, int WN, int WK, int MR, int NR, int CC, int P = 0>
constexpr bool chunk_ok(int budget)
{
    return CC / 8 % WK == 0 && (!P || (CC % 16 == 0 && CC / 16 % WK == 0)) &&
           Cfg<KT, CC, WM, WN, WK, MR, NR, P>::LDS2 * 4 <= budget;
}
template <int KT, int WM, int WN, int WK, int MR, int NR, int BIG>
constexpr int chunk_for()
{
    if constexpr (BIG)
        return chunk_ok<KT, WM, WN, WK, MR, NR, 64>(kMaxLds)   ? 64
               : chunk_ok<KT, WM, WN, WK, MR, NR, 32>(kMaxLds) ? 32
                                                               : 16 * (WK > 2 ? 2 : 1);
    return chunk_ok<KT, WM, WN, WK, MR, NR, 64>(kLdsTwoPerCu)   ? 64
           : chunk_ok<KT, WM, WN, WK, MR, NR, 32>(kLdsTwoPerCu) ? 32
           : chunk_ok<KT, WM, WN, WK, MR, NR, 16>(kLdsTwoPerCu) ? 16
           : chunk_ok<KT, WM, WN, WK, MR, NR, 8>(kLdsTwoPerCu)  ? 8
           : chunk_ok<KT, WM, WN, WK, MR, NR, 32>(kMaxLds)      ? 32
           : chunk_ok<KT, WM, WN, WK, MR, NR, 16>(kMaxLds)      ? 16
                                                                : 8 * WK;
}

// split-f16 chunk (8-pair groups per wave, 16-B aligned half rows); 0 when the
// shape has no split-f16 form
template <int KT, int WM, int WN, int WK, int MR, int NR, int BIG>
constexpr int chunk_for_split()
{
    constexpr int b1 = BIG ? kMaxLds : kLdsTwoPerCu;
    return chunk_ok<KT, WM, WN, WK, MR, NR, 64, 1>(b1)        ? 64
           : chunk_ok<KT, WM, WN, WK, MR, NR, 32, 1>(b1)      ? 32
           : chunk_ok<KT, WM, WN, WK, MR, NR, 16, 1>(b1)      ? 16
           : chunk_ok<KT, WM, WN, WK, MR, NR, 64, 1>(kMaxLds) ? 64
           : chunk_ok<KT, WM, WN, WK, MR, NR, 32, 1>(kMaxLds) ? 32
           : chunk_ok<KT, WM, WN, WK, MR, NR, 16, 1>(kMaxLds) ? 16
                                                              : 0;
}
template <int KT, int WM, int WN, int WK, int MR, int NR, int BIG>
constexpr int lds_bytes_split_t()
{
    constexpr int CC = chunk_for_split<KT, WM, WN, WK, MR, NR, BIG>();
    if constexpr (CC == 0) return -1;
    else return Cfg<KT, CC, WM, WN, WK, MR, NR, 1>::LDS2 * 4;
}

template <int KT, int WM, int WN, int WK, int MR, int NR, int BIG>
constexpr int lds_bytes_t()
{
    constexpr int CC = chunk_for<KT, WM, WN, WK, MR, NR, BIG>();
    return Cfg<KT, CC, WM, WN, WK, MR, NR>::LDS2 * 4;
}

template <int KT, int WM, int WN, int WK, int MR, int NR, int BIG, int P = 0>
int launch_t(const ou_conv_desc& d, int tpw, hipStream_t s)
{
    constexpr int CC = P ? chunk_for_split<KT, WM, WN, WK, MR, NR, BIG>() : chunk_for<KT, WM, WN, WK, MR, NR, BIG>();
    if constexpr (CC == 0) {
        (void)tpw;
        (void)s;
        return ou_fail(-2, "conv: tile shape has no split-f16 form (m %d, kt %d)", d.m, d.kt);
    } else {
    using C = Cfg<KT, CC, WM, WN, WK, MR, NR, P>;
    const int mtiles = (d.m + 31) / 32;
    const int cin_eff = d.cin * d.frame;
    const int cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
    const int nchunks = (cin_eff + CC - 1) / CC;
    const int64_t a_mt_stride = (int64_t)cin_pad * KT * 32;
    (void)tpw;   // one output tile per workgroup
    const int S = d.tile >= 0 ? 1 << ((d.tile >> 12) & 3) : 1;   // K slices
    dim3 grid((d.n_frames + C::BN - 1) / C::BN, (mtiles + WM * MR - 1) / (WM * MR), d.batch);
    if (S > 1) {
        const int64_t need = (int64_t)grid.x * grid.y * grid.z * S * C::BM * C::BN * 4;
        if (S > nchunks) return ou_fail(-2, "conv: %d K slices > %d chunks", S, nchunks);
        if (!d.ks_ws || d.ks_ws_bytes < need)
            return ou_fail(-2, "conv: K slices need %lld B of workspace (have %lld)", (long long)need,
                           (long long)d.ks_ws_bytes);
    }
    const int slice_chunks = S > 1 ? (nchunks + S - 1) / S : nchunks;
    const int lds = (slice_chunks > 1 ? C::LDS2 : C::LDS1) * (int)sizeof(float);
    auto kern = conv_kernel<KT, CC, WM, WN, WK, MR, NR, P>;
    static bool attr = false;   // opt in to more than 64 KiB of dynamic LDS, once
    if (!attr && C::LDS2 * 4 > 64 * 1024) {
        OU_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         C::LDS2 * 4),
                     "conv: LDS attribute");
        attr = true;
    }
    if (S == 1) {
        hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, d, nchunks, mtiles, a_mt_stride, 0);
        return ou_check_launch("conv");
    }
    hipLaunchKernelGGL(kern, dim3(grid.x, grid.y, grid.z * S), dim3(256), lds, s, d, nchunks, mtiles, a_mt_stride, 1);
    const int rc = ou_check_launch("conv");
    if (rc) return rc;
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, d, nchunks, mtiles, a_mt_stride, 2);
    return ou_check_launch("conv");
    }
}

// persistent launch: ceil(tiles / tpw) workgroups, each walking tpw tiles
template <int KT, int WM, int WN, int WK, int MR, int NR, int BIG>
int launch_p(const ou_conv_desc& d, int tpw, hipStream_t s)
{
    if constexpr (WK != 1) {
        return ou_fail(-2, "conv: tiles per workgroup > 1 needs a tile without split-K");
    } else {
        constexpr int CC = chunk_for<KT, WM, WN, WK, MR, NR, BIG>();
        using C = Cfg<KT, CC, WM, WN, WK, MR, NR>;
        const int mtiles = (d.m + 31) / 32;
        const int cin_eff = d.cin * d.frame;
        const int cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
        const int nchunks = (cin_eff + CC - 1) / CC;
        const int64_t a_mt_stride = (int64_t)cin_pad * KT * 32;
        const int ntn = (d.n_frames + C::BN - 1) / C::BN;
        const int mgroups = (mtiles + WM * MR - 1) / (WM * MR);
        const int ntiles = ntn * mgroups * d.batch;
        const int lds = 2 * C::STAGE * (int)sizeof(float);
        auto kern = conv_pkernel<KT, CC, WM, WN, MR, NR>;
        static bool attr = false;
        if (!attr && lds > 64 * 1024) {
            OU_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds),
                         "conv: LDS attribute");
            attr = true;
        }
        hipLaunchKernelGGL(kern, dim3((ntiles + tpw - 1) / tpw), dim3(256), lds, s, d, nchunks, mtiles, a_mt_stride,
                           ntn, mgroups, ntiles);
        return ou_check_launch("conv");
    }
}

// warp-specialised kernel: the largest channel chunk whose S-stage ring (+
// split-K area) fits one workgroup per CU
constexpr int kWStages = 3;
template <int KT, int WM, int WN, int WK, int MR, int NR, int CC>
constexpr bool wchunk_ok()
{
    return CC / 8 % WK == 0 && WCfg<KT, CC, WM, WN, WK, MR, NR, kWStages>::LDS * 4 <= kMaxLds;
}
template <int KT, int WM, int WN, int WK, int MR, int NR>
constexpr int wchunk_for()
{
    return wchunk_ok<KT, WM, WN, WK, MR, NR, 64>()   ? 64
           : wchunk_ok<KT, WM, WN, WK, MR, NR, 32>() ? 32
           : wchunk_ok<KT, WM, WN, WK, MR, NR, 16>() ? 16
                                                     : 8 * WK;
}
template <int KT, int WM, int WN, int WK, int MR, int NR>
constexpr int wlds_bytes_t()
{
    return WCfg<KT, wchunk_for<KT, WM, WN, WK, MR, NR>(), WM, WN, WK, MR, NR, kWStages>::LDS * 4;
}

int g_num_cus = 0;   // device CU count, queried once

template <int KT, int WM, int WN, int WK, int MR, int NR>
int launch_w(const ou_conv_desc& d, hipStream_t s)
{
    constexpr int CC = wchunk_for<KT, WM, WN, WK, MR, NR>();
    using C = WCfg<KT, CC, WM, WN, WK, MR, NR, kWStages>;
    constexpr int lds = C::LDS * 4;
    const int mtiles = (d.m + 31) / 32;
    const int cin_eff = d.cin * d.frame;
    const int cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
    const int nchunks = (cin_eff + CC - 1) / CC;
    if (nchunks < 2)   // one accumulator image: two tiles' last chunks must be a tick apart
        return ou_fail(-2, "conv: warp-specialised tile needs >= 2 K chunks (cin_eff %d, chunk %d)", cin_eff, CC);
    const int64_t a_mt_stride = (int64_t)cin_pad * KT * 32;
    const int ntn = (d.n_frames + C::BN - 1) / C::BN;
    const int mgroups = (mtiles + WM * MR - 1) / (WM * MR);
    const int ntiles = ntn * mgroups * d.batch;
    auto kern = conv_wkernel<KT, CC, WM, WN, WK, MR, NR, kWStages>;
    static bool attr = false;
    static int per_cu = 1;
    if (!attr) {
        if (lds > 64 * 1024)
            OU_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds),
                         "conv: LDS attribute");
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, 256 + 64 * kWsLoaders, lds) == hipSuccess && n > 0)
            per_cu = n;
        attr = true;
    }
    if (g_num_cus <= 0) {
        int dev = 0;
        OU_HIP_CHECK(hipGetDevice(&dev), "conv: device");
        OU_HIP_CHECK(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev), "conv: CUs");
        if (g_num_cus <= 0) g_num_cus = 1;
    }
    const int grid = std::min(ntiles, per_cu * g_num_cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256 + 64 * kWsLoaders), lds, s, d, nchunks, mtiles, a_mt_stride, ntn,
                       mgroups, ntiles);
    return ou_check_launch("conv");
}

constexpr int kWsBit = 1 << 10;   // tile bit: warp-specialised persistent kernel
constexpr int kRsBit = 1 << 14;   // tile bit: register-streamed kernel (conv_rkernel)
constexpr int kSplitBit = 1 << 11;   // tile-query bit (LDS size, tile_ok): the split-f16 kernel

template <int KT>
int lds_bytes_kt(int tile)
{
    if (tile & kSplitBit) {
        switch (tile & 0xff) {
#define OU_TILE_CASE(id, wm, wn, wk, mr, nr, big) case id: return lds_bytes_split_t<KT, wm, wn, wk, mr, nr, big>();
            OU_TILES(OU_TILE_CASE)
#undef OU_TILE_CASE
        }
        return -1;
    }
    if (tile & kWsBit) {
        switch (tile & 0xff) {
#define OU_TILE_CASE(id, wm, wn, wk, mr, nr, big) \
    case id: return big ? -1 : wlds_bytes_t<KT, wm, wn, wk, mr, nr>();
            OU_TILES(OU_TILE_CASE)
#undef OU_TILE_CASE
        }
        return -1;
    }
    switch (tile & 0xff) {
#define OU_TILE_CASE(id, wm, wn, wk, mr, nr, big) case id: return lds_bytes_t<KT, wm, wn, wk, mr, nr, big>();
        OU_TILES(OU_TILE_CASE)
#undef OU_TILE_CASE
    }
    return -1;
}


// register-streamed shapes (tile bit 14): id, WM (32-row m-tiles), WK (K parts), NR (32-frame tiles)
#define OU_RTILES(X) X(0, 2, 2, 1) X(1, 2, 2, 2) X(2, 4, 1, 1) X(3, 1, 4, 1) X(4, 4, 1, 2) X(5, 1, 4, 2)
[[maybe_unused]] constexpr int kNumRTiles = 6;

// K chunking of the register-streamed kernel: the whole window (pc = R
// phases x cch = cin channels) when it fits LDS, else chunks of at most half
// the LDS (two workgroups per CU) -- pc phases of every channel, or for R = 1
// cch channels.  Returns false when no chunking fits.
template <int KT, int WM, int WK, int NR, int P>
bool rchunks(int cin, int rf, int* pc, int* cch)
{
    if (rlds_bytes<KT, WM, WK, NR, P>(cin * rf) <= kMaxLds) {
        *pc = rf, *cch = cin;
        return true;
    }
    int best = 0;
    if (rf > 1) {
        for (int q = 1; q < rf; ++q)
            if (rf % q == 0 && (q * cin) % 16 == 0 && rlds_bytes<KT, WM, WK, NR, P>(q * cin) <= kMaxLds / 2)
                best = q;
        *pc = best, *cch = cin;
    } else {
        for (int c = 16; c < cin; c += 16)
            if (cin % c == 0 && rlds_bytes<KT, WM, WK, NR, P>(c) <= kMaxLds / 2) best = c;
        *pc = 1, *cch = best;
    }
    return best > 0;
}

template <int KT, int WM, int WK, int NR, int P>
int launch_r(const ou_conv_desc& d, hipStream_t s)
{
    using R = RCfg<KT, WM, WK, NR>;
    int pc = 0, cch = 0;
    if (!rchunks<KT, WM, WK, NR, P>(d.cin, d.frame, &pc, &cch))
        return ou_fail(-2, "conv: no register-streamed K chunking for cin %d x frame %d", d.cin, d.frame);
    const int S = 1 << ((d.tile >> 12) & 3);   // K slices
    const int nchunks = (d.frame / pc) * (d.cin / cch);
    if (S > nchunks)
        return ou_fail(-2, "conv: %d K slices for %d register-streamed K chunks", S, nchunks);
    const int lds = rlds_bytes<KT, WM, WK, NR, P>(pc * cch);
    auto kern = conv_rkernel<KT, WM, WK, NR, P>;
    static bool attr = false;   // opt in to the full 160 KiB once
    if (!attr) {
        OU_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds),
                     "conv: LDS attribute");
        attr = true;
    }
    const int mtiles = (d.m + 31) / 32;
    const int cin_eff = d.cin * d.frame;
    const int cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
    const int64_t a_mt_stride = (int64_t)cin_pad * KT * 32;
    dim3 grid((d.n_frames + R::BN - 1) / R::BN, (mtiles + WM - 1) / WM, d.batch);
    if (S > 1) {
        const int64_t need = (int64_t)grid.x * grid.y * grid.z * S * WM * NR * 16 * 64 * 4;
        if (!d.ks_ws || d.ks_ws_bytes < need)
            return ou_fail(-2, "conv: K-slice workspace %lld B < %lld B", (long long)d.ks_ws_bytes, (long long)need);
    }
    hipLaunchKernelGGL(kern, dim3(grid.x, grid.y, grid.z * S), dim3(256), lds, s, d, mtiles, a_mt_stride, pc, cch, S);
    if (S > 1) {
        OU_HIP_CHECK(hipGetLastError(), "conv: register-streamed slices");
        hipLaunchKernelGGL((conv_rreduce<NR>), grid, dim3(64 * WM), 0, s, d, S, WM);
    }
    return ou_check_launch("conv");
}

template <int KT>
int launch_rs(const ou_conv_desc& d, int shape, hipStream_t s)
{
    if constexpr (KT == 1 || KT == 3 || KT == 5) {
        switch (shape) {
#define OU_RTILE_CASE(id, wm, wk, nr) \
    case id: return d.prec == 1 ? launch_r<KT, wm, wk, nr, 1>(d, s) : launch_r<KT, wm, wk, nr, 2>(d, s);
            OU_RTILES(OU_RTILE_CASE)
#undef OU_RTILE_CASE
        }
        return ou_fail(-2, "conv: bad register-streamed tile %d", shape);
    } else {
        (void)d, (void)shape, (void)s;
        return ou_fail(-2, "conv: no register-streamed kernel for kt %d", KT);
    }
}

// split-image shapes (tile bit 15): bits 0-7 = NR - 1 (32 NR frames per
// workgroup), + 3: rows prefetched U - 0.5 chunks ahead instead of half a
// chunk (more VGPRs: one wave per SIMD at NR 2 / 3)
constexpr int kSsBit = 1 << 15;
[[maybe_unused]] constexpr int kNumSTiles = 6;

template <int KT, int NR, int DEEP>
int launch_s1(const ou_conv_desc& d, hipStream_t s)
{
    using S = SCfg<KT, NR, DEEP>;
    auto kern = conv_skernel<KT, NR, DEEP>;
    static bool attr = false;
    if (!attr && S::LDS > 64 * 1024) {
        OU_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS),
                     "conv: LDS attribute");
        attr = true;
    }
    const int mtiles = (d.m + 31) / 32;
    const int cin_eff = d.cin * d.frame;
    const int cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
    const int64_t a_mt_stride = (int64_t)cin_pad * KT * 32;
    dim3 grid((d.n_frames + 32 * NR - 1) / (32 * NR), mtiles, d.batch);
    hipLaunchKernelGGL(kern, grid, dim3(256), S::LDS, s, d, mtiles, a_mt_stride);
    return ou_check_launch("conv (split image)");
}

template <int KT>
int launch_ss(const ou_conv_desc& d, int shape, hipStream_t s)
{
    if constexpr (KT == 1 || KT == 3 || KT == 5) {
        switch (shape) {
        case 0: return launch_s1<KT, 1, 0>(d, s);
        case 1: return launch_s1<KT, 2, 0>(d, s);
        case 2: return launch_s1<KT, 3, 0>(d, s);
        case 3: return launch_s1<KT, 1, 1>(d, s);
        case 4: return launch_s1<KT, 2, 1>(d, s);
        case 5: return launch_s1<KT, 3, 1>(d, s);
        }
        return ou_fail(-2, "conv: bad split-image tile %d", shape);
    } else {
        (void)d, (void)shape, (void)s;
        return ou_fail(-2, "conv: no split-image kernel for kt %d", KT);
    }
}

// FIR shapes (tile bit 17): id, WM, WN, MR, NR (BM = 32 WM MR rows, BN = 32 WN NR frames)
#define OU_FTILES(X) \
    X(0, 2, 2, 1, 1) X(1, 4, 1, 1, 2) X(2, 2, 2, 2, 1) X(3, 1, 4, 2, 1) X(4, 2, 2, 1, 2) X(5, 4, 1, 2, 1) \
    X(6, 2, 2, 2, 2) X(7, 4, 1, 1, 1)
[[maybe_unused]] constexpr int kNumFTiles = 8;

template <typename K>
int fir_launch(K kern, int lds, dim3 grid, const ou_conv_desc& d, int mtiles, int64_t a_mt_stride, bool& attr,
               hipStream_t s)
{
    if (!attr && lds > 64 * 1024) {
        OU_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds),
                     "conv: LDS attribute");
        attr = true;
    }
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, d, mtiles, a_mt_stride);
    return ou_check_launch("conv (FIR)");
}

template <int R, int WM, int WN, int MR, int NR>
int launch_f(const ou_conv_desc& d, hipStream_t s)
{
    using F = FCfg<R, WM, WN, MR, NR>;
    static bool attr[4] = {false, false, false, false};   // (direction, precision) opted in to > 64 KiB
    if (d.fir == 1 || d.fir == 3) {   // down / st_conv: K = cin frame in chunks of 16 channels x R phases
        const int mtiles = (d.m + 31) / 32;
        const int64_t a_mt_stride = (int64_t)((d.cin * d.frame + kCinAlign - 1) / kCinAlign * kCinAlign) * 32;
        const dim3 grid((d.n_frames + F::BN - 1) / F::BN, (mtiles + WM * MR - 1) / (WM * MR), d.batch);
        const bool lean = !d.res1 && !d.res2 && !d.film;   // bias (+ split image) only: the lean epilogue
        if constexpr (R == 4 || R == 8) {
            static bool sattr[4] = {false, false, false, false};
            if (d.fir == 3 && lean)
                return d.prec == 1 ? fir_launch(conv_fdkernel<R, WM, WN, MR, NR, 1, 1, 1>, F::DLDS, grid, d, mtiles,
                                                a_mt_stride, sattr[0], s)
                                   : fir_launch(conv_fdkernel<R, WM, WN, MR, NR, 2, 1, 1>, F::DLDS, grid, d, mtiles,
                                                a_mt_stride, sattr[1], s);
            if (d.fir == 3)   // the st_convs' running sum: residuals in the epilogue
                return d.prec == 1 ? fir_launch(conv_fdkernel<R, WM, WN, MR, NR, 1, 1, 0>, F::DLDS, grid, d, mtiles,
                                                a_mt_stride, sattr[2], s)
                                   : fir_launch(conv_fdkernel<R, WM, WN, MR, NR, 2, 1, 0>, F::DLDS, grid, d, mtiles,
                                                a_mt_stride, sattr[3], s);
        }
        if (d.fir == 3) return ou_fail(-2, "conv: FIR mode 3 needs rate 4 or 8 chunks");
        static bool lattr[4] = {false, false, false, false};
        if (lean && (d.tile & kFirDeep))
            return d.prec == 1 ? fir_launch(conv_fdkernel<R, WM, WN, MR, NR, 1, 0, 1, 2>, F::DLDS, grid, d, mtiles,
                                            a_mt_stride, lattr[2], s)
                               : fir_launch(conv_fdkernel<R, WM, WN, MR, NR, 2, 0, 1, 2>, F::DLDS, grid, d, mtiles,
                                            a_mt_stride, lattr[3], s);
        if (d.tile & kFirDeep) return ou_fail(-2, "conv: FIR tile bit 9 needs a down conv without residuals / FiLM");
        if (lean)
            return d.prec == 1
                       ? fir_launch(conv_fdkernel<R, WM, WN, MR, NR, 1, 0, 1>, F::DLDS, grid, d, mtiles, a_mt_stride, lattr[0], s)
                       : fir_launch(conv_fdkernel<R, WM, WN, MR, NR, 2, 0, 1>, F::DLDS, grid, d, mtiles, a_mt_stride, lattr[1], s);
        return d.prec == 1
                   ? fir_launch(conv_fdkernel<R, WM, WN, MR, NR, 1>, F::DLDS, grid, d, mtiles, a_mt_stride, attr[0], s)
                   : fir_launch(conv_fdkernel<R, WM, WN, MR, NR, 2>, F::DLDS, grid, d, mtiles, a_mt_stride, attr[1], s);
    }
    // up: K = cin in chunks of 32; P = 32 / R whole channels per packed m-tile
    const int mtiles = (d.m / R + F::CPT - 1) / F::CPT;
    const int64_t a_mt_stride = (int64_t)((d.cin + kCinAlign - 1) / kCinAlign * kCinAlign) * 32;
    const dim3 grid((d.n_frames + F::BN - 3) / (F::BN - 2), (mtiles + WM * MR - 1) / (WM * MR), d.batch);
    if (d.tile & kFirDeep) {
        if (d.tile & kFirEarly) return ou_fail(-2, "conv: FIR tile bits 8 and 9 together");
        static bool pattr[2] = {false, false};
        return d.prec == 1
                   ? fir_launch(conv_fukernel<R, WM, WN, MR, NR, 1, 0, 2>, F::ULDS, grid, d, mtiles, a_mt_stride, pattr[0], s)
                   : fir_launch(conv_fukernel<R, WM, WN, MR, NR, 2, 0, 2>, F::ULDS, grid, d, mtiles, a_mt_stride, pattr[1], s);
    }
    if (d.tile & kFirEarly) {
        static bool eattr[2] = {false, false};
        return d.prec == 1
                   ? fir_launch(conv_fukernel<R, WM, WN, MR, NR, 1, 1>, F::ULDS, grid, d, mtiles, a_mt_stride, eattr[0], s)
                   : fir_launch(conv_fukernel<R, WM, WN, MR, NR, 2, 1>, F::ULDS, grid, d, mtiles, a_mt_stride, eattr[1], s);
    }
    return d.prec == 1
               ? fir_launch(conv_fukernel<R, WM, WN, MR, NR, 1>, F::ULDS, grid, d, mtiles, a_mt_stride, attr[2], s)
               : fir_launch(conv_fukernel<R, WM, WN, MR, NR, 2>, F::ULDS, grid, d, mtiles, a_mt_stride, attr[3], s);
}

template <int R>
int launch_fr(const ou_conv_desc& d, int shape, hipStream_t s)
{
    switch (shape) {
#define OU_FTILE_CASE(id, wm, wn, mr, nr) case id: return launch_f<R, wm, wn, mr, nr>(d, s);
        OU_FTILES(OU_FTILE_CASE)
#undef OU_FTILE_CASE
    }
    return ou_fail(-2, "conv: bad FIR tile %d", shape);
}

template <int KT>
int launch_kt(const ou_conv_desc& d, int tile, int tpw, bool ws, hipStream_t s)
{
    if (tile & kSsBit) return launch_ss<KT>(d, tile & 0xff, s);
    if (tile & kRsBit) return launch_rs<KT>(d, tile & 0xff, s);
    if (d.prec == 1) {   // split-f16: one-tile workgroups (checked by ou_conv)
        switch (tile) {
#define OU_TILE_CASE(id, wm, wn, wk, mr, nr, big) case id: return launch_t<KT, wm, wn, wk, mr, nr, big, 1>(d, 1, s);
            OU_TILES(OU_TILE_CASE)
#undef OU_TILE_CASE
        }
        return ou_fail(-2, "conv: bad tile %d", tile);
    }
    if (d.prec == 2) {   // plain f16 (same layout and tiles as split-f16)
        switch (tile) {
#define OU_TILE_CASE(id, wm, wn, wk, mr, nr, big) case id: return launch_t<KT, wm, wn, wk, mr, nr, big, 2>(d, 1, s);
            OU_TILES(OU_TILE_CASE)
#undef OU_TILE_CASE
        }
        return ou_fail(-2, "conv: bad tile %d", tile);
    }
    if (ws) {
        switch (tile) {
#define OU_TILE_CASE(id, wm, wn, wk, mr, nr, big) \
    case id:                                      \
        if constexpr (!big) return launch_w<KT, wm, wn, wk, mr, nr>(d, s); \
        else return ou_fail(-2, "conv: tile %d has no warp-specialised form", tile);
            OU_TILES(OU_TILE_CASE)
#undef OU_TILE_CASE
        }
        return ou_fail(-2, "conv: bad warp-specialised tile %d", tile);
    }
    switch (tile) {
#define OU_TILE_CASE(id, wm, wn, wk, mr, nr, big)                                              \
    case id:                                                                                   \
        return tpw > 1 ? launch_p<KT, wm, wn, wk, mr, nr, big>(d, tpw, s)                     \
                       : launch_t<KT, wm, wn, wk, mr, nr, big>(d, tpw, s);
        OU_TILES(OU_TILE_CASE)
#undef OU_TILE_CASE
    }
    return ou_fail(-2, "conv: bad tile %d", tile);
}

// Static choice (used when the host has not autotuned the layer): the
// largest tile that still gives >= 1 workgroup per CU, split-K when N is short.
int pick_tile(const ou_conv_desc& d)
{
    auto wgs = [&](int t) {
        const Tile& k = kTiles[t];
        const int bm = 32 * k.wm * k.mr, bn = 32 * k.nr * k.wn;
        return (int64_t)((d.m + bm - 1) / bm) * ((d.n_frames + bn - 1) / bn) * d.batch;
    };
    if (d.m <= 32) {
        for (int t : {0, 1}) if (wgs(t) >= 256) return t;
        return 12;
    }
    if (d.m <= 64) {
        for (int t : {3, 11}) if (wgs(t) >= 256) return t;
        return 9;
    }
    for (int t : {5, 6}) if (wgs(t) >= 256) return t;
    if (wgs(10) >= 256) return 10;
    return 9;
}

}  // namespace

// ---- translation-unit split (build speed) -----------------------------------
// The build compiles this file once per tap count with -DOU_CONV_SPLIT_KT=K
// (kernels and launchers for that K only, exported as ou_conv_launch_ktK /
// ou_conv_lds_ktK) and once with -DOU_CONV_SPLIT_MAIN (the C ABI below, no
// kernels).  Without either macro (tests/emu) everything is one unit.
#define OU_CAT2(a, b) a##b
#define OU_CAT(a, b) OU_CAT2(a, b)
#if defined(OU_CONV_SPLIT_KT)
int OU_CAT(ou_conv_launch_kt, OU_CONV_SPLIT_KT)(const ou_conv_desc& d, int tile, int tpw, bool ws, hipStream_t s)
{
    return launch_kt<OU_CONV_SPLIT_KT>(d, tile, tpw, ws, s);
}
int OU_CAT(ou_conv_lds_kt, OU_CONV_SPLIT_KT)(int tile) { return lds_bytes_kt<OU_CONV_SPLIT_KT>(tile); }
#elif defined(OU_CONV_SPLIT_FIR)   // the FIR kernels of one rate R (-DOU_CONV_SPLIT_FIR=R)
int OU_CAT(ou_conv_launch_fir, OU_CONV_SPLIT_FIR)(const ou_conv_desc& d, int shape, hipStream_t s)
{
    return launch_fr<OU_CONV_SPLIT_FIR>(d, shape, s);
}
#elif defined(OU_CONV_SPLIT_MAIN)
#define OU_KT_DECL(K)                                                                           \
    int ou_conv_launch_kt##K(const ou_conv_desc& d, int tile, int tpw, bool ws, hipStream_t s); \
    int ou_conv_lds_kt##K(int tile);
OU_KT_DECL(1) OU_KT_DECL(3) OU_KT_DECL(4) OU_KT_DECL(5)
#undef OU_KT_DECL
#define OU_FIR_DECL(R) int ou_conv_launch_fir##R(const ou_conv_desc& d, int shape, hipStream_t s);
OU_FIR_DECL(2) OU_FIR_DECL(3) OU_FIR_DECL(4) OU_FIR_DECL(5) OU_FIR_DECL(8)
#undef OU_FIR_DECL
#define OU_LAUNCH_KT(K, ...) ou_conv_launch_kt##K(__VA_ARGS__)
#define OU_LDS_KT(K, tile) ou_conv_lds_kt##K(tile)
#define OU_LAUNCH_FIR(R, ...) ou_conv_launch_fir##R(__VA_ARGS__)
#else
#define OU_LAUNCH_KT(K, ...) launch_kt<K>(__VA_ARGS__)
#define OU_LDS_KT(K, tile) lds_bytes_kt<K>(tile)
#define OU_LAUNCH_FIR(R, ...) launch_fr<R>(__VA_ARGS__)
#endif

#if !defined(OU_CONV_SPLIT_KT) && !defined(OU_CONV_SPLIT_FIR)
namespace {
int lds_bytes(int kt, int tile)
{
    switch (kt) {
    case 1: return OU_LDS_KT(1, tile);
    case 3: return OU_LDS_KT(3, tile);
    case 4: return OU_LDS_KT(4, tile);
    case 5: return OU_LDS_KT(5, tile);
    }
    return -1;
}

// static choice for a precision: the split-f16 form lacks some shapes (LDS)
int pick_tile_for(const ou_conv_desc& d)
{
    const int t = pick_tile(d);
    if (d.prec == 0 || lds_bytes(d.kt, t | kSplitBit) > 0) return t;
    for (int c : {11, 3, 6, 5, 1, 0, 10, 8, 2, 4, 7, 12})
        if (lds_bytes(d.kt, c | kSplitBit) > 0) return c;
    return t;
}
}  // namespace

extern "C" int ou_conv_chunk(int kt, int frame)
{
    (void)frame;
    return kt == 1 ? 32 : 16;
}

extern "C" int64_t ou_conv_packed_size(int m, int cin_eff, int kt, int cc)
{
    (void)cc;
    const int64_t mtiles = (m + 31) / 32;
    const int64_t cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
    return mtiles * (cin_pad / 2) * kt * 64;
}

// Packed order: [m-tile][p / 4][tap k][lane][p % 4] over channel pairs p;
// lane -> row mt*32 + (lane & 31), channel 2 p + (lane >> 5); zero outside
// [0, m) x [0, cin_eff).  A K chunk of CC channels is then one contiguous run
// per m-tile, and one float4 per lane holds 4 consecutive k-steps.
extern "C" int ou_conv_pack(const float* w, int m, int cin_eff, int kt, int cc, float* out)
{
    (void)cc;
    if (!w || !out || m <= 0 || cin_eff <= 0 || kt <= 0)
        return ou_fail(-1, "conv_pack: bad arguments");
    const int mtiles = (m + 31) / 32;
    const int cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
    int64_t o = 0;
    for (int mt = 0; mt < mtiles; ++mt)
        for (int pq = 0; pq < cin_pad / 8; ++pq)
            for (int k = 0; k < kt; ++k)
                for (int lane = 0; lane < 64; ++lane)
                    for (int j = 0; j < 4; ++j) {
                        const int row = mt * 32 + (lane & 31);
                        const int c = 2 * (4 * pq + j) + (lane >> 5);
                        out[o++] = (row < m && c < cin_eff) ? w[((int64_t)row * cin_eff + c) * kt + k] : 0.f;
                    }
    return 0;
}

// Split-f16 packing (include/ouhip.h): [m-tile][8-pair group][hi | lo][tap]
// [lane][8 halves] of a = w * 2^e; the same byte count per K chunk as the f32
// packing, so the kernel's chunk addressing is unchanged.
extern "C" int ou_conv_pack_split(const float* w, int m, int cin_eff, int kt, float* out, float* w_unscale)
{
    if (!w || !out || !w_unscale || m <= 0 || cin_eff <= 0 || kt <= 0)
        return ou_fail(-1, "conv_pack_split: bad arguments");
    const int64_t n = (int64_t)m * cin_eff * kt;
    float mx = 0.f;
    for (int64_t i = 0; i < n; ++i) {
        if (!std::isfinite(w[i])) return ou_fail(-1, "conv_pack_split: non-finite weight at %lld", (long long)i);
        mx = std::max(mx, std::fabs(w[i]));
    }
    int e = 0;
    if (mx > 0.f) {
        int ex = 0;
        std::frexp(mx, &ex);                  // mx in [2^(ex-1), 2^ex)
        e = std::min(100, std::max(-100, 10 - ex));   // max|a| in [2^9, 2^10)
    }
    const float sc = std::ldexp(1.f, e);
    const int mtiles = (m + 31) / 32;
    const int cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
    _Float16* o = (_Float16*)out;
    for (int mt = 0; mt < mtiles; ++mt)
        for (int g = 0; g < cin_pad / 16; ++g)
            for (int part = 0; part < 2; ++part)
                for (int k = 0; k < kt; ++k)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int j = 0; j < 8; ++j) {
                            const int row = mt * 32 + (lane & 31);
                            const int c = 2 * (8 * g + j) + (lane >> 5);
                            const float a =
                                (row < m && c < cin_eff) ? w[((int64_t)row * cin_eff + c) * kt + k] * sc : 0.f;
                            const _Float16 hi = (_Float16)a;
                            *o++ = part == 0 ? hi : (_Float16)((a - (float)hi) * 2048.f);
                        }
    *w_unscale = std::ldexp(1.f, kSplitShift - e);
    return 0;
}

// Natural-order split packing (include/ouhip.h): as ou_conv_pack_split with
// lane l holding channel 16 g + 8 (l >> 5) + j of row l & 31 in half j.
extern "C" int ou_conv_pack_split_nat(const float* w, int m, int cin_eff, int kt, float* out, float* w_unscale)
{
    if (!w || !out || !w_unscale || m <= 0 || cin_eff <= 0 || kt <= 0)
        return ou_fail(-1, "conv_pack_split_nat: bad arguments");
    const int64_t n = (int64_t)m * cin_eff * kt;
    float mx = 0.f;
    for (int64_t i = 0; i < n; ++i) {
        if (!std::isfinite(w[i])) return ou_fail(-1, "conv_pack_split_nat: non-finite weight at %lld", (long long)i);
        mx = std::max(mx, std::fabs(w[i]));
    }
    int e = 0;
    if (mx > 0.f) {
        int ex = 0;
        std::frexp(mx, &ex);
        e = std::min(100, std::max(-100, 10 - ex));
    }
    const float sc = std::ldexp(1.f, e);
    const int mtiles = (m + 31) / 32;
    const int cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
    _Float16* o = (_Float16*)out;
    for (int mt = 0; mt < mtiles; ++mt)
        for (int g = 0; g < cin_pad / 16; ++g)
            for (int part = 0; part < 2; ++part)
                for (int k = 0; k < kt; ++k)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int j = 0; j < 8; ++j) {
                            const int row = mt * 32 + (lane & 31);
                            const int c = 16 * g + 8 * (lane >> 5) + j;
                            const float a =
                                (row < m && c < cin_eff) ? w[((int64_t)row * cin_eff + c) * kt + k] * sc : 0.f;
                            const _Float16 hi = (_Float16)a;
                            *o++ = part == 0 ? hi : (_Float16)((a - (float)hi) * 2048.f);
                        }
    *w_unscale = std::ldexp(1.f, kSplitShift - e);
    return 0;
}

extern "C" int ou_conv(const ou_conv_desc* dp, void* stream)
{
    if (!dp) return ou_fail(-1, "conv: null descriptor");
    const ou_conv_desc& d = *dp;
    if (!d.x || !d.w || !d.y || d.m <= 0 || d.batch <= 0 || d.n_frames <= 0 || d.cin <= 0 ||
        d.frame <= 0 || d.rout == 0 || d.m % d.rout != 0 || d.in_len <= 0 || d.out_len <= 0 || d.f0 < 0)
        return ou_fail(-1, "conv: invalid descriptor (m=%d rout=%d frame=%d f0=%d)", d.m, d.rout, d.frame, d.f0);
    {   // buffer resources take 32-bit offsets with a sentinel for "outside":
        // every per-item tensor must stay below it
        const int64_t lim = kSentinel, cout = d.m / (d.rout < 0 ? -d.rout : d.rout);
        if ((int64_t)d.cin * d.x_cstride * 4 >= lim || cout * d.y_cstride * 4 >= lim ||
            (d.res1 && cout * d.r1_cstride * 4 >= lim) || (d.res2 && cout * d.r2_cstride * 4 >= lim))
            return ou_fail(-1, "conv: a per-item tensor (cin %d x %lld, cout %lld x %lld floats) exceeds the 32-bit "
                               "buffer range", d.cin, (long long)d.x_cstride, (long long)cout,
                           (long long)d.y_cstride);
    }
    if (d.sy) {   // split-image output (any split-f16 kernel's epilogue)
        if (d.prec != 1 || d.rout != 1 || d.m % 32 || d.sy_rows < d.out_len || d.sy_shift < -100 ||
            d.sy_shift > 100 || (int64_t)(d.m / 32) * d.sy_rows * 128 >= kSentinel)
            return ou_fail(-1, "conv: split-image output needs prec 1, rout 1, m %% 32 == 0, sy_rows >= out_len "
                               "(m %d rout %d rows %d out_len %d)", d.m, d.rout, d.sy_rows, d.out_len);
    }
    if (d.fir || (d.tile >= 0 && (d.tile & kFirBit))) {   // FIR applied (bits 0-7: OU_FTILES shape)
        // fir 3 (st_convs, no FIR): chunks of R = 8 (or 4) of the frame's phases
        const int R = d.fir == 1 ? d.frame : d.fir == 3 ? (d.frame % 8 == 0 ? 8 : 4) : (d.rout < 0 ? -d.rout : d.rout);
        if (d.fir < 1 || d.fir > 3 || (d.fir != 3 && !d.fir_taps) || (d.prec != 1 && d.prec != 2) || d.kt != 1 ||
            d.pad || d.shift || d.in_scale || d.xs || (d.fir != 2 && (d.rout != 1 || d.cin % 16)) ||
            (d.fir == 2 && (d.frame != 1 || d.cin % 32)) || (d.fir == 3 && (d.frame < 4 || d.frame % 4)) ||
            (R != 2 && R != 3 && R != 4 && R != 5 && R != 8))
            return ou_fail(-1, "conv: FIR mode %d needs prec 1/2, kt 1, pad 0, shift 0, no in_scale / xs, rate 2/3/4/5/8 "
                               "(mode 3: a multiple of 4), cin %% 16 (down) / 32 (up) == 0 (cin %d frame %d rout %d kt %d)",
                           d.fir, d.cin, d.frame, d.rout, d.kt);
        if (!(d.w_unscale > 0.f)) return ou_fail(-1, "conv: FIR mode needs the w_unscale of ou_conv_pack_split_nat");
        const int tile = d.tile >= 0 ? d.tile : (kFirBit | 2);
        if (!(tile & kFirBit) || (tile & ~(kFirBit | kMajBit | kFirEarly | kFirDeep | 0xff)) || (tile & 0xff) >= kNumFTiles)
            return ou_fail(-2, "conv: FIR mode needs a FIR tile (tile 0x%x)", d.tile);
        ou_conv_desc dd = d;   // the kernels read their order bit from the tile
        dd.tile = tile;
        hipStream_t fs = (hipStream_t)stream;
        switch (R) {
        case 2: return OU_LAUNCH_FIR(2, dd, tile & 0xff, fs);
        case 3: return OU_LAUNCH_FIR(3, dd, tile & 0xff, fs);
        case 4: return OU_LAUNCH_FIR(4, dd, tile & 0xff, fs);
        case 5: return OU_LAUNCH_FIR(5, dd, tile & 0xff, fs);
        case 8: return OU_LAUNCH_FIR(8, dd, tile & 0xff, fs);
        }
        return ou_fail(-2, "conv: no FIR kernel for rate %d", R);
    }
    if (d.xs || (d.tile >= 0 && (d.tile & kSsBit))) {   // split-image input (bits 0-7: NR - 1)
        // static choice: 64-frame workgroups while they still give one per CU
        const int tile = d.tile >= 0 ? d.tile
                         : kSsBit | ((int64_t)(d.n_frames + 63) / 64 * ((d.m + 31) / 32) * d.batch >= 256 ? 1 : 0);
        if (!d.xs || !(tile & kSsBit) || (tile & ~(kSsBit | kMajBit | 0xff)) || (tile & 0xff) >= kNumSTiles)
            return ou_fail(-2, "conv: a split-image input needs a split-image tile (tile 0x%x)", d.tile);
        if (d.prec != 1 || d.cin % 32 || d.xs_rows < d.in_len || d.xs_shift < -100 ||
            d.xs_shift > 100 || (int64_t)(d.cin / 32) * d.xs_rows * 128 >= kSentinel)
            return ou_fail(-2, "conv: the split-image kernel needs prec 1, cin %% 32 == 0, xs_rows >= in_len, "
                               "(cin %d rows %d in_len %d)", d.cin, d.xs_rows, d.in_len);
        if (!(d.w_unscale > 0.f)) return ou_fail(-1, "conv: split-f16 needs the w_unscale of ou_conv_pack_split_nat");
        hipStream_t ss = (hipStream_t)stream;
        ou_conv_desc dd = d;   // the kernel reads its order bit from the tile
        dd.tile = tile;
        switch (d.kt) {
        case 1: return OU_LAUNCH_KT(1, dd, tile, 1, false, ss);
        case 3: return OU_LAUNCH_KT(3, dd, tile, 1, false, ss);
        case 5: return OU_LAUNCH_KT(5, dd, tile, 1, false, ss);
        }
        return ou_fail(-2, "conv: no split-image kernel for kt %d", d.kt);
    }
    if (d.tile >= 0 && (d.tile & kRsBit)) {   // register-streamed kernel (bits 0-7: RTILES shape)
        if ((d.tile & ~(kRsBit | kMajBit | 0x3ff | (3 << 12))) || (d.tile & 0xff) >= kNumRTiles)
            return ou_fail(-2, "conv: bad register-streamed tile 0x%x", d.tile);
        if ((d.prec != 1 && d.prec != 2) || d.cin % 16)
            return ou_fail(-2, "conv: the register-streamed kernel needs prec 1/2, cin %% 16 == 0");
        if (!(d.w_unscale > 0.f)) return ou_fail(-1, "conv: split-f16 needs the w_unscale of ou_conv_pack_split");
        hipStream_t rs = (hipStream_t)stream;
        const int t = d.tile & (0xff | kRsBit);   // bits 8-9 (diagnostics), 12-13 (K slices), 16 travel in d.tile
        switch (d.kt) {
        case 1: return OU_LAUNCH_KT(1, d, t, 1, false, rs);
        case 3: return OU_LAUNCH_KT(3, d, t, 1, false, rs);
        case 5: return OU_LAUNCH_KT(5, d, t, 1, false, rs);
        }
        return ou_fail(-2, "conv: no register-streamed kernel for kt %d", d.kt);
    }
    // d.tile: bits 0-7 tile shape (kTiles), bits 8-9 log2(output tiles per
    // workgroup: > 1 selects the persistent kernel, shapes without split-K),
    // bit 10 the warp-specialised persistent kernel (shapes 0-12)
    const int tile = d.tile >= 0 && (d.tile & 0xff) < kNumTiles ? (d.tile & 0xff) : pick_tile_for(d);
    const bool ws = d.tile >= 0 && (d.tile & kWsBit);
    const int tpw = d.tile >= 0 && !ws ? 1 << ((d.tile >> 8) & 3) : 1;
    const int kslices = d.tile >= 0 ? 1 << ((d.tile >> 12) & 3) : 1;
    if (kslices > 1 && (ws || tpw > 1))
        return ou_fail(-2, "conv: K slices need the one-tile kernel (tile 0x%x)", d.tile);
    if (d.tile >= 0 && (d.tile & kMajBit) && (ws || tpw > 1))
        return ou_fail(-2, "conv: the m-major order needs the one-tile kernel (tile 0x%x)", d.tile);
    if (ws && d.rout != 1) return ou_fail(-2, "conv: the warp-specialised kernel has no transposed (rout %d) form", d.rout);
    if (d.prec < 0 || d.prec > 2) return ou_fail(-1, "conv: bad precision %d", d.prec);
    if (d.prec != 0 && (ws || tpw > 1))
        return ou_fail(-2, "conv: the split-f16 form has one-tile workgroups only (tile 0x%x)", d.tile);
    if (d.f0 != 0 && (ws || tpw > 1))
        return ou_fail(-2, "conv: a frame offset (f0 %d) needs the one-tile kernel (tile 0x%x)", d.f0, d.tile);
    if (d.prec != 0 && !(d.w_unscale > 0.f))
        return ou_fail(-1, "conv: split-f16 needs the w_unscale of ou_conv_pack_split");
    const int lb = lds_bytes(d.kt, tile | (ws ? kWsBit : 0) | (d.prec != 0 ? kSplitBit : 0));
    if (lb <= 0 || lb > kMaxLds)
        return ou_fail(-2, "conv: tile %d (ws %d) needs %d B of LDS for kt=%d", tile, (int)ws, lb, d.kt);
    hipStream_t s = (hipStream_t)stream;
    switch (d.kt) {
    case 1: return OU_LAUNCH_KT(1, d, tile, tpw, ws, s);
    case 3: return OU_LAUNCH_KT(3, d, tile, tpw, ws, s);
    case 4: return OU_LAUNCH_KT(4, d, tile, tpw, ws, s);
    case 5: return OU_LAUNCH_KT(5, d, tile, tpw, ws, s);
    }
    return ou_fail(-1, "conv: unsupported kt %d", d.kt);
}

#ifdef OU_CONV_STAMPS
extern "C" int ou_conv_read_stamps(uint64_t* host, int n)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_conv_stamps), sizeof(uint64_t) * (size_t)n) == hipSuccess ? 0 : -1;
}
#endif

// LDS bytes a tile shape requests at a tap count, and the device's opt-in
// per-workgroup LDS limit (diagnostics: tools/conv_bench.py --info)
extern "C" int ou_conv_lds_info(int kt, int tile, int* lds_request, int* device_optin_max)
{
    if (lds_request) *lds_request = lds_bytes(kt, tile & (0xff | kWsBit | kSplitBit));
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess) return -1;
    if (device_optin_max) *device_optin_max = v;
    return 0;
}

extern "C" int ou_conv_pick_tile(const ou_conv_desc* d) { return d ? pick_tile_for(*d) : -1; }
extern "C" int ou_conv_num_tiles(void) { return kNumTiles; }
extern "C" int ou_conv_tile_ok(int kt, int tile)
{
    if (tile & kFirBit)   // FIR applied (ou_conv_desc.fir): shape (+ m-major order); one tap
        return !(tile & ~(kFirBit | kMajBit | kFirEarly | kFirDeep | 0xff)) && (tile & 0xff) < kNumFTiles && kt == 1;
    if (tile & kSsBit)   // split-image input: shape = NR - 1 (+ m-major order)
        return !(tile & ~(kSsBit | kMajBit | 0xff)) && (tile & 0xff) < kNumSTiles && (kt == 1 || kt == 3 || kt == 5);
    if (tile & kRsBit)   // register-streamed: shape id (+ K slices, m-major order); LDS and chunks checked at launch
        return !(tile & ~(kRsBit | kMajBit | 0xff | (3 << 12))) && (tile & 0xff) < kNumRTiles &&
               (kt == 1 || kt == 3 || kt == 5);
    if ((tile & kMajBit) && (tile & (kWsBit | (3 << 8)))) return 0;   // one-tile kernels only
    tile &= ~kMajBit;
    if (tile & kSplitBit) {   // split-f16 (d.prec = 1): one-tile workgroups, no other bits
        if (tile & ~(kSplitBit | 0xff)) return 0;
        if ((tile & 0xff) >= kNumTiles) return 0;
        const int lb = lds_bytes(kt, tile);
        return lb > 0 && lb <= kMaxLds;
    }
    if (tile & kWsBit) {   // warp-specialised: shapes without the 'big' chunking, no tpw bits
        if (tile & ~(kWsBit | 0xff)) return 0;
        const int t = tile & 0xff;
        if (t >= kNumTiles || kTiles[t].big) return 0;
        const int lb = lds_bytes(kt, tile);
        return lb > 0 && lb <= kMaxLds;
    }
    if ((tile >> 8) & 3) {   // persistent: shapes without split-K only
        const int t = tile & 0xff;
        if (t >= kNumTiles || kTiles[t].wk != 1) return 0;
    }
    tile &= 0xff;
    return tile >= 0 && tile < kNumTiles && lds_bytes(kt, tile) > 0 && lds_bytes(kt, tile) <= kMaxLds;
}
#endif  // !OU_CONV_SPLIT_KT
