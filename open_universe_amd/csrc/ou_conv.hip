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
#include <cstdio>
#include <cstring>

#include "../../include/ouhip.h"
#include "ou_common.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int kCinAlign = 64;   // packed weights pad the channel axis to this

template <int KT, int CC, int WM, int WN, int WK, int NR>
struct Cfg {
    static constexpr int BM = 32 * WM;
    static constexpr int BN = 32 * NR * WN;
    static constexpr int W = BN + KT - 1;           // staged frames per chunk
    static constexpr int WS = W | 1;                 // odd LDS row stride
    static constexpr int HALF = CC / 2;              // channel pairs per chunk
    static constexpr int S = HALF * KT;              // k-steps per chunk
    static constexpr int HPW = HALF / WK;            // channel pairs per wave
    static constexpr int XN = CC * W;                // staged input floats
    static constexpr int XE = (XN + 255) / 256;      // per thread
    static constexpr int AN = WM * S * 64;           // staged weight floats
    static constexpr int AE4 = (AN / 4 + 255) / 256; // float4 per thread
    static constexpr int XBUF = (CC * WS + 3) / 4 * 4;
    static constexpr int ABUF = AE4 * 1024;          // padded: every thread stores AE4 float4
    static constexpr int STAGE = XBUF + ABUF;
    static constexpr int RED = (WK - 1) * WM * WN * NR * 16 * 64;
    static constexpr int LDS = (2 * STAGE > RED ? 2 * STAGE : RED);
    static_assert(HALF % WK == 0, "channel pairs must split evenly over WK");
    static_assert(WM * WN * WK == 4, "4 waves per workgroup");
};

constexpr int kSentinel = 0x7ffffff0;   // byte offset past any buffer: loads return 0

template <int KT, int CC, int WM, int WN, int WK, int NR>
__global__ __launch_bounds__(256) void conv_kernel(ou_conv_desc d, int nchunks, int mtiles,
                                                   int64_t a_mt_stride)
{
    using C = Cfg<KT, CC, WM, WN, WK, NR>;
    extern __shared__ __attribute__((aligned(16))) float lds[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wn = wave % WN;
    const int wm = (wave / WN) % WM;
    const int wk = wave / (WN * WM);
    const int b = blockIdx.z;
    const int n0 = blockIdx.x * C::BN;
    const int mt0 = blockIdx.y * WM;           // first m-tile of the workgroup
    const int mt = mt0 + wm;
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int R = d.frame;
    const int cin = d.cin;
    const int in_len = d.in_len;
    const int xc = (int)d.x_cstride;
    const float* xb = d.x + (int64_t)b * d.x_bstride;
    const float scale = d.in_scale ? d.in_scale[b] : 1.0f;
    const float slope = d.slope;
    const int t0 = n0 - d.pad;

    // ---- per-element staging geometry, fixed for the whole K loop -------
    // R == 1: element (c, w) reads x[q*CC + c][t0 + w + shift]; the chunk
    // advances the buffer base by CC channels and shrinks its size, so the
    // channel bound is the buffer's range check.  R > 1 (frame view): element
    // (w, c) reads channel c' = q*CC + c -> (c'/R, c'%R), recomputed per chunk.
    int xoff[C::XE];
    int loff[C::XE];
#pragma unroll
    for (int e = 0; e < C::XE; ++e) {
        const int idx = tid + e * 256;
        int c, w;
        if (R == 1) {
            c = idx / C::W;
            w = idx - c * C::W;
        } else {
            w = idx / CC;
            c = idx - w * CC;
        }
        loff[e] = idx < C::XN ? c * C::WS + w : -1;
        if (R == 1) {
            const int pos = t0 + w + d.shift;
            xoff[e] = (idx < C::XN && pos >= 0 && pos < in_len) ? (c * xc + pos) * 4 : kSentinel;
        } else {
            xoff[e] = (t0 + w) * R + d.shift;   // sample index of phase 0 of frame w
        }
    }
    const float* wbase = d.w;
    int aoff[C::AE4];
#pragma unroll
    for (int e = 0; e < C::AE4; ++e) {
        const int f = min(tid + e * 256, C::AN / 4 - 1);
        const int ml = f / (C::S * 16);
        const int r = f - ml * (C::S * 16);
        const int mtg = min(mt0 + ml, mtiles - 1);   // rows past M are computed, never stored
        aoff[e] = (int)(mtg * a_mt_stride) + r * 4;   // float index of the float4
    }

    float xr[C::XE];
    float ar[4 * C::AE4];

#define OU_LOAD_CHUNK(q)                                                                       \
    {                                                                                          \
        const int q_ = (q);                                                                    \
        if (R == 1) {                                                                          \
            const int nch = cin - q_ * CC;                                                     \
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(               \
                (void*)(xb + (int64_t)q_ * CC * xc), (short)0, nch > 0 ? nch * xc * 4 : 0,     \
                0x00020000);                                                                   \
            _Pragma("unroll") for (int e = 0; e < C::XE; ++e) xr[e] =                          \
                __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, xoff[e], 0, 0));      \
        } else {                                                                               \
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(               \
                (void*)xb, (short)0, cin * xc * 4, 0x00020000);                               \
            _Pragma("unroll") for (int e = 0; e < C::XE; ++e) {                                \
                const int idx = tid + e * 256;                                                 \
                const int cq = q_ * CC + (idx - (idx / CC) * CC);                              \
                const int ci = cq / R;                                                         \
                const int pos = xoff[e] + (cq - ci * R);                                       \
                const int off = (idx < C::XN && ci < cin && pos >= 0 && pos < in_len)          \
                                    ? (ci * xc + pos) * 4                                      \
                                    : kSentinel;                                               \
                xr[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));  \
            }                                                                                  \
        }                                                                                      \
        _Pragma("unroll") for (int e = 0; e < C::AE4; ++e) {                                   \
            const float4 v4 = *(const float4*)(wbase + aoff[e] + (int64_t)q_ * C::S * 64);     \
            ar[4 * e] = v4.x;                                                                  \
            ar[4 * e + 1] = v4.y;                                                              \
            ar[4 * e + 2] = v4.z;                                                              \
            ar[4 * e + 3] = v4.w;                                                              \
        }                                                                                      \
    }

#define OU_STORE_CHUNK(buf)                                                                    \
    {                                                                                          \
        float* xs_ = lds + (buf) * C::STAGE;                                                   \
        _Pragma("unroll") for (int e = 0; e < C::XE; ++e) {                                    \
            float v = xr[e] * scale;                                                           \
            v = v >= 0.f ? v : v * slope;                                                      \
            if (loff[e] >= 0) xs_[loff[e]] = v;                                                \
        }                                                                                      \
        float4* as_ = (float4*)(xs_ + C::XBUF);                                                \
        _Pragma("unroll") for (int e = 0; e < C::AE4; ++e) as_[tid + e * 256] =                \
            make_float4(ar[4 * e], ar[4 * e + 1], ar[4 * e + 2], ar[4 * e + 3]);               \
    }

    floatx16 acc[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

    OU_LOAD_CHUNK(0);
    OU_STORE_CHUNK(0);
    __syncthreads();
    for (int q = 0; q < nchunks; ++q) {
        const int cur = q & 1;
        if (q + 1 < nchunks) OU_LOAD_CHUNK(q + 1);
        {
            const float* xs = lds + cur * C::STAGE;
            const float* as = xs + C::XBUF + wm * (C::S * 64) + lane;
            const float* xrow = xs + h * C::WS + wn * (32 * NR) + l32;
#pragma unroll
            for (int cpl = 0; cpl < C::HPW; ++cpl) {
                const int cp = wk * C::HPW + cpl;
#pragma unroll
                for (int k = 0; k < KT; ++k) {
                    const float a = as[(cp * KT + k) * 64];
                    const float* xr_ = xrow + (2 * cp) * C::WS + k;
#pragma unroll
                    for (int nr = 0; nr < NR; ++nr)
                        acc[nr] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xr_[nr * 32], acc[nr],
                                                                       0, 0, 0);
                }
            }
        }
        if (q + 1 < nchunks) OU_STORE_CHUNK(cur ^ 1);
        __syncthreads();
    }
#undef OU_LOAD_CHUNK
#undef OU_STORE_CHUNK

    // ---- intra-workgroup split-K reduction (fixed order: deterministic) ----
    if (WK > 1) {
        float* red = lds;
        const int sub = wm * WN + wn;
        if (wk > 0) {
#pragma unroll
            for (int nr = 0; nr < NR; ++nr)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    red[((((wk - 1) * WM * WN + sub) * NR + nr) * 16 + r) * 64 + lane] = acc[nr][r];
        }
        __syncthreads();
        if (wk > 0) return;
#pragma unroll
        for (int j = 1; j < WK; ++j)
#pragma unroll
            for (int nr = 0; nr < NR; ++nr)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    acc[nr][r] += red[((((j - 1) * WM * WN + sub) * NR + nr) * 16 + r) * 64 + lane];
    }
    if (mt >= mtiles) return;

    // ---- epilogue ----
    const int M = d.m;
    const int rout = d.rout;
    const int cout = M / rout;
    float* __restrict__ y = d.y + (int64_t)b * d.y_bstride;
    const float* r1 = d.res1 ? d.res1 + (int64_t)b * d.r1_bstride : nullptr;
    const float* r2 = d.res2 ? d.res2 + (int64_t)b * d.r2_bstride : nullptr;
    const float* fm = d.film ? d.film + (int64_t)b * d.film_bstride : nullptr;
#pragma unroll
    for (int nr = 0; nr < NR; ++nr) {
        const int u = n0 + wn * (32 * NR) + nr * 32 + l32;
        if (u >= d.n_frames) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int m = mt * 32 + row;
            if (m >= M) continue;
            int co = m, ph = 0;
            if (rout > 1) {
                ph = m / cout;
                co = m - ph * cout;
            }
            const int t = u * rout + ph;
            if (t >= d.out_len) continue;
            float v = acc[nr][r];
            if (d.bias) v += d.bias[co];
            if (t >= d.valid_len) v = 0.f;
            if (r1) v = (v + r1[(int64_t)co * d.r1_cstride + t]) * d.s1;
            if (fm) v = fm[co] * v + fm[cout + co];
            if (r2) v = (v + r2[(int64_t)co * d.r2_cstride + t]) * d.s2;
            y[(int64_t)co * d.y_cstride + t] = v;
        }
    }
}

// ---- tile table ------------------------------------------------------------
struct Tile {
    int wm, wn, wk, nr;
};
// id: 0 32x512, 1 32x256, 2 64x128, 3 64x64, 4 32x32/K4, 5 64x32/K2, 6 32x64/K2, 7 128x32
constexpr Tile kTiles[] = {{1, 4, 1, 4}, {1, 4, 1, 2}, {2, 2, 1, 2}, {2, 2, 1, 1},
                           {1, 1, 4, 1}, {2, 1, 2, 1}, {1, 2, 2, 1}, {4, 1, 1, 1}};
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

constexpr int kMaxLds = 64 * 1024;

// channel chunk: the largest of 64/32/16 whose double-buffered stage fits LDS
template <int KT, int WM, int WN, int WK, int NR>
constexpr int chunk_for()
{
    return Cfg<KT, 64, WM, WN, WK, NR>::LDS * 4 <= kMaxLds   ? 64
           : Cfg<KT, 32, WM, WN, WK, NR>::LDS * 4 <= kMaxLds ? 32
                                                              : 16;
}

template <int KT, int WM, int WN, int WK, int NR>
int launch_t(const ou_conv_desc& d, hipStream_t s)
{
    constexpr int CC = chunk_for<KT, WM, WN, WK, NR>();
    using C = Cfg<KT, CC, WM, WN, WK, NR>;
    const int mtiles = (d.m + 31) / 32;
    const int cin_eff = d.cin * d.frame;
    const int cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
    const int nchunks = (cin_eff + CC - 1) / CC;
    const int64_t a_mt_stride = (int64_t)(cin_pad / 2) * KT * 64;
    dim3 grid((d.n_frames + C::BN - 1) / C::BN, (mtiles + WM - 1) / WM, d.batch);
    const size_t lds = (size_t)C::LDS * sizeof(float);
    hipLaunchKernelGGL((conv_kernel<KT, CC, WM, WN, WK, NR>), grid, dim3(256), lds, s, d, nchunks,
                       mtiles, a_mt_stride);
    return ou_check_launch("conv");
}

template <int KT, int WM, int WN, int WK, int NR>
constexpr int lds_bytes_t()
{
    return Cfg<KT, chunk_for<KT, WM, WN, WK, NR>(), WM, WN, WK, NR>::LDS * 4;
}

template <int KT>
int lds_bytes_kt(int tile)
{
    switch (tile) {
    case 0: return lds_bytes_t<KT, 1, 4, 1, 4>();
    case 1: return lds_bytes_t<KT, 1, 4, 1, 2>();
    case 2: return lds_bytes_t<KT, 2, 2, 1, 2>();
    case 3: return lds_bytes_t<KT, 2, 2, 1, 1>();
    case 4: return lds_bytes_t<KT, 1, 1, 4, 1>();
    case 5: return lds_bytes_t<KT, 2, 1, 2, 1>();
    case 6: return lds_bytes_t<KT, 1, 2, 2, 1>();
    case 7: return lds_bytes_t<KT, 4, 1, 1, 1>();
    }
    return -1;
}

int lds_bytes(int kt, int tile)
{
    switch (kt) {
    case 1: return lds_bytes_kt<1>(tile);
    case 3: return lds_bytes_kt<3>(tile);
    case 4: return lds_bytes_kt<4>(tile);
    case 5: return lds_bytes_kt<5>(tile);
    }
    return -1;
}

template <int KT>
int launch_kt(const ou_conv_desc& d, int tile, hipStream_t s)
{
    switch (tile) {
    case 0: return launch_t<KT, 1, 4, 1, 4>(d, s);
    case 1: return launch_t<KT, 1, 4, 1, 2>(d, s);
    case 2: return launch_t<KT, 2, 2, 1, 2>(d, s);
    case 3: return launch_t<KT, 2, 2, 1, 1>(d, s);
    case 4: return launch_t<KT, 1, 1, 4, 1>(d, s);
    case 5: return launch_t<KT, 2, 1, 2, 1>(d, s);
    case 6: return launch_t<KT, 1, 2, 2, 1>(d, s);
    case 7: return launch_t<KT, 4, 1, 1, 1>(d, s);
    }
    return ou_fail(-2, "conv: bad tile %d", tile);
}

// Static choice (used when the host has not autotuned the layer): the
// largest tile that still gives >= 2 workgroups per CU, split-K when N is short.
int pick_tile(const ou_conv_desc& d)
{
    auto wgs = [&](int t) {
        const Tile& k = kTiles[t];
        const int bm = 32 * k.wm, bn = 32 * k.nr * k.wn;
        return (int64_t)((d.m + bm - 1) / bm) * ((d.n_frames + bn - 1) / bn) * d.batch;
    };
    auto ok = [&](int t) { return lds_bytes(d.kt, t) <= kMaxLds; };
    if (d.m <= 32) {
        for (int t : {0, 1}) if (ok(t) && wgs(t) >= 512) return t;
        return 4;
    }
    for (int t : {2, 3}) if (ok(t) && wgs(t) >= 512) return t;
    if (wgs(6) >= 512) return 6;
    return 4;
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

// Packed order: [m-tile][channel pair cp][tap k][lane]; lane -> (row mt*32 +
// (lane & 31), channel 2*cp + (lane >> 5)); zero outside [0, m) x [0, cin_eff).
extern "C" int ou_conv_pack(const float* w, int m, int cin_eff, int kt, int cc, float* out)
{
    (void)cc;
    if (!w || !out || m <= 0 || cin_eff <= 0 || kt <= 0)
        return ou_fail(-1, "conv_pack: bad arguments");
    const int mtiles = (m + 31) / 32;
    const int cin_pad = (cin_eff + kCinAlign - 1) / kCinAlign * kCinAlign;
    int64_t o = 0;
    for (int mt = 0; mt < mtiles; ++mt)
        for (int cp = 0; cp < cin_pad / 2; ++cp)
            for (int k = 0; k < kt; ++k)
                for (int lane = 0; lane < 64; ++lane) {
                    const int row = mt * 32 + (lane & 31);
                    const int c = 2 * cp + (lane >> 5);
                    out[o++] = (row < m && c < cin_eff) ? w[((int64_t)row * cin_eff + c) * kt + k]
                                                        : 0.f;
                }
    return 0;
}

extern "C" int ou_conv(const ou_conv_desc* dp, void* stream)
{
    if (!dp) return ou_fail(-1, "conv: null descriptor");
    const ou_conv_desc& d = *dp;
    if (!d.x || !d.w || !d.y || d.m <= 0 || d.batch <= 0 || d.n_frames <= 0 || d.cin <= 0 ||
        d.frame <= 0 || d.rout <= 0 || d.m % d.rout != 0 || d.in_len <= 0 || d.out_len <= 0)
        return ou_fail(-1, "conv: invalid descriptor (m=%d rout=%d frame=%d)", d.m, d.rout, d.frame);
    const int tile = d.tile >= 0 && d.tile < kNumTiles ? d.tile : pick_tile(d);
    if (lds_bytes(d.kt, tile) > kMaxLds)
        return ou_fail(-2, "conv: tile %d needs %d B of LDS for kt=%d", tile, lds_bytes(d.kt, tile), d.kt);
    hipStream_t s = (hipStream_t)stream;
    switch (d.kt) {
    case 1: return launch_kt<1>(d, tile, s);
    case 3: return launch_kt<3>(d, tile, s);
    case 4: return launch_kt<4>(d, tile, s);
    case 5: return launch_kt<5>(d, tile, s);
    }
    return ou_fail(-1, "conv: unsupported kt %d", d.kt);
}

extern "C" int ou_conv_pick_tile(const ou_conv_desc* d) { return d ? pick_tile(*d) : -1; }
extern "C" int ou_conv_num_tiles(void) { return kNumTiles; }
extern "C" int ou_conv_tile_ok(int kt, int tile)
{
    return tile >= 0 && tile < kNumTiles && lds_bytes(kt, tile) > 0 && lds_bytes(kt, tile) <= kMaxLds;
}
