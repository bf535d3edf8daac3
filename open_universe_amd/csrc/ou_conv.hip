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
//   * fp32 inputs => v_mfma_f32_32x32x2_f32 (exact f32 FMA chain, 157 TF peak).
//   * workgroup = 4 waves; each wave owns a 32 x (32*NR) output tile.
//   * K is walked in chunks of cc frame-view channels.  The chunk's input
//     window (cc x (BN + KT - 1) frames) is staged into LDS once, with the
//     PReLU (and the optional per-item input scale) applied on the way in, so
//     the k-tap re-reads of the same sample hit LDS, not HBM.
//   * A (weights) streams straight from global/L2 into VGPRs in per-lane
//     fragment order (packed once on the host by ou_conv_pack), 256 B per wave
//     per MFMA step, coalesced.
//   * Lane halves (lane>>5) take channel c and c+cc/2 of the chunk at the same
//     tap, so every B-fragment read is 32 consecutive floats of one LDS row
//     (conflict-free ds_read_b32) and no per-step index decode is needed.
//   * Epilogue (bias, zero-fill, residual, FiLM, residual) runs on the
//     accumulator registers; each 32-lane half stores one contiguous 128-B
//     row segment.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/ouhip.h"
#include "ou_common.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

template <int KT, int WM, int WN, int NR>
struct ConvCfg {
    static constexpr int BM = 32 * WM;
    static constexpr int BN = 32 * NR * WN;
    static constexpr int W = BN + KT - 1;   // staged frames per chunk
    static constexpr int WS = W;            // LDS row stride (floats)
};

template <int KT, int WM, int WN, int NR>
__global__ __launch_bounds__(256) void conv_kernel(ou_conv_desc d, int nchunks, int mtiles)
{
    using C = ConvCfg<KT, WM, WN, NR>;
    extern __shared__ __attribute__((aligned(16))) float xs[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN;
    const int wn = wave % WN;
    const int b = blockIdx.z;
    const int n0 = blockIdx.x * C::BN;
    const int mt = blockIdx.y * WM + wm;
    const bool active = mt < mtiles;          // wave-uniform
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int cc = d.cc;
    const int half = cc >> 1;
    const int R = d.frame;

    floatx16 acc[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

    const float* __restrict__ x = d.x + (int64_t)b * d.x_bstride;
    const float scale = d.in_scale ? d.in_scale[b] : 1.0f;
    const float slope = d.slope;
    const int t0 = n0 - d.pad;
    const int steps = half * KT;              // MFMA k-steps per chunk
    const int64_t xc = d.x_cstride;
    const int in_len = d.in_len;
    const int cin = d.cin;

    for (int q = 0; q < nchunks; ++q) {
        __syncthreads();
        // ---- stage the chunk's input window into LDS (PReLU applied) ----
        if (R == 1) {
            const int total = cc * C::W;
            for (int e = tid; e < total; e += 256) {
                const int c = e / C::W;
                const int w = e - c * C::W;
                const int ci = q * cc + c;
                const int pos = t0 + w + d.shift;
                float v = 0.f;
                if (ci < cin && pos >= 0 && pos < in_len) {
                    v = x[(int64_t)ci * xc + pos] * scale;
                    v = v >= 0.f ? v : v * slope;
                }
                xs[c * C::WS + w] = v;
            }
        } else {
            // frame view: chunk = cc/R whole channels; walk samples in order so
            // consecutive lanes read consecutive addresses
            const int span = C::W * R;
            const int total = cc * C::W;        // = (cc/R) * span
            const int ci0 = (q * cc) / R;
            const int pos0 = t0 * R + d.shift;
            for (int e = tid; e < total; e += 256) {
                const int cl = e / span;
                const int pl = e - cl * span;
                const int w = pl / R;
                const int p = pl - w * R;
                const int ci = ci0 + cl;
                const int pos = pos0 + pl;
                float v = 0.f;
                if (ci < cin && pos >= 0 && pos < in_len) {
                    v = x[(int64_t)ci * xc + pos] * scale;
                    v = v >= 0.f ? v : v * slope;
                }
                xs[(cl * R + p) * C::WS + w] = v;
            }
        }
        __syncthreads();
        if (!active) continue;

        // ---- MFMA over the chunk ----
        const float* __restrict__ ap =
            d.w + ((int64_t)(mt * nchunks + q) * steps) * 64 + lane;
        const float* xrow = xs + h * half * C::WS + wn * (32 * NR) + l32;
        float a_next[KT];
#pragma unroll
        for (int k = 0; k < KT; ++k) a_next[k] = ap[k * 64];
        for (int cp = 0; cp < half; ++cp) {
            float a[KT];
#pragma unroll
            for (int k = 0; k < KT; ++k) a[k] = a_next[k];
            if (cp + 1 < half) {
#pragma unroll
                for (int k = 0; k < KT; ++k) a_next[k] = ap[((cp + 1) * KT + k) * 64];
            }
            const float* xr = xrow + cp * C::WS;
#pragma unroll
            for (int k = 0; k < KT; ++k) {
#pragma unroll
                for (int nr = 0; nr < NR; ++nr) {
                    acc[nr] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], xr[nr * 32 + k],
                                                                   acc[nr], 0, 0, 0);
                }
            }
        }
    }
    if (!active) return;

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

struct TileShape {
    int wm, wn, nr;
};
// tile ids: 0 = 32x256, 1 = 64x128, 2 = 64x64, 3 = 128x32, 4 = 32x128, 5 = 32x64
constexpr TileShape kTiles[] = {{1, 4, 2}, {2, 2, 2}, {2, 2, 1}, {4, 1, 1}, {1, 4, 1}, {2, 1, 1}};
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

template <int KT, int WM, int WN, int NR>
int launch_t(const ou_conv_desc& d, hipStream_t s)
{
    using C = ConvCfg<KT, WM, WN, NR>;
    const int mtiles = (d.m + 31) / 32;
    const int cin_eff = d.cin * d.frame;
    const int nchunks = (cin_eff + d.cc - 1) / d.cc;
    dim3 grid((d.n_frames + C::BN - 1) / C::BN, (mtiles + WM - 1) / WM, d.batch);
    size_t lds = (size_t)d.cc * C::WS * sizeof(float);
    if (lds > 160 * 1024) return ou_fail(-3, "conv: LDS window too large (cc=%d)", d.cc);
    hipLaunchKernelGGL((conv_kernel<KT, WM, WN, NR>), grid, dim3(256), lds, s, d, nchunks, mtiles);
    return ou_check_launch("conv");
}

template <int KT>
int launch_kt(const ou_conv_desc& d, int tile, hipStream_t s)
{
    switch (tile) {
    case 0: return launch_t<KT, 1, 4, 2>(d, s);
    case 1: return launch_t<KT, 2, 2, 2>(d, s);
    case 2: return launch_t<KT, 2, 2, 1>(d, s);
    case 3: return launch_t<KT, 4, 1, 1>(d, s);
    case 4: return launch_t<KT, 1, 4, 1>(d, s);
    case 5: return launch_t<KT, 2, 1, 1>(d, s);
    }
    return ou_fail(-2, "conv: bad tile %d", tile);
}

int pick_tile(const ou_conv_desc& d)
{
    const int64_t target = 1024;  // workgroups: >= 4 per CU when possible
    auto wgs = [&](int t) {
        const int bm = 32 * kTiles[t].wm, bn = 32 * kTiles[t].nr * kTiles[t].wn;
        return (int64_t)((d.m + bm - 1) / bm) * ((d.n_frames + bn - 1) / bn) * d.batch;
    };
    const int order_small_m[] = {0, 4, 5};
    const int order_big_m[] = {1, 2, 3};
    const int* order = d.m <= 32 ? order_small_m : order_big_m;
    for (int i = 0; i < 3; ++i) {
        const int t = order[i];
        const int bn = 32 * kTiles[t].nr * kTiles[t].wn;
        const size_t lds = (size_t)d.cc * (bn + d.kt - 1) * sizeof(float);
        if (lds > 64 * 1024) continue;
        if (wgs(t) >= target || i == 2) return t;
    }
    return d.m <= 32 ? 5 : 3;
}

}  // namespace

extern "C" int ou_conv_chunk(int kt, int frame)
{
    const int base = kt >= 3 ? 16 : 32;
    int unit = 8;
    // lcm(frame, 8)
    int a = frame, bb = 8;
    while (bb) { int t = a % bb; a = bb; bb = t; }
    unit = frame / a * 8;
    int cc = unit;
    while (cc < base) cc += unit;
    // (cc/2)*kt must be a multiple of 4 for the packed layout: cc % 8 == 0 ensures it
    return cc;
}

extern "C" int64_t ou_conv_packed_size(int m, int cin_eff, int kt, int cc)
{
    const int64_t mtiles = (m + 31) / 32;
    const int64_t nchunks = (cin_eff + cc - 1) / cc;
    return mtiles * nchunks * (int64_t)(cc / 2) * kt * 64;
}

extern "C" int ou_conv_pack(const float* w, int m, int cin_eff, int kt, int cc, float* out)
{
    if (!w || !out || m <= 0 || cin_eff <= 0 || kt <= 0 || cc <= 0 || (cc & 1))
        return ou_fail(-1, "conv_pack: bad arguments");
    const int mtiles = (m + 31) / 32;
    const int nchunks = (cin_eff + cc - 1) / cc;
    const int half = cc / 2;
    int64_t o = 0;
    for (int mt = 0; mt < mtiles; ++mt)
        for (int q = 0; q < nchunks; ++q)
            for (int cp = 0; cp < half; ++cp)
                for (int k = 0; k < kt; ++k)
                    for (int lane = 0; lane < 64; ++lane) {
                        const int row = mt * 32 + (lane & 31);
                        const int c = q * cc + cp + (lane >> 5) * half;
                        out[o++] = (row < m && c < cin_eff)
                                       ? w[((int64_t)row * cin_eff + c) * kt + k]
                                       : 0.f;
                    }
    return 0;
}

extern "C" int ou_conv(const ou_conv_desc* dp, void* stream)
{
    if (!dp) return ou_fail(-1, "conv: null descriptor");
    ou_conv_desc d = *dp;
    if (!d.x || !d.w || !d.y || d.m <= 0 || d.batch <= 0 || d.n_frames <= 0 || d.cin <= 0 ||
        d.frame <= 0 || d.rout <= 0 || d.m % d.rout != 0 || d.cc <= 0 || (d.cc & 1) ||
        (d.frame > 1 && d.cc % d.frame != 0))
        return ou_fail(-1, "conv: invalid descriptor (m=%d rout=%d cc=%d frame=%d)", d.m, d.rout,
                       d.cc, d.frame);
    int tile = d.tile >= 0 && d.tile < kNumTiles ? d.tile : pick_tile(d);
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
