// ou_misc.hip -- the small kernels around the convolution stack (gfx950).
//
//  * ou_embed     noise-level embedding + all FiLM projections (SURVEY.md K7;
//                 networks/universe/sigma_block.py:24-78, score.py:104-110,197-210)
//  * ou_head      score-net output (two PReLUs + Conv1d(C->1,k3)) fused with
//                 the EDM wrapper and the sampler update (K9; score.py:290-296,
//                 universe.py:197-209,334-343)
//  * reductions   normalize_batch (utils/norm.py:47-87), mel normalisation
//                 (condition.py:104-106), keep_rms / peak normalisation
//                 (universe.py:259,352-357)
//  * ou_snake_aa  alias-free Snake of the signal-decoupling layer
//                 (bigvgan/snake.py:131-157, alias_free_act.py:8-30)
//  * small elementwise helpers (pad, scale, |STFT|^2, ensemble mean/median)
//  * ou_signal_median  ensemble signal_median (utils/stats.py:22-66)
//
// All of these are HBM- or latency-bound and tiny next to the conv stack; they
// exist so that no op of the sampler leaves the device or touches ATen.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "../../include/ouhip.h"
#include "ou_common.h"

namespace {

constexpr float kPi = 3.14159265358979323846f;

__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ __forceinline__ float wave_max(float v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

// block (<= 1024 threads) sum; result valid in every thread
__device__ float block_sum(float v, float* red)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nw = (blockDim.x + 63) >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[i];
    return s;
}

__device__ float block_max(float v, float* red)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nw = (blockDim.x + 63) >> 6;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    float s = red[0];
    for (int i = 1; i < nw; ++i) s = fmaxf(s, red[i]);
    return s;
}

// ---------------------------------------------------------------- embedding
// g for one sigma per workgroup -> gbuf[i][dim]
__global__ __launch_bounds__(256) void embed_g_kernel(ou_embed_desc d, float* gbuf)
{
    __shared__ float s0[1024], s1[1024];
    const int i = blockIdx.x;
    const float ls = log10f(d.sigma[i]);
    float* g = gbuf + (int64_t)i * d.dim;
    if (d.kind == 0) {
        // SimpleTimeEmbedding: f = 0.5 sigmoid(w*ls + b); p = (2 pi f) * k
        const float f = 0.5f * (1.0f / (1.0f + expf(-(d.te_weight * ls + d.te_bias))));
        const float tpf = (2.0f * kPi) * f;
        const int half = d.dim / 2;
        for (int k = threadIdx.x; k < half; k += blockDim.x) {
            const float p = tpf * (float)k;
            g[k] = sinf(p);
            g[half + k] = cosf(p);
        }
        return;
    }
    // SigmaBlock: rff -> 3 x (Linear + PReLU)
    const int nr = d.n_rff;
    for (int k = threadIdx.x; k < nr; k += blockDim.x) {
        const float p = (2.0f * kPi) * d.rff_freq[k] * ls;
        s0[k] = sinf(p);
        s0[nr + k] = cosf(p);
    }
    __syncthreads();
    int din = 2 * nr;
    float* src = s0;
    float* dst = s1;
    for (int l = 0; l < 3; ++l) {
        const int dout = l == 2 ? d.dim : din * 2;
        for (int o = threadIdx.x; o < dout; o += blockDim.x) {
            const float* wr = d.mlp_w[l] + (int64_t)o * din;
            float acc = 0.f;
            for (int k = 0; k < din; ++k) acc = fmaf(wr[k], src[k], acc);
            acc += d.mlp_b[l][o];
            dst[o] = acc >= 0.f ? acc : acc * d.mlp_slope[l];
        }
        __syncthreads();
        float* t = src; src = dst; dst = t;
        din = dout;
    }
    for (int k = threadIdx.x; k < d.dim; k += blockDim.x) g[k] = src[k];
}

// one wave per (sigma, row): out[i][r] = W[r] . g_i + bias[r]
__global__ __launch_bounds__(256) void embed_proj_kernel(ou_embed_desc d, const float* gbuf)
{
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int i = blockIdx.y;
    if (r >= d.rows) return;
    const float* w = d.w + (int64_t)r * d.dim;
    const float* g = gbuf + (int64_t)i * d.dim;
    float acc = 0.f;
    for (int k = lane; k < d.dim; k += 64) acc = fmaf(w[k], g[k], acc);
    acc = wave_sum(acc);
    if (lane == 0) d.out[(int64_t)i * d.rows + r] = acc + d.bias[r];
}

// ---------------------------------------------------------------- head
__global__ __launch_bounds__(256) void head_kernel(ou_head_desc d)
{
    const int b = blockIdx.y;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= d.length) return;
    const float* h = d.h + (int64_t)b * d.h_bstride;
    const int T = d.length;
    // taps t-1, t, t+1 with zero padding: clamped (always valid) addresses and
    // 0/1 masks, so the loads of a channel group issue back to back instead of
    // one branch-guarded round trip each; the FMA order (c, then k) is the
    // reference's conv1d summation order
    const int tl = max(t - 1, 0), tr = min(t + 1, T - 1);
    const float ml = t >= 1 ? 1.f : 0.f, mr = t + 1 < T ? 1.f : 0.f;
    float net = 0.f;
    constexpr int CG = 8;   // channels per load group
    for (int c0 = 0; c0 < d.channels; c0 += CG) {
        float v[CG][3];
#pragma unroll
        for (int j = 0; j < CG; ++j) {
            const int c = min(c0 + j, d.channels - 1);
            const float* hc = h + (int64_t)c * T;
            v[j][0] = hc[tl];
            v[j][1] = hc[t];
            v[j][2] = hc[tr];
        }
#pragma unroll
        for (int j = 0; j < CG; ++j) {
            if (c0 + j >= d.channels) break;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                float x = v[j][k];
                x = x >= 0.f ? x : x * d.slope1;
                x = x >= 0.f ? x : x * d.slope2;
                x = k == 0 ? x * ml : (k == 2 ? x * mr : x);
                net = fmaf(d.w[(c0 + j) * 3 + k], x, net);
            }
        }
    }
    net += d.bias;
    const int64_t o = (int64_t)b * T + t;
    float out;
    if (d.mode == 0) {
        out = net;
    } else {
        const float x = d.x[o];
        float score;
        if (d.edm) {
            const float est = __fadd_rn(__fmul_rn(d.w_skip, x), __fmul_rn(d.w_out, net));
            score = __fdiv_rn(__fsub_rn(est, x), d.s2);
        } else {
            score = net;
        }
        out = __fadd_rn(x, __fmul_rn(d.c_score, score));
        if (d.mode == 1) out = __fadd_rn(out, __fmul_rn(d.c_noise, __fmul_rn(d.z[o], d.s_next)));
    }
    d.out[o] = out;
}

// ---------------------------------------------------------------- reductions
// One workgroup per batch item reads the whole signal (128k samples at 8 s):
// 16-B loads with four independent partial sums per thread keep several loads
// in flight, instead of one dependent scalar load per iteration.
template <class F>
__device__ float reduce_sum(const float* x, int64_t n, F f, float* red)
{
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    const int64_t bd = blockDim.x;
    int64_t done = 0;
    if (((uintptr_t)x & 15) == 0) {
        const float4* x4 = (const float4*)x;
        const int64_t n4 = n >> 2;
        int64_t i = threadIdx.x;
        for (; i + 3 * bd < n4; i += 4 * bd) {
            const float4 v0 = x4[i], v1 = x4[i + bd], v2 = x4[i + 2 * bd], v3 = x4[i + 3 * bd];
            a0 += (f(v0.x) + f(v0.y)) + (f(v0.z) + f(v0.w));
            a1 += (f(v1.x) + f(v1.y)) + (f(v1.z) + f(v1.w));
            a2 += (f(v2.x) + f(v2.y)) + (f(v2.z) + f(v2.w));
            a3 += (f(v3.x) + f(v3.y)) + (f(v3.z) + f(v3.w));
        }
        for (; i < n4; i += bd) {
            const float4 v = x4[i];
            a0 += (f(v.x) + f(v.y)) + (f(v.z) + f(v.w));
        }
        done = n4 << 2;
    }
    for (int64_t i = done + threadIdx.x; i < n; i += bd) a1 += f(x[i]);
    return block_sum((a0 + a1) + (a2 + a3), red);
}

template <class F>
__device__ float reduce_max(const float* x, int64_t n, F f, float* red)
{
    float m0 = 0.f, m1 = 0.f;
    const int64_t bd = blockDim.x;
    int64_t done = 0;
    if (((uintptr_t)x & 15) == 0) {
        const float4* x4 = (const float4*)x;
        const int64_t n4 = n >> 2;
        int64_t i = threadIdx.x;
        for (; i + bd < n4; i += 2 * bd) {
            const float4 v0 = x4[i], v1 = x4[i + bd];
            m0 = fmaxf(m0, fmaxf(fmaxf(f(v0.x), f(v0.y)), fmaxf(f(v0.z), f(v0.w))));
            m1 = fmaxf(m1, fmaxf(fmaxf(f(v1.x), f(v1.y)), fmaxf(f(v1.z), f(v1.w))));
        }
        for (; i < n4; i += bd) {
            const float4 v = x4[i];
            m0 = fmaxf(m0, fmaxf(fmaxf(f(v.x), f(v.y)), fmaxf(f(v.z), f(v.w))));
        }
        done = n4 << 2;
    }
    for (int64_t i = done + threadIdx.x; i < n; i += bd) m1 = fmaxf(m1, f(x[i]));
    return block_max(fmaxf(m0, m1), red);
}

__global__ __launch_bounds__(1024) void normalize_kernel(const float* x, float* y, int64_t n,
                                                          float level, float eps)
{
    __shared__ float red[16];
    const int b = blockIdx.x;
    const float* xb = x + (int64_t)b * n;
    float* yb = y + (int64_t)b * n;
    const float mean = reduce_sum(xb, n, [](float v) { return v; }, red) / (float)n;
    const float ss = reduce_sum(xb, n, [mean](float v) { return (v - mean) * (v - mean); }, red);
    const float var = ss / (float)(n > 1 ? n - 1 : 1);
    const float gain = level / fmaxf(sqrtf(var), eps);
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) yb[i] = (xb[i] - mean) * gain;
}

__global__ __launch_bounds__(1024) void sumsq_kernel(const float* x, float* out, int64_t n,
                                                      float denom, float eps, int mode)
{
    __shared__ float red[16];
    const int b = blockIdx.x;
    const float tot = reduce_sum(x + (int64_t)b * n, n, [](float v) { return v * v; }, red);
    if (threadIdx.x == 0) {
        const float rms = sqrtf(tot / denom);
        out[b] = mode == 0 ? 1.0f / fmaxf(rms, eps) : rms;
    }
}

__global__ __launch_bounds__(1024) void finish_kernel(const float* x, int64_t xb_stride, int left,
                                                       float* y, int len, const float* mix_rms)
{
    __shared__ float red[16];
    const int b = blockIdx.x;
    const float* xb = x + (int64_t)b * xb_stride + left;
    float* yb = y + (int64_t)b * len;
    float ratio = 1.f;
    if (mix_rms) {
        const float ss = reduce_sum(xb, len, [](float v) { return v * v; }, red);
        const float xr = fmaxf(sqrtf(ss / (float)len), 1e-5f);
        ratio = mix_rms[b] / xr;
    }
    const float peak = reduce_max(xb, len, [ratio](float v) { return fabsf(v * ratio); }, red);
    for (int i = threadIdx.x; i < len; i += blockDim.x) {
        float v = mix_rms ? xb[i] * ratio : xb[i];
        if (peak > 1.0f) v = v / peak;
        yb[i] = v;
    }
}

// ---------------------------------------------------------------- elementwise
__global__ void power_kernel(const float* x, float* y, int nf, int frames, int64_t total)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t per = (int64_t)nf * frames;
    const int64_t b = i / per;
    const int64_t r = i - b * per;
    const float* xb = x + b * 2 * per;
    const float re = xb[r], im = xb[per + r];
    y[i] = re * re + im * im;
}

__global__ void pad_kernel(const float* x, int64_t xbs, float* y, int n_in, int n_out, int left,
                           int64_t total)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t b = i / n_out;
    const int t = (int)(i - b * n_out) - left;
    y[i] = (t >= 0 && t < n_in) ? x[b * xbs + t] : 0.f;
}

__global__ void scale_kernel(const float* z, float* y, int64_t n, float s, const float* add)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = z[i] * s;
    y[i] = add ? __fadd_rn(add[i], v) : v;
}

__global__ void ensemble_kernel(const float* x, float* y, int E, int64_t n, int mode)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (mode == 0) {
        float s = 0.f;
        for (int e = 0; e < E; ++e) s += x[(int64_t)e * n + i];
        y[i] = s / (float)E;
        return;
    }
    float v[32];
    for (int e = 0; e < E; ++e) {
        const float a = x[(int64_t)e * n + i];
        int p = e;
        while (p > 0 && v[p - 1] > a) { v[p] = v[p - 1]; --p; }
        v[p] = a;
    }
    y[i] = v[(E - 1) / 2];   // torch.median: lower median
}

// ---------------------------------------------------------------- signal median
// utils/stats.py:22-66 (signal_median) over x[E][B][n]: at every sample the
// reference sorts the E members, takes the rank position k at which the member
// whose INDEX is closest to E/2 sits (argmin over the sorted index list, first
// occurrence), histograms k over the samples of each batch item, and returns
// the member whose index equals the most frequent k (argmax, first
// occurrence).  Rank of member j: #{i : x_i < x_j} + #{i < j : x_i == x_j}
// (the order of a stable sort; torch's CPU sort is stable up to 16 members,
// unstable beyond, which only matters for exact ties).  Candidates: j = E/2 for even E; for odd
// E the two members (E-1)/2 and (E+1)/2 tie at distance 1/2 and the one
// sorted first wins.
__device__ __forceinline__ int member_rank(const float* x, int64_t estride, int E, int j)
{
    const float v = x[(int64_t)j * estride];
    int r = 0;
    for (int i = 0; i < E; ++i) {
        const float u = x[(int64_t)i * estride];
        r += (u < v) || (u == v && i < j);
    }
    return r;
}

__global__ __launch_bounds__(256) void sigmed_vote_kernel(const float* x, int E, int B, int64_t n,
                                                          int* counts)
{
    __shared__ int hist[32];
    const int b = blockIdx.y;
    if (threadIdx.x < 32) hist[threadIdx.x] = 0;
    __syncthreads();
    const int64_t es = (int64_t)B * n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float* xs = x + (int64_t)b * n + i;
        int k;
        if ((E & 1) == 0) {
            k = member_rank(xs, es, E, E / 2);
        } else {
            k = member_rank(xs, es, E, (E - 1) / 2);
            if (E > 1) k = min(k, member_rank(xs, es, E, (E + 1) / 2));
        }
        atomicAdd(&hist[k], 1);
    }
    __syncthreads();
    if (threadIdx.x < E && hist[threadIdx.x]) atomicAdd(&counts[b * 32 + threadIdx.x], hist[threadIdx.x]);
}

__global__ __launch_bounds__(256) void sigmed_pick_kernel(const float* x, float* y, int E, int B, int64_t n,
                                                          const int* counts)
{
    const int b = blockIdx.y;
    int sel = 0, best = counts[b * 32];
    for (int e = 1; e < E; ++e) {
        const int c = counts[b * 32 + e];
        if (c > best) best = c, sel = e;
    }
    const float* xs = x + ((int64_t)sel * B + b) * n;
    float* ys = y + (int64_t)b * n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        ys[i] = xs[i];
}

// ---------------------------------------------------------------- alias-free snake
// y[b][c][t] = down2( snake( up2(h[b][c][:]) ) )[t]
//   up2:   u[2s + i] = sum_k ku[i][k] * h[s + k - wu]       (torchaudio Resample 1->2)
//   snake: v = u + sin(a u)^2 / (a + 1e-9)
//   down2: y[t] = sum_k kd[k] * v[2t + k - wd]              (torchaudio Resample 2->1)
constexpr int kSnakeTile = 256;
__global__ __launch_bounds__(256) void snake_aa_kernel(ou_snake_desc d)
{
    __shared__ float sh[kSnakeTile + 64];
    __shared__ float sv[2 * kSnakeTile + 64];
    const int c = blockIdx.y, b = blockIdx.z;
    const int t0 = blockIdx.x * kSnakeTile;
    const int T = d.length;
    const int wu = d.width_up, wd = d.width_down;
    const int tu = d.taps_up, td = d.taps_down;
    const float* h = d.h + (int64_t)b * d.h_bstride + (int64_t)c * T;
    const float a = d.alpha[c];
    const float inv = 1.0f / (a + 1e-9f);
    // up-sampled range needed: v index [2*t0 - wd, 2*(t0+tile-1) - wd + td - 1]
    const int v0 = 2 * t0 - wd;
    const int nv = 2 * (kSnakeTile - 1) + td;
    // which h samples feed v[v0 .. v0+nv): s = floor(v/2) + k - wu
    const int s0 = (v0 >= 0 ? v0 / 2 : -((-v0 + 1) / 2)) - wu;
    const int ns = nv / 2 + tu + 2;
    for (int i = threadIdx.x; i < ns; i += blockDim.x) {
        const int s = s0 + i;
        sh[i] = (s >= 0 && s < T) ? h[s] : 0.f;
    }
    __syncthreads();
    const int L2 = 2 * T;   // length of the up-sampled signal
    for (int i = threadIdx.x; i < nv; i += blockDim.x) {
        const int vi = v0 + i;
        float v = 0.f;
        if (vi >= 0 && vi < L2) {
            const int s = vi >> 1, ph = vi & 1;
            const float* k = d.k_up + ph * tu;
            float u = 0.f;
            for (int q = 0; q < tu; ++q) u = fmaf(k[q], sh[s + q - wu - s0], u);
            const float sn = sinf(u * a);
            v = u + inv * (sn * sn);
        }
        sv[i] = v;
    }
    __syncthreads();
    const int t = t0 + threadIdx.x;
    if (t < T) {
        float y = 0.f;
        for (int q = 0; q < td; ++q) y = fmaf(d.k_down[q], sv[2 * threadIdx.x + q], y);
        d.out[((int64_t)b * d.channels + c) * T + t] = y;
    }
}

inline unsigned blocks_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

extern "C" int ou_embed(const ou_embed_desc* d, void* stream)
{
    if (!d || !d->sigma || !d->out || !d->w || !d->gbuf || d->n <= 0)
        return ou_fail(-1, "embed: invalid descriptor");
    if (d->kind == 1 && (d->n_rff * 2 > 1024 || d->dim > 1024 || !d->rff_freq))
        return ou_fail(-1, "embed: bad SigmaBlock sizes");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(embed_g_kernel, dim3(d->n), dim3(256), 0, s, *d, d->gbuf);
    int rc = ou_check_launch("embed_g");
    if (rc) return rc;
    hipLaunchKernelGGL(embed_proj_kernel, dim3((d->rows + 3) / 4, d->n), dim3(256), 0, s, *d,
                       (const float*)d->gbuf);
    return ou_check_launch("embed_proj");
}

extern "C" int ou_head(const ou_head_desc* d, void* stream)
{
    if (!d || !d->h || !d->w || !d->out || d->length <= 0 || d->batch <= 0)
        return ou_fail(-1, "head: invalid descriptor");
    if (d->mode != 0 && !d->x) return ou_fail(-1, "head: sampler mode needs x");
    if (d->mode == 1 && !d->z) return ou_fail(-1, "head: step mode needs z");
    hipLaunchKernelGGL(head_kernel, dim3(blocks_for(d->length, 256), d->batch), dim3(256), 0,
                       (hipStream_t)stream, *d);
    return ou_check_launch("head");
}

extern "C" int ou_normalize(const float* x, float* y, int batch, int64_t n, float level, float eps,
                            void* stream)
{
    if (!x || !y || batch <= 0 || n <= 0) return ou_fail(-1, "normalize: bad args");
    hipLaunchKernelGGL(normalize_kernel, dim3(batch), dim3(1024), 0, (hipStream_t)stream, x, y, n,
                       level, eps);
    return ou_check_launch("normalize");
}

extern "C" int ou_inv_rms(const float* x, float* out, int batch, int64_t n, float denom, float eps,
                          void* stream)
{
    if (!x || !out || batch <= 0 || n <= 0) return ou_fail(-1, "inv_rms: bad args");
    hipLaunchKernelGGL(sumsq_kernel, dim3(batch), dim3(1024), 0, (hipStream_t)stream, x, out, n,
                       denom, eps, 0);
    return ou_check_launch("inv_rms");
}

extern "C" int ou_rms(const float* x, float* out, int batch, int64_t n, void* stream)
{
    if (!x || !out || batch <= 0 || n <= 0) return ou_fail(-1, "rms: bad args");
    hipLaunchKernelGGL(sumsq_kernel, dim3(batch), dim3(1024), 0, (hipStream_t)stream, x, out, n,
                       (float)n, 0.f, 1);
    return ou_check_launch("rms");
}

extern "C" int ou_power(const float* x, float* y, int batch, int nf, int frames, void* stream)
{
    const int64_t total = (int64_t)batch * nf * frames;
    if (!x || !y || total <= 0) return ou_fail(-1, "power: bad args");
    hipLaunchKernelGGL(power_kernel, dim3(blocks_for(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, y, nf, frames, total);
    return ou_check_launch("power");
}

extern "C" int ou_pad(const float* x, int64_t x_bstride, float* y, int batch, int n_in, int n_out,
                      int left, void* stream)
{
    const int64_t total = (int64_t)batch * n_out;
    if (!x || !y || total <= 0) return ou_fail(-1, "pad: bad args");
    hipLaunchKernelGGL(pad_kernel, dim3(blocks_for(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, x_bstride, y, n_in, n_out, left, total);
    return ou_check_launch("pad");
}

extern "C" int ou_scale(const float* z, float* y, int64_t n, float scale, const float* add,
                        void* stream)
{
    if (!z || !y || n <= 0) return ou_fail(-1, "scale: bad args");
    hipLaunchKernelGGL(scale_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                       z, y, n, scale, add);
    return ou_check_launch("scale");
}

extern "C" int ou_finish(const float* x, int64_t x_bstride, int left, float* y, int batch, int len,
                         const float* mix_rms, void* stream)
{
    if (!x || !y || batch <= 0 || len <= 0) return ou_fail(-1, "finish: bad args");
    hipLaunchKernelGGL(finish_kernel, dim3(batch), dim3(1024), 0, (hipStream_t)stream, x,
                       x_bstride, left, y, len, mix_rms);
    return ou_check_launch("finish");
}

extern "C" int ou_ensemble_reduce(const float* x, float* y, int ensemble, int64_t n, int mode,
                                  void* stream)
{
    if (!x || !y || ensemble <= 0 || ensemble > 32 || n <= 0)
        return ou_fail(-1, "ensemble: bad args (ensemble <= 32)");
    hipLaunchKernelGGL(ensemble_kernel, dim3(blocks_for(n, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, y, ensemble, n, mode);
    return ou_check_launch("ensemble");
}

extern "C" int ou_signal_median(const float* x, float* y, int ensemble, int batch, int64_t n, int* counts,
                                void* stream)
{
    if (!x || !y || !counts || ensemble <= 0 || ensemble > 32 || batch <= 0 || n <= 0)
        return ou_fail(-1, "signal_median: bad args (ensemble <= 32)");
    hipStream_t s = (hipStream_t)stream;
    OU_HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(int) * 32 * (size_t)batch, s), "signal_median counts");
    const unsigned gx = (unsigned)std::min<int64_t>(blocks_for(n, 256), 1024);
    hipLaunchKernelGGL(sigmed_vote_kernel, dim3(gx, batch), dim3(256), 0, s, x, ensemble, batch, n, counts);
    int rc = ou_check_launch("signal_median vote");
    if (rc) return rc;
    hipLaunchKernelGGL(sigmed_pick_kernel, dim3(gx, batch), dim3(256), 0, s, x, y, ensemble, batch, n,
                       (const int*)counts);
    return ou_check_launch("signal_median pick");
}

extern "C" int ou_snake_aa(const ou_snake_desc* d, void* stream)
{
    if (!d || !d->h || !d->out || !d->alpha || !d->k_up || !d->k_down || d->length <= 0)
        return ou_fail(-1, "snake_aa: invalid descriptor");
    if (d->taps_up > 32 || d->taps_down > 64)
        return ou_fail(-1, "snake_aa: kernel too long");
    dim3 grid(blocks_for(d->length, kSnakeTile), d->channels, d->batch);
    hipLaunchKernelGGL(snake_aa_kernel, grid, dim3(256), 0, (hipStream_t)stream, *d);
    return ou_check_launch("snake_aa");
}
