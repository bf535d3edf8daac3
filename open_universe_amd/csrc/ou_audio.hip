// ou_audio.hip -- audio-rate resampling around enhance().
//
// Replaces torchaudio.functional.resample(x, orig_freq, new_freq) with its
// defaults (sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99), which the
// reference CLI applies before and after the model (bin/enhance.py:61-64,
// 186-190).  torchaudio computes, with orig/new reduced by their gcd and the
// polyphase table K[new][taps] (taps = 2*width + orig),
//   y[j*new + p] = sum_k K[p][k] * xpad[j*orig + k],  xpad[n] = x[n - width]
// (zero outside [0, n_in)), keeping the first ceil(new * n_in / orig) outputs.
// The table is built on the host (dsp.sinc_resample_kernel) and stays in
// device memory; it is small enough to live in L2 for every common rate pair.
//
// One thread per output sample; neighbouring outputs read overlapping input
// windows, which the vector L1 serves.  HBM-bound: one pass over x and y.
#include <hip/hip_runtime.h>

#include "../../include/ouhip.h"
#include "ou_common.h"

namespace {

__global__ __launch_bounds__(256) void resample_kernel(const float* __restrict__ x, int64_t xbs,
                                                       float* __restrict__ y, int64_t ybs, int n_in, int n_out,
                                                       const float* __restrict__ kern, int phases, int taps,
                                                       int orig, int width)
{
    const int b = blockIdx.y;
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_out) return;
    const int j = o / phases;
    const int p = o - j * phases;
    const float* xb = x + (int64_t)b * xbs;
    const float* k = kern + (int64_t)p * taps;
    const int s0 = j * orig - width;
    float acc = 0.f;
    if (s0 >= 0 && s0 + taps <= n_in) {
        for (int t = 0; t < taps; ++t) acc = fmaf(k[t], xb[s0 + t], acc);
    } else {
        for (int t = 0; t < taps; ++t) {
            const int s = s0 + t;
            if (s >= 0 && s < n_in) acc = fmaf(k[t], xb[s], acc);
        }
    }
    y[(int64_t)b * ybs + o] = acc;
}

}  // namespace

extern "C" int ou_resample(const float* x, int64_t x_bstride, float* y, int64_t y_bstride, int batch, int n_in,
                           int n_out, const float* kernel, int phases, int taps, int orig, int width, void* stream)
{
    if (!x || !y || !kernel || batch <= 0 || n_in <= 0 || n_out <= 0 || phases <= 0 || orig <= 0 || width < 0 ||
        taps != 2 * width + orig)
        return ou_fail(-1, "resample: invalid arguments (phases %d taps %d orig %d width %d)", phases, taps, orig,
                       width);
    if ((int64_t)(n_out - 1) / phases * orig + taps > (int64_t)1 << 31)
        return ou_fail(-1, "resample: signal too long");
    dim3 grid((n_out + 255) / 256, batch);
    hipLaunchKernelGGL(resample_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, x_bstride, y, y_bstride, n_in,
                       n_out, kernel, phases, taps, orig, width);
    return ou_check_launch("resample");
}
