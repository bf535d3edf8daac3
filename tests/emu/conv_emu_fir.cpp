// Numerics of the FIR-applied rate-change kernels on the CPU (fiber emulator,
// OU_EMU_FIBERS; tile bit 17, ou_conv_desc.fir):
//   down: y[co][u] = bias + sum_{ci,ph} W[co][ci][ph] f[ci][u R + ph],
//         f = FIR(prelu(x)) ('same', zero outside [0, T))     blocks.py:214-218
//   up:   z[co][s] = sum_ci W[ci][co][s % R] prelu(x)[ci][s / R]  (s < T R),
//         y[co][t] = FIR(z)[t] + bias (zero outside [0, T R))   blocks.py:221-225
// then zero-fill past valid_len, residual, FiLM, residual -- against a
// double-precision evaluation, for every OU_FTILES shape, split-f16 and f16.
// argv[1] = rate R (2, 3, 4, 5, 8); prints one line per failure, exits 1.
#include "../../open_universe_amd/csrc/ou_conv.hip"

#include <cmath>
#include <string>

static uint32_t g_seed = 4242;
static float rnd()
{
    g_seed = g_seed * 1664525u + 1013904223u;
    return ((g_seed >> 8) & 0xffff) / 32768.0f - 1.0f;
}

static std::vector<float> binomial(int n)
{
    std::vector<double> c(n, 0.0);
    c[0] = 1.0;
    for (int i = 1; i < n; ++i)
        for (int j = i; j > 0; --j) c[j] += c[j - 1];
    double ss = 0;
    for (double v : c) ss += v * v;
    std::vector<float> t(n);
    for (int i = 0; i < n; ++i) t[i] = (float)(c[i] / std::sqrt(ss / n));
    return t;
}

struct Case {
    int dir;            // 1 down, 2 up
    int cin, cout, T, B;
    bool res1, res2, film, sy;
    int valid_cut;      // valid_len = full - cut
    int crop;           // up: out_len = T R - crop (-1: 1 when R > 2)
};

// fir 3 (st_convs): a plain strided conv, kernel = stride = Rt, in the FIR
// kernels' blocked K order, walked in chunks of 8 (or 4) phases
static int st_cases(int& n)
{
    int bad = 0;
    const float slope = 0.25f;
    const int rts[] = {20, 40, 24};
    for (int Rt : rts) {
        const int cin = 32, cout = 64, B = 2, T = 7 * Rt + 5, U = (T + Rt - 1) / Rt;
        std::vector<float> w((size_t)cout * cin * Rt), x((size_t)B * cin * T), bias(cout),
            r1((size_t)B * cout * U), r2(r1.size());
        for (auto* v : {&w, &x, &bias, &r1, &r2})
            for (auto& e : *v) e = rnd();
        const bool res = Rt == 40;   // the running st_conv sum: two residuals (the generic epilogue)
        std::vector<double> ref((size_t)B * cout * U);
        for (int b = 0; b < B; ++b)
            for (int co = 0; co < cout; ++co)
                for (int u = 0; u < U; ++u) {
                    double acc = bias[co];
                    for (int ci = 0; ci < cin; ++ci)
                        for (int ph = 0; ph < Rt; ++ph) {
                            const int t = u * Rt + ph;
                            if (t >= T) continue;
                            double v = x[((size_t)b * cin + ci) * T + t];
                            v = v >= 0 ? v : v * slope;
                            acc += (double)w[((size_t)co * cin + ci) * Rt + ph] * v;
                        }
                    const size_t o = ((size_t)b * cout + co) * U + u;
                    ref[o] = res ? (acc + r1[o] + r2[o]) : acc;
                }
        const int keff = cin * Rt;
        const int R = Rt % 8 == 0 ? 8 : 4;   // phases per K chunk (ou_conv)
        std::vector<float> wl((size_t)cout * keff);
        for (int co = 0; co < cout; ++co)
            for (int ci = 0; ci < cin; ++ci)
                for (int ph = 0; ph < Rt; ++ph)
                    wl[(size_t)co * keff + (((ci / 16) * (Rt / R) + ph / R) * 16 + ci % 16) * R + ph % R] =
                        w[((size_t)co * cin + ci) * Rt + ph];
        std::vector<float> packed(ou_conv_packed_size(cout, keff, 1, 0));
        float unscale = 0.f;
        ou_conv_pack_split_nat(wl.data(), cout, keff, 1, packed.data(), &unscale);
        double rn = 0;
        for (double v : ref) rn += v * v;
        for (int shape = 0; shape < kNumFTiles; ++shape) {
            std::vector<float> y(ref.size(), 1e30f);
            ou_conv_desc d{};
            d.x = x.data(); d.x_bstride = (int64_t)cin * T; d.x_cstride = T;
            d.cin = cin; d.in_len = T; d.frame = Rt; d.slope = slope;
            d.w = packed.data(); d.m = cout; d.kt = 1; d.pad = 0;
            d.n_frames = U; d.batch = B; d.y = y.data(); d.y_bstride = (int64_t)cout * U; d.y_cstride = U;
            d.rout = 1; d.out_len = U; d.valid_len = 1 << 30; d.bias = bias.data();
            d.prec = 1; d.w_unscale = unscale; d.xs_shift = 6; d.fir = 3;
            if (res) {
                d.res1 = r1.data(); d.r1_bstride = d.y_bstride; d.r1_cstride = U; d.s1 = 1.f;
                d.res2 = r2.data(); d.r2_bstride = d.y_bstride; d.r2_cstride = U; d.s2 = 1.f;
            }
            d.tile = kFirBit | shape;
            if (ou_conv(&d, nullptr) != 0) {
                std::printf("st Rt %d shape %d: launch error %s\n", Rt, shape, ouhip_detail::err_buf());
                ++bad;
                continue;
            }
            double en = 0;
            for (size_t i = 0; i < y.size(); ++i) en += (y[i] - ref[i]) * (y[i] - ref[i]);
            ++n;
            if (!(std::sqrt(en / rn) < 2e-6)) {
                std::printf("st Rt %d shape %d: rel err %.3g\n", Rt, shape, std::sqrt(en / rn));
                ++bad;
            }
        }
    }
    return bad;
}

int main(int argc, char** argv)
{
    if (argc > 1 && std::string(argv[1]) == "st") {
        int n = 0;
        const int bad = st_cases(n);
        std::printf("%s: %d launches checked, %d bad\n", bad ? "FAIL" : "ok", n, bad);
        return bad ? 1 : 0;
    }
    const int R = argc > 1 ? std::atoi(argv[1]) : 2;
    int bad = 0, n = 0;
    const Case cases[] = {
        {1, 32, 64, 157, 2, false, false, true, true, 0, 0},
        {1, 16, 32, 29, 1, true, false, false, false, 1, 0},
        {1, 48, 96, 203, 2, false, false, false, true, 2, 0},   // bias only: the lean epilogue (+ split image)
        {2, 64, 32, 41, 2, true, false, false, false, 3, -1},
        {2, 32, 16, 13, 1, true, true, true, false, 0, -1},
        {2, 32, 32, 40, 2, true, false, false, false, 0, 0},    // rows 16-B aligned: the 16-B epilogue
    };
    const std::vector<float> tap = binomial(2 * R + 1);
    const float slope = 0.25f;
    for (const Case& c : cases) {
        const bool down = c.dir == 1;
        const int U = down ? (c.T + R - 1) / R : c.T;          // frames (output frames down, input frames up)
        const int out_len = down ? U : c.T * R - (c.crop < 0 ? (R > 2 ? 1 : 0) : c.crop);
        const int full = down ? U : c.T * R;
        const int valid = full - c.valid_cut;
        const int s = 5 + R % 3;   // staging exponent
        std::vector<float> w((size_t)c.cout * c.cin * R), x((size_t)c.B * c.cin * c.T), bias(c.cout),
            r1((size_t)c.B * c.cout * out_len), r2(r1.size()), fm((size_t)c.B * 2 * c.cout);
        for (auto* v : {&w, &x, &bias, &r1, &r2, &fm})
            for (auto& e : *v) e = rnd();
        // the reference weight: down Conv1d (cout, cin, R); up ConvTranspose1d (cin, cout, R)
        auto W = [&](int co, int ci, int ph) {
            return down ? w[((size_t)co * c.cin + ci) * R + ph] : w[((size_t)ci * c.cout + co) * R + ph];
        };
        // ---- double-precision reference
        std::vector<double> ref((size_t)c.B * c.cout * out_len, 0.0);
        for (int b = 0; b < c.B; ++b) {
            auto P = [&](int ci, int t) -> double {
                if (t < 0 || t >= c.T) return 0.0;
                const double v = x[((size_t)b * c.cin + ci) * c.T + t];
                return v >= 0 ? v : v * slope;
            };
            for (int co = 0; co < c.cout; ++co) {
                std::vector<double> pre;   // before bias
                if (down) {
                    pre.assign(U, 0.0);
                    for (int u = 0; u < U; ++u)
                        for (int ci = 0; ci < c.cin; ++ci)
                            for (int ph = 0; ph < R; ++ph) {
                                double f = 0;
                                for (int j = 0; j <= 2 * R; ++j) f += (double)tap[j] * P(ci, u * R + ph - R + j);
                                pre[u] += (double)W(co, ci, ph) * f;
                            }
                } else {
                    std::vector<double> z(full, 0.0);
                    for (int t = 0; t < full; ++t)
                        for (int ci = 0; ci < c.cin; ++ci) z[t] += (double)W(co, ci, t % R) * P(ci, t / R);
                    pre.assign(out_len, 0.0);
                    for (int t = 0; t < out_len; ++t)
                        for (int j = 0; j <= 2 * R; ++j) {
                            const int q = t - R + j;
                            if (q >= 0 && q < full) pre[t] += (double)tap[j] * z[q];
                        }
                }
                for (int t = 0; t < out_len; ++t) {
                    double v = pre[t] + bias[co];
                    if (t >= valid) v = 0;
                    const size_t o = ((size_t)b * c.cout + co) * out_len + t;
                    if (c.res1) v = (v + r1[o]) * 0.7;
                    if (c.film) v = fm[(size_t)b * 2 * c.cout + co] * v + fm[(size_t)b * 2 * c.cout + c.cout + co];
                    if (c.res2) v = (v + r2[o]) * 0.5;
                    ref[o] = v;
                }
            }
        }
        double rn = 0;
        for (double v : ref) rn += v * v;
        // ---- logical weights in the FIR kernels' orders (include/ouhip.h), packed
        int mrows, keff;
        std::vector<float> wl;
        if (down) {
            mrows = c.cout, keff = c.cin * R;
            wl.assign((size_t)mrows * keff, 0.f);
            for (int co = 0; co < c.cout; ++co)
                for (int ci = 0; ci < c.cin; ++ci)
                    for (int ph = 0; ph < R; ++ph)
                        wl[(size_t)co * keff + ci * R + ph] = W(co, ci, ph);
        } else {
            const int P = 32 / R;
            mrows = (c.cout + P - 1) / P * 32, keff = c.cin;
            wl.assign((size_t)mrows * keff, 0.f);
            for (int co = 0; co < c.cout; ++co)
                for (int ph = 0; ph < R; ++ph)
                    for (int ci = 0; ci < c.cin; ++ci)
                        wl[(size_t)(32 * (co / P) + (co % P) * R + ph) * keff + ci] = W(co, ci, ph);
        }
        std::vector<float> packed(ou_conv_packed_size(mrows, keff, 1, 0));
        float unscale = 0.f;
        ou_conv_pack_split_nat(wl.data(), mrows, keff, 1, packed.data(), &unscale);
        const int rows = out_len + 3;
        for (int prec = 1; prec <= 2; ++prec)
            for (int shape = 0; shape < kNumFTiles; ++shape) {
                if (prec == 2 && shape != 2) continue;
                std::vector<float> y(ref.size(), 1e30f);
                std::vector<uint16_t> img;
                ou_conv_desc d{};
                d.x = x.data(); d.x_bstride = (int64_t)c.cin * c.T; d.x_cstride = c.T;
                d.cin = c.cin; d.in_len = c.T; d.frame = down ? R : 1; d.slope = slope;
                d.w = packed.data(); d.m = down ? c.cout : c.cout * R; d.kt = 1; d.pad = 0;
                d.n_frames = U; d.batch = c.B; d.y = y.data(); d.y_bstride = (int64_t)c.cout * out_len;
                d.y_cstride = out_len; d.rout = down ? 1 : -R; d.out_len = out_len; d.valid_len = valid;
                d.bias = bias.data();
                d.res1 = c.res1 ? r1.data() : nullptr; d.r1_bstride = d.y_bstride; d.r1_cstride = out_len; d.s1 = 0.7f;
                d.film = c.film ? fm.data() : nullptr; d.film_bstride = 2 * c.cout;
                d.res2 = c.res2 ? r2.data() : nullptr; d.r2_bstride = d.y_bstride; d.r2_cstride = out_len; d.s2 = 0.5f;
                d.prec = prec; d.w_unscale = unscale; d.xs_shift = s;
                d.fir = c.dir; d.fir_taps = tap.data();
                // m-major order on shape 3; the up kernel's early epilogue loads on odd shapes;
                // two chunks in flight on shapes 2 and 6 (down: bias-only layers)
                const bool lean = !c.res1 && !c.res2 && !c.film;
                d.tile = kFirBit | shape | (shape == 3 ? kMajBit : 0) | (!down && shape % 2 ? kFirEarly : 0) |
                         (shape % 4 == 2 && (!down || lean) ? kFirDeep : 0);
                if (down && c.sy && prec == 1) {
                    img.assign((size_t)c.B * (c.cout / 32) * rows * 64, 0x7e00);
                    d.sy = img.data(); d.sy_bstride = (int64_t)(c.cout / 32) * rows * 128; d.sy_rows = rows;
                    d.sy_shift = 6; d.sy_slope = 0.5f;
                }
                const int rc = ou_conv(&d, nullptr);
                if (rc != 0) {
                    std::printf("R %d dir %d shape %d prec %d: launch error %s\n", R, c.dir, shape, prec,
                                ouhip_detail::err_buf());
                    ++bad;
                    continue;
                }
                double en = 0;
                for (size_t i = 0; i < y.size(); ++i) en += (y[i] - ref[i]) * (y[i] - ref[i]);
                const double rel = std::sqrt(en / rn);
                ++n;
                if (!(rel < (prec == 1 ? 2e-6 : 2e-3))) {
                    std::printf("R %d dir %d cin %d cout %d T %d shape %d prec %d: rel err %.3g\n", R, c.dir, c.cin,
                                c.cout, c.T, shape, prec, rel);
                    for (size_t i = 0, k = 0; i < y.size() && k < 4; ++i)
                        if (std::fabs(y[i] - ref[i]) > 1e-3 * std::sqrt(rn / ref.size())) {
                            std::printf("   [%zu] got %.7g want %.7g\n", i, y[i], ref[i]);
                            ++k;
                        }
                    ++bad;
                }
                if (!img.empty()) {   // the split image of prelu(y) 2^-6 beside y
                    int wrong = 0;
                    for (int b = 0; b < c.B; ++b)
                        for (int co = 0; co < c.cout; ++co)
                            for (int t = 0; t < out_len; ++t) {
                                const size_t o = (((size_t)b * (c.cout / 32) + co / 32) * rows + t) * 64 + co % 32;
                                float p = std::ldexp(y[((size_t)b * c.cout + co) * out_len + t], -6);
                                p = p >= 0.f ? p : p * 0.5f;
                                _Float16 hi, lo;
                                std::memcpy(&hi, &img[o], 2);
                                std::memcpy(&lo, &img[o + 32], 2);
                                const double got = (double)hi + (double)lo / 2048.0;
                                wrong += !(std::fabs(got - p) <= std::ldexp(std::fabs(p), -21) + std::ldexp(1.0, -35));
                            }
                    if (wrong) {
                        std::printf("R %d shape %d: %d split-image elements wrong\n", R, shape, wrong);
                        ++bad;
                    }
                }
            }
    }
    std::printf("%s: %d launches checked, %d bad\n", bad ? "FAIL" : "ok", n, bad);
    return bad ? 1 : 0;
}
