// Numerics of the fused ConvBlock kernel (ou_block.hip) on the CPU (fiber
// emulator, tests/emu/hip/hip_runtime.h with OU_EMU_FIBERS): each launch is
// compared with a double-precision evaluation of the ou_block_desc formula
// (include/ouhip.h, blocks.py:393-416), whole-signal and on a frame range
// (f0, f1, h0, h1: only the range is stored and compared).  Channel counts
// 32 / 48 / 64 / 96 / 128 / 192 (48: MFMA rows padded to 64), f32,
// split-f16 and f16 operands, the epilogues FiLM, input_cond + FiLM, cond_out and res2,
// and split images (ou_block_desc.xs: stage 0 copies the producer's image of
// the operand; .sy: the epilogue stores prelu(y) 2^-s for the next conv).
// Prints one line per failing case and exits 1.
#include "../../open_universe_amd/csrc/ou_block.hip"

#include <cmath>

static uint32_t g_seed = 777;
static float rnd()
{
    g_seed = g_seed * 1664525u + 1013904223u;
    return ((g_seed >> 8) & 0xffff) / 32768.0f - 1.0f;
}

struct Case {
    int C, T, prec;
    bool film, sc, cond, res2, chunk;
    bool xs = false, sy = false;
};

// prelu_slope(v) 2^-shift as a split image [C / 32][rows][hi | lo][32] f16
static std::vector<_Float16> split_image(const std::vector<float>& v, int C, int T, int rows, float slope, int shift)
{
    std::vector<_Float16> img((size_t)C / 32 * rows * 64, (_Float16)0.f);
    for (int c = 0; c < C; ++c)
        for (int t = 0; t < T; ++t) {
            float p = std::ldexp(v[(size_t)c * T + t], -shift);
            if (p < 0) p *= slope;
            const _Float16 hi = (_Float16)p;
            const size_t o = ((size_t)(c / 32) * rows + t) * 64 + c % 32;
            img[o] = hi;
            img[o + 32] = (_Float16)((p - (float)hi) * 2048.f);
        }
    return img;
}

// conv over [0, T) with zero padding: out[m][t] = b[m] + sum w[m][c][k] prelu(in[c][t + k - pad])
static void conv_ref(const std::vector<double>& in, const std::vector<float>& w, const std::vector<float>& b, int C,
                     int T, int kt, double slope, std::vector<double>& out)
{
    const int pad = (kt - 1) / 2;
    out.assign((size_t)C * T, 0.0);
    for (int m = 0; m < C; ++m)
        for (int t = 0; t < T; ++t) {
            double acc = b[m];
            for (int c = 0; c < C; ++c)
                for (int k = 0; k < kt; ++k) {
                    const int u = t + k - pad;
                    if (u < 0 || u >= T) continue;
                    double v = in[(size_t)c * T + u];
                    if (v < 0) v *= slope;
                    acc += (double)w[((size_t)m * C + c) * kt + k] * v;
                }
            out[(size_t)m * T + t] = acc;
        }
}

static int run(const Case& cs)
{
    const int C = cs.C, T = cs.T;
    const int kts[3] = {5, 3, 3};
    const float slopes[3] = {0.25f, 0.1f, 0.3f};
    std::vector<float> w[3], bias[3];
    std::vector<std::vector<_Float16>> packed(3);
    std::vector<std::vector<float>> packed32(3);
    ou_block_desc d{};
    for (int i = 0; i < 3; ++i) {
        w[i].resize((size_t)C * C * kts[i]);
        for (auto& e : w[i]) e = rnd() / std::sqrt((float)(C * kts[i]));
        bias[i].resize(C);
        for (auto& e : bias[i]) e = 0.1f * rnd();
        if (cs.prec == 0) {
            packed32[i].resize(ou_block_packed_f32(C, kts[i]));
            if (ou_block_pack_f32(w[i].data(), C, kts[i], packed32[i].data(), &d.w_unscale[i]) != 0) return 10;
            d.w[i] = packed32[i].data();
        } else {
            packed[i].resize(ou_block_packed_halves(C, kts[i]));
            if (ou_block_pack(w[i].data(), C, kts[i], packed[i].data(), &d.w_unscale[i]) != 0) return 10;
            d.w[i] = packed[i].data();
        }
        d.bias[i] = bias[i].data();
        d.slope[i] = slopes[i];
    }
    std::vector<float> h((size_t)C * T), sc((size_t)C * T), film(2 * C), res2((size_t)C * T);
    for (auto* v : {&h, &sc, &film, &res2})
        for (auto& e : *v) e = rnd();
    for (int c = 0; c < C; ++c) film[c] = 1.0f + 0.2f * film[c];   // gamma near 1
    std::vector<float> y((size_t)C * T, 1e30f), co((size_t)C * T, 1e30f);
    int status = 0;
    d.h = h.data(); d.h_bstride = (int64_t)C * T; d.h_cstride = T;
    d.channels = C; d.length = T; d.batch = 1; d.prec = cs.prec;
    if (cs.sc) { d.sc = sc.data(); d.sc_bstride = (int64_t)C * T; d.sc_cstride = T; d.s_sc = 0.7f; }
    if (cs.film) { d.film = film.data(); d.film_bstride = 2 * C; }
    if (cs.cond) { d.cond_out = co.data(); d.co_bstride = (int64_t)C * T; d.co_cstride = T; }
    d.y = y.data(); d.y_bstride = (int64_t)C * T; d.y_cstride = T; d.s_res = 0.7f; d.s2 = 0.5f;
    if (cs.res2) { d.res2 = res2.data(); d.r2_bstride = (int64_t)C * T; d.r2_cstride = T; }
    d.status = &status;
    d.shift[0] = 7; d.shift[1] = 5; d.shift[2] = 6; d.shift[3] = 6;
    const int rows = T + 3, sshift = 9;
    const float sslope = 0.125f;
    std::vector<_Float16> ximg, yimg((size_t)C / 32 * rows * 64, (_Float16)1e4f);
    if (cs.xs) {
        ximg = split_image(h, C, T, rows, slopes[0], d.shift[0]);
        d.xs = (const uint16_t*)ximg.data(); d.xs_bstride = (int64_t)ximg.size() * 2; d.xs_rows = rows;
    }
    if (cs.sy) {
        d.sy = (uint16_t*)yimg.data(); d.sy_bstride = (int64_t)yimg.size() * 2; d.sy_rows = rows;
        d.sy_shift = sshift; d.sy_slope = sslope;
    }
    int f0 = 0, f1 = T;
    if (cs.chunk) {
        f0 = T / 3;
        f1 = 2 * T / 3 + 1;
        d.f0 = f0; d.f1 = f1;
        d.h0 = std::max(0, f0 - 4); d.h1 = std::min(T, f1 + 4);   // exactly what [f0, f1) reads
        for (int c = 0; c < C; ++c)   // h outside [h0, h1) is garbage the kernel must not read
            for (int t = 0; t < T; ++t)
                if (t < d.h0 || t >= d.h1) h[(size_t)c * T + t] = 1e30f;
    }
    // reference (h outside [h0, h1) is not needed by [f0, f1))
    std::vector<double> hd((size_t)C * T), c1, c2, c3;
    for (size_t i = 0; i < hd.size(); ++i) hd[i] = h[i] == 1e30f ? 0.0 : h[i];
    conv_ref(hd, w[0], bias[0], C, T, 5, slopes[0], c1);
    for (int m = 0; m < C; ++m)
        for (int t = 0; t < T; ++t) {
            double& v = c1[(size_t)m * T + t];
            if (cs.sc) v = (v + sc[(size_t)m * T + t]) * 0.7;
            if (cs.film) v = film[m] * v + film[C + m];
        }
    conv_ref(c1, w[1], bias[1], C, T, 3, slopes[1], c2);
    conv_ref(c2, w[2], bias[2], C, T, 3, slopes[2], c3);
    const int rc = ou_block(&d, nullptr);
    if (rc != 0) {
        std::printf("C %d T %d prec %d: launch error %d: %s\n", C, T, cs.prec, rc, ouhip_detail::err_buf());
        return 1;
    }
    double en = 0, rn = 0, ec = 0, rc2 = 0;
    bool outside = false;
    for (int m = 0; m < C; ++m)
        for (int t = 0; t < T; ++t) {
            const size_t o = (size_t)m * T + t;
            if (t < f0 || t >= f1) {
                outside |= y[o] != 1e30f || (cs.cond && co[o] != 1e30f);
                continue;
            }
            double want = (hd[o] + c3[o]) * 0.7;
            if (cs.res2) want = (want + res2[o]) * 0.5;
            en += (y[o] - want) * (y[o] - want);
            rn += want * want;
            if (cs.cond) {
                ec += (co[o] - c1[o]) * (co[o] - c1[o]);
                rc2 += c1[o] * c1[o];
            }
        }
    bool img_bad = false;   // the stored split image: prelu(y) 2^-s element by element, rows >= T untouched
    if (cs.sy)
        for (int c = 0; c < C; ++c)
            for (int t = 0; t < rows; ++t) {
                const size_t o = ((size_t)(c / 32) * rows + t) * 64 + c % 32;
                if (t >= T) {
                    img_bad |= (float)yimg[o] != 1e4f || (float)yimg[o + 32] != 1e4f;
                    continue;
                }
                double p = std::ldexp((double)y[(size_t)c * T + t], -sshift);
                if (p < 0) p *= sslope;
                const double got = (double)yimg[o] + (double)yimg[o + 32] / 2048.0;
                img_bad |= !(std::fabs(got - p) <= std::fabs(p) * std::ldexp(1.0, -21) + std::ldexp(1.0, -35));
            }
    const double rel = std::sqrt(en / rn), relc = cs.cond ? std::sqrt(ec / rc2) : 0.0;
    const double tol = cs.prec == 2 ? 3e-3 : 2e-5;
    if (!(rel < tol) || !(relc < tol) || outside || status || img_bad) {
        std::printf("C %d T %d prec %d film %d sc %d cond %d res2 %d chunk %d xs %d sy %d: rel %.3g cond %.3g "
                    "outside %d status %d image %d\n",
                    C, T, cs.prec, cs.film, cs.sc, cs.cond, cs.res2, cs.chunk, cs.xs, cs.sy, rel, relc, outside,
                    status, img_bad);
        return 1;
    }
    return 0;
}

int main(int argc, char** argv)
{
    std::vector<Case> cases;
    for (int C : {48, 96, 192, 32, 64, 128})
        for (int prec : {0, 1, 2}) {
            const int T = C >= 128 ? 45 : 70;
            cases.push_back({C, T, prec, false, false, false, false, false});
            cases.push_back({C, T, prec, true, true, false, false, false});
            cases.push_back({C, T, prec, false, false, true, false, true});
            cases.push_back({C, T, prec, false, false, false, true, true});
            const bool img = prec == 1 && C % 32 == 0;   // split images: both ends, then input only
            cases.push_back({C, T, prec, true, true, false, false, false, img, img});
            cases.push_back({C, T, prec, false, false, true, false, false, img, false});
        }
    const int only = argc > 1 ? std::atoi(argv[1]) : -1;
    int bad = 0, n = 0;
    for (int i = 0; i < (int)cases.size(); ++i) {
        if (only >= 0 && i / 18 != only) continue;   // argv: channel-count group (18 cases each)
        bad += run(cases[i]);
        ++n;
    }
    std::printf("%s: %d block launches checked, %d bad\n", bad ? "FAIL" : "ok", n, bad);
    return bad ? 1 : 0;
}
