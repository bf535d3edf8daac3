// Numerics of the split-image path on the CPU (fiber emulator, OU_EMU_FIBERS):
//  1. a producer conv (chunked / register-streamed / split-image kernels)
//     with ou_conv_desc.sy set stores, beside y, the split image of
//     prelu(y) * 2^-s -- checked element by element (hi + lo 2^-11 within
//     2^-21 relative of the f32 value, zero rows never written);
//  2. the split-image kernel (tile bit 15) reading a host-built split image
//     matches a double-precision evaluation of the ou_conv_desc formula for
//     every NR shape, frame views, ragged lengths, residuals / FiLM and
//     transposed (channel-major) outputs.
// Prints one line per failure and exits 1.
#include "../../open_universe_amd/csrc/ou_conv.hip"

#include <cmath>

static uint32_t g_seed = 777;
static float rnd()
{
    g_seed = g_seed * 1664525u + 1013904223u;
    return ((g_seed >> 8) & 0xffff) / 32768.0f - 1.0f;
}

static float h2f(uint16_t u)
{
    _Float16 h;
    std::memcpy(&h, &u, 2);
    return (float)h;
}

// host split image of prelu(x) * 2^-s: [b][c / 32][t][hi | lo][c % 32]
static void make_split(const std::vector<float>& x, int B, int C, int T, int rows, float slope, int s,
                       std::vector<uint16_t>& img)
{
    img.assign((size_t)B * (C / 32) * rows * 64, 0x7e00);   // NaN halves where nothing is written
    const float sc = std::ldexp(1.f, -s);
    for (int b = 0; b < B; ++b)
        for (int c = 0; c < C; ++c)
            for (int t = 0; t < T; ++t) {
                float p = x[((size_t)b * C + c) * T + t] * sc;
                p = p >= 0.f ? p : p * slope;
                const _Float16 hi = (_Float16)p, lo = (_Float16)((p - (float)hi) * 2048.f);
                const size_t o = (((size_t)b * (C / 32) + c / 32) * rows + t) * 64 + (c % 32);
                std::memcpy(&img[o], &hi, 2);
                std::memcpy(&img[o + 32], &lo, 2);
            }
}

struct Geom {
    int cout, cin, frame, kt, T, B, rout;
    bool res1, res2, film;
    bool cm;
};

int main(int argc, char** argv)
{
    const int only = argc > 1 ? std::atoi(argv[1]) : -1;
    int bad = 0, n = 0;
    // ---- 2. consumer: the split-image kernel against the formula
    const Geom geoms[] = {
        {64, 64, 1, 3, 133, 2, 1, true, false, false, false},
        {32, 96, 1, 5, 70, 1, 1, false, true, true, false},
        {96, 32, 1, 1, 41, 2, 1, true, false, false, false},
        {64, 32, 5, 3, 103, 1, 1, false, false, false, false},   // frame view, rate 5
        {32, 64, 4, 3, 97, 2, 1, true, false, true, false},      // frame view, rate 4
        {128, 64, 1, 3, 29, 1, 4, true, false, false, true},     // transposed, channel-major rows
        {64, 32, 1, 3, 45, 1, 1, false, false, false, false},    // one chunk: three zero-chunk waves
    };
    for (int gi = 0; gi < (int)(sizeof(geoms) / sizeof(geoms[0])); ++gi) {
        if (only >= 0 && gi != only) continue;
        const Geom& g = geoms[gi];
        const int cin_eff = g.cin * g.frame, m = g.cout * g.rout;
        const int U = g.rout > 1 ? g.T : (g.T + g.frame - 1) / g.frame;
        const int out_len = U * g.rout, valid = out_len - 2, pad = (g.kt - 1) / 2;
        const float slope = 0.25f;
        const int s = 5 + gi % 3;   // staging exponent
        std::vector<float> wl((size_t)m * cin_eff * g.kt), x((size_t)g.B * g.cin * g.T), bias(g.cout),
            r1((size_t)g.B * g.cout * out_len), r2(r1.size()), fm((size_t)g.B * 2 * g.cout);
        for (auto* v : {&wl, &x, &bias, &r1, &r2, &fm})
            for (auto& e : *v) e = rnd();
        // the kernel's logical weight order is the phase-major frame view (ph * cin + ci)
        std::vector<float> wpm(wl.size());
        for (int mm = 0; mm < m; ++mm)
            for (int ci = 0; ci < g.cin; ++ci)
                for (int p = 0; p < g.frame; ++p)
                    for (int k = 0; k < g.kt; ++k)
                        wpm[((size_t)mm * cin_eff + p * g.cin + ci) * g.kt + k] =
                            wl[((size_t)mm * cin_eff + ci * g.frame + p) * g.kt + k];
        std::vector<float> packed(ou_conv_packed_size(m, cin_eff, g.kt, 0));
        float unscale = 0.f;
        ou_conv_pack_split_nat(wpm.data(), m, cin_eff, g.kt, packed.data(), &unscale);
        const int rows = g.T + 3;
        std::vector<uint16_t> img;
        make_split(x, g.B, g.cin, g.T, rows, slope, s, img);
        std::vector<double> ref((size_t)g.B * g.cout * out_len, 0.0);
        for (int b = 0; b < g.B; ++b)
            for (int mm = 0; mm < m; ++mm) {
                const int ph = g.cm ? mm % g.rout : mm / g.cout, co = g.cm ? mm / g.rout : mm % g.cout;
                for (int u = 0; u < U; ++u) {
                    double acc = 0.0;
                    for (int c = 0; c < cin_eff; ++c)
                        for (int k = 0; k < g.kt; ++k) {
                            const int fu = u + k - pad;
                            if (fu < 0 || fu >= U) continue;
                            const int ci = c / g.frame, fph = c % g.frame;   // logical order ci * R + ph
                            const int pos = fu * g.frame + fph;
                            if (pos >= g.T) continue;
                            double xv = x[((size_t)b * g.cin + ci) * g.T + pos];
                            if (xv < 0) xv *= slope;
                            acc += (double)wl[((size_t)mm * cin_eff + c) * g.kt + k] * xv;
                        }
                    const int t = u * g.rout + ph;
                    double v = acc + bias[co];
                    if (t >= valid) v = 0;
                    const size_t o = ((size_t)b * g.cout + co) * out_len + t;
                    if (g.res1) v = (v + r1[o]) * 0.7;
                    if (g.film) v = fm[(size_t)b * 2 * g.cout + co] * v + fm[(size_t)b * 2 * g.cout + g.cout + co];
                    if (g.res2) v = (v + r2[o]) * 0.5;
                    ref[o] = v;
                }
            }
        double rn = 0;
        for (double v : ref) rn += v * v;
        for (int shape = 0; shape < 6; ++shape) {
            std::vector<float> y(ref.size(), 1e30f);
            ou_conv_desc d{};
            d.x = x.data(); d.x_bstride = (int64_t)g.cin * g.T; d.x_cstride = g.T;   // unused by the kernel
            d.cin = g.cin; d.in_len = g.T; d.frame = g.frame; d.slope = 0.5f;       // slope unused: in the image
            d.w = packed.data(); d.m = m; d.kt = g.kt; d.pad = pad;
            d.n_frames = U; d.batch = g.B; d.y = y.data(); d.y_bstride = (int64_t)g.cout * out_len;
            d.y_cstride = out_len; d.rout = g.cm ? -g.rout : g.rout; d.out_len = out_len; d.valid_len = valid;
            d.bias = bias.data();
            d.res1 = g.res1 ? r1.data() : nullptr; d.r1_bstride = d.y_bstride; d.r1_cstride = out_len; d.s1 = 0.7f;
            d.film = g.film ? fm.data() : nullptr; d.film_bstride = 2 * g.cout;
            d.res2 = g.res2 ? r2.data() : nullptr; d.r2_bstride = d.y_bstride; d.r2_cstride = out_len; d.s2 = 0.5f;
            d.prec = 1; d.w_unscale = unscale;
            d.xs = img.data(); d.xs_bstride = (int64_t)(g.cin / 32) * rows * 128; d.xs_rows = rows; d.xs_shift = s;
            d.tile = (1 << 15) | shape;
            const int rc = ou_conv(&d, nullptr);
            if (rc != 0) {
                std::printf("consumer geom %d shape %d: launch error %s\n", gi, shape, ouhip_detail::err_buf());
                ++bad;
                continue;
            }
            double en = 0;
            for (size_t i = 0; i < y.size(); ++i) en += (y[i] - ref[i]) * (y[i] - ref[i]);
            const double rel = std::sqrt(en / rn);
            ++n;
            if (!(rel < 1e-5)) {
                std::printf("consumer geom %d shape %d: rel err %.3g\n", gi, shape, rel);
                ++bad;
            }
        }
    }
    // ---- 1. producers: y and its split image, for every kernel family
    if (only < 0 || only == 100) {
        const int C = 64, T = 77, B = 2, kt = 3, s = 6;
        const float yslope = 0.125f;
        std::vector<float> wl((size_t)C * C * kt), x((size_t)B * C * T), r1(x.size());
        for (auto* v : {&wl, &x, &r1})
            for (auto& e : *v) e = rnd();
        std::vector<float> pk(ou_conv_packed_size(C, C, kt, 0)), pkn(pk.size());
        float un = 0.f, unn = 0.f;
        ou_conv_pack_split(wl.data(), C, C, kt, pk.data(), &un);
        ou_conv_pack_split_nat(wl.data(), C, C, kt, pkn.data(), &unn);
        const int rows = T + 5;
        std::vector<uint16_t> xin;
        make_split(x, B, C, T, rows, 0.25f, 6, xin);
        std::vector<float> ksws(1 << 20);
        // tiles: chunked 11, chunked 11 in 2 K slices, register-streamed 0 and 0 in 2 K slices, split-image 1
        const int tiles[] = {11, 11 | (1 << 12), (1 << 14) | 0, (1 << 14) | (1 << 12), (1 << 15) | 1};
        for (int tile : tiles) {
            std::vector<float> y((size_t)B * C * T, 1e30f);
            std::vector<uint16_t> img((size_t)B * (C / 32) * rows * 64, 0x7e00);
            ou_conv_desc d{};
            d.x = x.data(); d.x_bstride = (int64_t)C * T; d.x_cstride = T;
            d.cin = C; d.in_len = T; d.frame = 1; d.slope = 0.25f;
            d.w = (tile & (1 << 15)) ? pkn.data() : pk.data(); d.w_unscale = (tile & (1 << 15)) ? unn : un;
            d.m = C; d.kt = kt; d.pad = 1; d.n_frames = T; d.batch = B;
            d.y = y.data(); d.y_bstride = (int64_t)C * T; d.y_cstride = T; d.rout = 1; d.out_len = T;
            d.valid_len = T - 3; d.res1 = r1.data(); d.r1_bstride = (int64_t)C * T; d.r1_cstride = T; d.s1 = 0.7f;
            d.prec = 1; d.tile = tile; d.ks_ws = ksws.data(); d.ks_ws_bytes = (int64_t)ksws.size() * 4;
            if (tile & (1 << 15)) {
                d.xs = xin.data(); d.xs_bstride = (int64_t)(C / 32) * rows * 128; d.xs_rows = rows; d.xs_shift = 6;
            }
            d.sy = img.data(); d.sy_bstride = (int64_t)(C / 32) * rows * 128; d.sy_rows = rows; d.sy_shift = s;
            d.sy_slope = yslope;
            const int rc = ou_conv(&d, nullptr);
            if (rc == -2 && (tile & (3 << 12))) continue;   // more K slices than K chunks
            if (rc != 0) {
                std::printf("producer tile 0x%x: launch error %s\n", tile, ouhip_detail::err_buf());
                ++bad;
                continue;
            }
            ++n;
            int wrong = 0;
            for (int b = 0; b < B; ++b)
                for (int c = 0; c < C; ++c)
                    for (int t = 0; t < rows; ++t) {
                        const size_t o = (((size_t)b * (C / 32) + c / 32) * rows + t) * 64 + (c % 32);
                        if (t >= T) {   // never written
                            wrong += img[o] != 0x7e00 || img[o + 32] != 0x7e00;
                            continue;
                        }
                        float p = std::ldexp(y[((size_t)b * C + c) * T + t], -s);
                        p = p >= 0.f ? p : p * yslope;
                        const double got = (double)h2f(img[o]) + (double)h2f(img[o + 32]) / 2048.0;
                        const bool w_ = !(std::fabs(got - p) <= std::ldexp(std::fabs(p), -21) + std::ldexp(1.0, -35));
                        if (w_ && wrong < 4)
                            std::printf("   b %d c %d t %d: got %.9g want %.9g (y %.9g)\n", b, c, t, got, p,
                                        y[((size_t)b * C + c) * T + t]);
                        wrong += w_;
                    }
            if (wrong) {
                std::printf("producer tile 0x%x: %d split-image elements wrong\n", tile, wrong);
                ++bad;
            }
        }
    }
    std::printf("%s: %d launches checked, %d bad\n", bad ? "FAIL" : "ok", n, bad);
    return bad ? 1 : 0;
}
