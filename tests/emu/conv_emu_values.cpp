// Numerics of every ou_conv tile configuration on the CPU (fiber emulator,
// tests/emu/hip/hip_runtime.h with OU_EMU_FIBERS): each launch is compared
// with a double-precision evaluation of the ou_conv_desc formula in
// include/ouhip.h.  Prints one line per failing (geometry, tile) and exits 1.
#include "../../open_universe_amd/csrc/ou_conv.hip"

#include <cmath>

struct Geom {
    int cout, cin, frame, kt, T, B, rout;
    bool res1, res2, film, scale;
    bool cm = false;   // channel-major output rows (ou_conv_desc.rout < 0)
};

static uint32_t g_seed = 12345;
static float rnd()
{
    g_seed = g_seed * 1664525u + 1013904223u;
    return ((g_seed >> 8) & 0xffff) / 32768.0f - 1.0f;
}

int main(int argc, char** argv)
{
    const Geom geoms[] = {
        {64, 64, 1, 3, 133, 2, 1, false, false, false, false},
        {64, 64, 1, 3, 517, 2, 1, false, false, false, false},   // test_same_conv_layer[conv3-3-1-517]
        {64, 64, 1, 5, 70, 2, 1, true, false, false, false},
        {32, 32, 1, 3, 300, 1, 1, true, false, false, true},
        {96, 40, 1, 1, 41, 2, 1, false, true, true, false},
        {64, 32, 2, 3, 100, 2, 1, false, false, false, false},
        {48, 24, 5, 3, 103, 1, 1, false, false, false, false},
        {64, 48, 1, 3, 29, 2, 4, true, false, false, false},   // transposed conv, 4 phases
        {64, 48, 1, 3, 29, 2, 4, true, false, false, false, true},   // channel-major rows: 16-B epilogue
        {32, 64, 1, 3, 45, 1, 2, true, true, true, false, true},     // channel-major, 2 phases: 8-B epilogue
        {24, 32, 1, 1, 37, 2, 5, true, false, false, false, true},   // channel-major, 5 phases: scalar epilogue
        {16, 32, 1, 3, 27, 2, 8, true, true, false, false, true},    // channel-major, 8 phases: two 16-B groups a channel
    };
    const int only = argc > 1 ? std::atoi(argv[1]) : -1;
    int bad = 0, n = 0;
    for (int gi = 0; gi < (int)(sizeof(geoms) / sizeof(geoms[0])); ++gi) {
        if (only >= 0 && gi != only) continue;
        const Geom& g = geoms[gi];
        const int cin_eff = g.cin * g.frame, m = g.cout * g.rout;
        const int U = g.rout > 1 ? g.T : (g.T + g.frame - 1) / g.frame;
        const int out_len = U * g.rout, valid = out_len - 2, pad = (g.kt - 1) / 2;
        std::vector<float> wl((size_t)m * cin_eff * g.kt), x((size_t)g.B * g.cin * g.T), bias(g.cout),
            r1((size_t)g.B * g.cout * out_len), r2(r1.size()), fm((size_t)g.B * 2 * g.cout), sc(g.B);
        for (auto* v : {&wl, &x, &bias, &r1, &r2, &fm, &sc})
            for (auto& e : *v) e = rnd();
        std::vector<float> packed(ou_conv_packed_size(m, cin_eff, g.kt, 0)), packed_s(packed.size());
        std::vector<float> ksws(4 << 20);   // K-slice partial sums
        ou_conv_pack(wl.data(), m, cin_eff, g.kt, 0, packed.data());
        float unscale = 0.f;
        ou_conv_pack_split(wl.data(), m, cin_eff, g.kt, packed_s.data(), &unscale);
        // reference
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
                            const int ci = c % g.cin, fph = c / g.cin;
                            const int pos = fu * g.frame + fph;
                            if (pos >= g.T) continue;
                            double xv = x[((size_t)b * g.cin + ci) * g.T + pos] * (g.scale ? sc[b] : 1.0f);
                            if (xv < 0) xv *= 0.25;
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
        for (int t = 0; t < ou_conv_num_tiles(); ++t) {
            if (!ou_conv_tile_ok(g.kt, t)) continue;
            // 3: warp-specialised, 4: split-f16, 5: f32 in 2 K slices, 6: split-f16 in 4 K slices,
            // 7: f16 operands, 8: f16 in 2 K slices, 9: f16 in 4 K slices,
            // 10: register-streamed kernel (tile bit 14), split-f16
            for (int tpw = 0; tpw < 11; ++tpw) {
                if (tpw == 3 && g.rout != 1) continue;   // warp-specialised: plain convs only
                if (tpw == 10 ? (t >= 6 || g.cin % 16 || !ou_conv_tile_ok(g.kt, t | (1 << 14)))
                              : !ou_conv_tile_ok(g.kt, t | (tpw >= 6 || tpw == 4 ? 2048 : tpw == 3 ? 1024
                                                                                : tpw == 5 ? 0 : tpw << 8)))
                    continue;
                std::vector<float> y(ref.size(), 1e30f);
                ou_conv_desc d{};
                d.x = x.data(); d.x_bstride = (int64_t)g.cin * g.T; d.x_cstride = g.T;
                d.cin = g.cin; d.in_len = g.T; d.frame = g.frame; d.in_scale = g.scale ? sc.data() : nullptr;
                d.slope = 0.25f; d.w = packed.data(); d.m = m; d.kt = g.kt; d.pad = pad;
                d.n_frames = U; d.batch = g.B; d.y = y.data(); d.y_bstride = (int64_t)g.cout * out_len;
                d.y_cstride = out_len; d.rout = g.cm ? -g.rout : g.rout; d.out_len = out_len; d.valid_len = valid;
                d.bias = bias.data();
                d.res1 = g.res1 ? r1.data() : nullptr; d.r1_bstride = d.y_bstride; d.r1_cstride = out_len; d.s1 = 0.7f;
                d.film = g.film ? fm.data() : nullptr; d.film_bstride = 2 * g.cout;
                d.res2 = g.res2 ? r2.data() : nullptr; d.r2_bstride = d.y_bstride; d.r2_cstride = out_len; d.s2 = 0.5f;
                d.tile = t | (tpw == 10 ? 1 << 14 : tpw == 4 || tpw == 7 ? 0 : tpw == 5 || tpw == 8 ? 1 << 12
                                                    : tpw == 6 || tpw == 9 ? 2 << 12 : tpw == 3 ? 1024 : tpw << 8);
                const bool f16 = tpw >= 7 && tpw <= 9;
                if (tpw == 4 || tpw == 6 || tpw == 10 || f16) {
                    d.prec = f16 ? 2 : 1;
                    d.w = packed_s.data();
                    d.w_unscale = unscale;
                }
                d.ks_ws = ksws.data();
                d.ks_ws_bytes = (int64_t)ksws.size() * 4;
                const int rc_ = ou_conv(&d, nullptr);
                if (rc_ == -2 && tpw >= 5) continue;   // more K slices than chunks
                if (rc_ == -2 && tpw == 3) continue;   // warp-specialised form refused for this geometry
                if (rc_ != 0 && tpw == 10) continue;   // register-streamed form refused (window / LDS)
                if (rc_ != 0) {
                    std::printf("geom %d tile %d tpw %d: launch error\n", gi, t, tpw);
                    ++bad;
                    continue;
                }
                double en = 0;
                for (size_t i = 0; i < y.size(); ++i) en += (y[i] - ref[i]) * (y[i] - ref[i]);
                const double rel = std::sqrt(en / rn);
                ++n;
                // f16 operands: rounded to 11 bits, so neither f32-exact nor wrong
                if (f16 ? !(rel > 1e-6 && rel < 3e-3) : !(rel < 1e-5)) {
                    std::printf("geom %d tile %d tpw %d: rel err %.3g\n", gi, t, tpw, rel);
                    if (std::getenv("OUHIP_EMU_VERBOSE")) {
                        int shown = 0;
                        for (size_t e = 0; e < y.size() && shown < 8; ++e)
                            if (std::fabs(y[e] - ref[e]) > 1e-3 * (1 + std::fabs(ref[e]))) {
                                std::printf("   [b %zu co %zu t %zu] got %g want %g\n", e / ((size_t)g.cout * out_len),
                                            (e / out_len) % g.cout, e % out_len, y[e], ref[e]);
                                ++shown;
                            }
                    }
                    ++bad;
                }
            }
        }
    }
    std::printf("%s: %d launches checked, %d bad\n", bad ? "FAIL" : "ok", n, bad);
    return bad ? 1 : 0;
}
