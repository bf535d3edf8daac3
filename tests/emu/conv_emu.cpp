// Bounds check of every ou_conv tile configuration on the CPU: the HIP
// source compiled for the host against tests/emu/hip/hip_runtime.h, under
// AddressSanitizer.  Exits nonzero (ASan report / EMU message) on the first
// out-of-bounds global, buffer or LDS access.  See tests/test_emu_bounds.py.
#ifdef OU_EMU_CONV_SRC   // a modified copy of the kernel source (tests/test_emu_kernels.py)
#include OU_EMU_CONV_SRC
#else
#include "../../open_universe_amd/csrc/ou_conv.hip"
#endif

#include <memory>

struct Geom {
    int cout, cin, frame, kt, T, B, rout;
    bool res1, res2, film, scale;
    bool cm = false;   // channel-major output rows (ou_conv_desc.rout < 0)
};

static float* alloc(size_t n)
{
    float* p = (float*)std::malloc(n * sizeof(float));   // exact size: ASan guards both ends
    for (size_t i = 0; i < n; ++i) p[i] = 0.25f;
    return p;
}

// chunk: launch output frames [U / 3, 2 U / 3 + 1) only, reading x up to the
// last sample they need (as engine.conv_desc(rng=...) records it), and check
// that nothing outside those frames' outputs was written
static int run(const Geom& g, int tile, bool chunk = false, int kslices = 1)
{
    const int cin_eff = g.cin * g.frame;
    const int m = g.cout * g.rout;
    const int U = g.rout > 1 ? g.T : (g.T + g.frame - 1) / g.frame;   // frames
    const int out_len = U * g.rout;
    std::vector<float> wl((size_t)m * cin_eff * g.kt, 0.1f);
    const int64_t np = ou_conv_packed_size(m, cin_eff, g.kt, 0);
    float* w = alloc(np);
    float unscale = 1.f;
    const bool split = tile & 2048;   // split-f16 form (d.prec = 1; 2 with bit 12: f16)
    if (split)
        ou_conv_pack_split(wl.data(), m, cin_eff, g.kt, w, &unscale);
    else
        ou_conv_pack(wl.data(), m, cin_eff, g.kt, 0, w);
    float* x = alloc((size_t)g.B * g.cin * g.T);
    float* y = alloc((size_t)g.B * g.cout * out_len);
    float* bias = alloc(g.cout);
    float* r1 = g.res1 ? alloc((size_t)g.B * g.cout * out_len) : nullptr;
    float* r2 = g.res2 ? alloc((size_t)g.B * g.cout * out_len) : nullptr;
    float* fm = g.film ? alloc((size_t)g.B * 2 * g.cout) : nullptr;
    float* sc = g.scale ? alloc(g.B) : nullptr;
    ou_conv_desc d{};
    d.x = x; d.x_bstride = (int64_t)g.cin * g.T; d.x_cstride = g.T;
    d.cin = g.cin; d.in_len = g.T; d.frame = g.frame; d.shift = 0; d.in_scale = sc; d.slope = 0.25f;
    d.w = w; d.m = m; d.kt = g.kt; d.pad = (g.kt - 1) / 2; d.cc = 0;
    d.n_frames = U; d.batch = g.B;
    d.y = y; d.y_bstride = (int64_t)g.cout * out_len; d.y_cstride = out_len;
    d.rout = g.cm ? -g.rout : g.rout; d.out_len = out_len; d.valid_len = out_len - 3;
    d.bias = bias;
    d.res1 = r1; d.r1_bstride = d.y_bstride; d.r1_cstride = d.y_cstride; d.s1 = 0.7f;
    d.film = fm; d.film_bstride = 2 * g.cout;
    d.res2 = r2; d.r2_bstride = d.y_bstride; d.r2_cstride = d.y_cstride; d.s2 = 0.5f;
    d.tile = tile & ~(2048 | 4096);
    d.prec = split ? ((tile & 4096) ? 2 : 1) : 0;
    d.w_unscale = unscale;
    float* ksws = nullptr;   // K-slice partial sums (register-streamed slices: tile bits 12-13)
    if (kslices > 1) {
        d.tile |= (kslices == 2 ? 1 : kslices == 4 ? 2 : 3) << 12;
        const int64_t n = (int64_t)((U + 31) / 32 + 2) * ((m + 31) / 32 + 4) * g.B * kslices * 4 * 1024;
        ksws = alloc((size_t)n);
        d.ks_ws = ksws;
        d.ks_ws_bytes = n * 4;
    }
    int a = 0, bnd = U;
    if (chunk) {
        a = U / 3;
        bnd = std::min(U, 2 * U / 3 + 1);
        d.f0 = a;
        d.n_frames = bnd - a;
        d.in_len = std::max(1, std::min(d.in_len, (bnd - d.pad + g.kt - 1) * g.frame + d.shift));
    }
    int rc = ou_conv(&d, nullptr);
    if (rc == 0 && chunk) {
        for (int b = 0; b < g.B; ++b)
            for (int c = 0; c < g.cout; ++c)
                for (int t = 0; t < out_len; ++t) {
                    const bool mine = t >= a * g.rout && t < bnd * g.rout;
                    if (!mine && y[((size_t)b * g.cout + c) * out_len + t] != 0.25f) {
                        std::fprintf(stderr, "EMU: chunk [%d, %d) wrote output sample %d (b %d c %d)\n", a, bnd, t, b, c);
                        rc = 3;
                        b = g.B; c = g.cout;
                        break;
                    }
                }
    }
    for (float* p : {w, x, y, bias, r1, r2, fm, sc, ksws}) std::free(p);
    return rc;
}

int main(int argc, char** argv)
{
    const Geom geoms[] = {
        {64, 64, 1, 3, 517, 2, 1, false, false, false, false},
        {64, 64, 1, 5, 517, 2, 1, true, false, false, false},
        {32, 32, 1, 3, 1000, 1, 1, true, false, false, true},
        {96, 40, 1, 1, 77, 2, 1, false, true, true, false},
        {512, 256, 1, 3, 33, 2, 1, true, false, true, false},
        {64, 32, 2, 3, 300, 2, 1, false, false, false, false},
        {48, 24, 5, 3, 203, 1, 1, false, false, false, false},
        {642, 1, 160, 4, 1600, 1, 1, false, false, false, false},   // STFT as a framed GEMM
        {128, 256, 1, 3, 41, 2, 4, true, false, false, false},      // transposed conv, 4 phases
        {160, 96, 1, 3, 67, 1, 5, false, false, false, false},      // M = 800, partial m-groups
        {128, 256, 1, 3, 41, 2, 4, true, false, false, false, true},  // channel-major rows: 16-B epilogue
        {32, 64, 1, 3, 301, 1, 2, true, true, true, false, true},     // channel-major, 2 phases: 8-B epilogue
        // register-streamed kernel (tile bit 14) shapes, run with its tiles
        // only (kFirstRsGeom on): ragged 16-channel up
        // conv (3 steps < 4 K waves: the b31c724 fault), 1 step, deep k3 / k5,
        // frame views with and without the folded FIR, the conditioner's
        // st_convs whose windows exceed LDS (K chunked by phases / channels)
        {32, 16, 1, 3, 301, 1, 2, true, false, false, false},
        {16, 16, 1, 1, 100, 2, 1, false, false, false, false},
        {512, 512, 1, 3, 41, 1, 1, false, false, false, false},
        {256, 256, 1, 5, 70, 1, 1, true, true, true, false},
        {256, 128, 4, 3, 148, 1, 1, false, false, false, false},
        {512, 256, 5, 1, 205, 1, 1, false, false, false, false},
        {512, 32, 160, 1, 1760, 1, 1, true, false, false, false},
        {512, 64, 80, 1, 880, 1, 1, false, false, false, false},
        {512, 128, 20, 1, 220, 1, 1, false, false, false, false},
    };
    const int only = argc > 1 ? std::atoi(argv[1]) : -1;
    int n = 0;
    constexpr int kFirstRsGeom = 12;   // geometries from here on: register-streamed tiles only
    int nrs = 0, nchunk = 0, nks = 0;
    const bool rs_only = std::getenv("OUHIP_EMU_RS_ONLY") != nullptr;   // register-streamed tiles only
    for (int gi = 0; gi < (int)(sizeof(geoms) / sizeof(geoms[0])); ++gi) {
        if (only >= 0 && gi != only) continue;
        const Geom& g = geoms[gi];
        for (int t = 0; t < std::max(ou_conv_num_tiles(), 16); ++t) {
            // 3: warp-specialised, 4: split-f16, 5: f16, 6 / 7: register-streamed
            // kernel (tile bit 14) split-f16 / f16
            for (int tpw = 0; tpw < 8; ++tpw) {
                if (tpw == 3 && g.rout != 1) continue;   // warp-specialised: plain convs only
                if (tpw >= 6 && (t >= 16 || g.cin % 16)) continue;   // register-streamed: cin % 16 == 0
                if (tpw < 6 && (rs_only || gi >= kFirstRsGeom || t >= ou_conv_num_tiles() || !ou_conv_tile_ok(g.kt, t)))
                    continue;
                const int v = tpw >= 6 ? (2048 | (1 << 14)) : tpw >= 4 ? 2048 : tpw == 3 ? 1024 : tpw << 8;
                if (!ou_conv_tile_ok(g.kt, tpw >= 6 ? (t | (1 << 14)) : (t | v))) continue;
                if (std::getenv("OUHIP_EMU_VERBOSE")) std::fprintf(stderr, "geom %d tile %d tpw %d\n", gi, t, tpw);
                const int rc = run(g, t | v | ((tpw == 5 || tpw == 7) ? 4096 : 0));
                if (rc == -2 && tpw == 3) continue;   // warp-specialised form refused for this geometry
                if (rc != 0 && tpw >= 6) continue;    // register-streamed form refused (window / LDS)
                if (rc != 0) {
                    std::fprintf(stderr, "geom %d tile %d tpw %d: ou_conv returned %d\n", gi, t, tpw, rc);
                    return 2;
                }
                ++n;
                nrs += tpw >= 6;
                // the same tile on a frame range of the op (one-tile workgroups)
                if (tpw == 0 || tpw >= 4) {
                    const int rc2 = run(g, t | v | ((tpw == 5 || tpw == 7) ? 4096 : 0), true);
                    if (rc2 != 0) {
                        std::fprintf(stderr, "geom %d tile %d tpw %d (frame range): ou_conv returned %d\n", gi, t, tpw, rc2);
                        return 2;
                    }
                    ++n;
                    ++nchunk;
                }
                // register-streamed K slices (K-chunked windows: the st_convs);
                // refused where the chunks are fewer than the slices
                if (tpw == 6)
                    for (int ksl : {2, 4, 8})
                        for (bool ch : {false, true}) {
                            const int rc3 = run(g, t | v, ch, ksl);
                            if (rc3 == -2) continue;
                            if (rc3 != 0) {
                                std::fprintf(stderr, "geom %d tile %d: %d K slices%s: ou_conv returned %d\n", gi, t, ksl,
                                             ch ? " (frame range)" : "", rc3);
                                return 2;
                            }
                            ++n;
                            ++nrs;
                            ++nks;
                        }
            }
        }
    }
    std::printf("ok: %d launches bounds-checked (%d register-streamed, %d of them K-sliced, %d on frame ranges)\n", n,
                nrs, nks, nchunk);
    return 0;
}
