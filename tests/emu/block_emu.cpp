// Bounds check of the fused ConvBlock kernel (ou_block.hip) on the CPU: the
// HIP source compiled for the host against tests/emu/hip/hip_runtime.h, under
// AddressSanitizer.  Every channel count (32 / 64 / 128), operand precision
// (split-f16, f16), epilogue variant the dispatcher instantiates (FiLM,
// input_cond + FiLM, cond_out, res2, the score ends kEpiIn / kEpiHead, the
// fused rate-change conv kEpiDown) and ragged lengths (shorter than one
// workgroup's frames, not a multiple of them, not a multiple of the rate).
// Every buffer is an exact-size heap block: any out-of-bounds global or LDS
// access aborts with its location.  See tests/test_emu_kernels.py.
#ifdef OU_EMU_BLOCK_SRC   // a modified copy of the kernel source (tests/test_emu_kernels.py)
#include OU_EMU_BLOCK_SRC
#else
#include "../../open_universe_amd/csrc/ou_block.hip"
#endif

#include <string>

namespace {

float* alloc(size_t n, float v = 0.25f)
{
    float* p = (float*)std::malloc((n ? n : 1) * sizeof(float));   // exact size: ASan guards both ends
    for (size_t i = 0; i < n; ++i) p[i] = v;
    return p;
}

void* pack(int m, int C, int kt, float* unscale)
{
    std::vector<float> w((size_t)m * C * kt);
    for (size_t i = 0; i < w.size(); ++i) w[i] = 0.01f * (float)((i * 37) % 17) - 0.08f;
    if (m == C) {   // the block's own convs: ou_block_pack (rows padded to 32 at 48 channels)
        void* out = std::malloc((size_t)ou_block_packed_halves(C, kt) * sizeof(_Float16));
        if (ou_block_pack(w.data(), C, kt, out, unscale) != 0) std::abort();
        return out;
    }
    void* out = std::malloc((size_t)m * C * kt * 2 * sizeof(_Float16));
    if (ou_block_pack_rect(w.data(), m, C, kt, out, unscale) != 0) std::abort();
    return out;
}

struct Case {
    int C, T, B, prec;
    bool film, sc, cond, res2, in, head;
    int rate, down_kt;   // rate 0: no fused rate-change conv
};

// chunk: outputs for frames [f0, f1) only (a third of the signal, aligned
// to the rate), h read over [h0, h1); checks that no y / cond_out / head /
// e element outside the range was written
int run(const Case& c, bool chunk = false)
{
    if (c.rate && c.prec == 0) return 0;   // the fused rate-change conv has split / f16 operands only
    const int C = c.C, T = c.T, B = c.B;
    ou_block_desc d{};
    std::vector<void*> own;
    auto f = [&](size_t n) { float* p = alloc(n); own.push_back(p); return p; };
    float* h = f((size_t)B * C * T);
    float* y = f((size_t)B * C * T);
    d.h = h; d.h_bstride = (int64_t)C * T; d.h_cstride = T;
    d.channels = C; d.length = T; d.batch = B; d.prec = c.prec;
    const int kts[3] = {5, 3, 3};
    for (int i = 0; i < 3; ++i) {
        if (c.prec == 0) {   // f32 operands: ou_block_pack_f32
            std::vector<float> wl((size_t)C * C * kts[i], 0.05f);
            float* wp = (float*)std::malloc((size_t)ou_block_packed_f32(C, kts[i]) * sizeof(float));
            if (ou_block_pack_f32(wl.data(), C, kts[i], wp, &d.w_unscale[i]) != 0) std::abort();
            d.w[i] = wp;
        } else {
            d.w[i] = pack(C, C, kts[i], &d.w_unscale[i]);
        }
        own.push_back((void*)d.w[i]);
        d.bias[i] = f(C);
        d.slope[i] = 0.2f;
    }
    if (c.sc) { d.sc = f((size_t)B * C * T); d.sc_bstride = (int64_t)C * T; d.sc_cstride = T; d.s_sc = 0.7f; }
    if (c.film) { d.film = f((size_t)B * 2 * C); d.film_bstride = 2 * C; }
    if (c.cond) { d.cond_out = f((size_t)B * C * T); d.co_bstride = (int64_t)C * T; d.co_cstride = T; }
    d.y = y; d.y_bstride = (int64_t)C * T; d.y_cstride = T; d.s_res = 0.7f; d.s2 = 0.5f;
    if (c.res2) { d.res2 = f((size_t)B * C * T); d.r2_bstride = (int64_t)C * T; d.r2_cstride = T; }
    int* status = (int*)alloc(1, 0.f);
    own.push_back(status);
    d.status = status;
    if (c.in) {
        d.x = f((size_t)B * T); d.x_bstride = T;
        d.in_scale = f(B); d.w_in = f((size_t)C * 3); d.b_in = f(C);
    }
    if (c.head) {
        ou_head_desc& hd = d.head;
        hd.channels = C; hd.length = T; hd.batch = B; hd.mode = 1;
        hd.slope1 = 0.3f; hd.slope2 = 0.1f;
        hd.w = f((size_t)C * 3); hd.bias = 0.01f; hd.edm = 1;
        hd.w_skip = 0.5f; hd.w_out = 0.4f; hd.s2 = 0.25f; hd.c_score = 0.1f; hd.c_noise = 0.2f; hd.s_next = 0.3f;
        hd.x = f((size_t)B * T); hd.z = f((size_t)B * T); hd.out = f((size_t)B * T);
    }
    if (c.rate) {
        const int TE = (T + c.rate - 1) / c.rate;
        d.w_down = pack(2 * C, C, c.down_kt * c.rate, &d.w_down_unscale);
        own.push_back((void*)d.w_down);
        d.b_down = f(2 * C);
        d.slope_down = 0.15f; d.rate = c.rate; d.down_kt = c.down_kt;
        d.e = f((size_t)B * 2 * C * TE); d.e_bstride = (int64_t)2 * C * TE; d.e_cstride = TE;
    }
    int f0 = 0, f1 = T;
    if (chunk) {
        const int r = c.rate ? c.rate : 1;
        f0 = T / 3 / r * r;
        f1 = std::min(T, (2 * T / 3 + 1 + r - 1) / r * r);
        if (f1 <= f0) f1 = std::min(T, f0 + r);
        d.f0 = f0; d.f1 = f1;
        d.h0 = std::max(0, f0 - 4 - 2 * r); d.h1 = std::min(T, f1 + 4 + 2 * r);
    }
    int rc = ou_block(&d, nullptr);
    if (rc == 0 && chunk) {
        auto check = [&](const float* buf, int rows, int len, int a, int bnd, const char* what) {
            if (!buf) return;
            for (int b = 0; b < B; ++b)
                for (int ch = 0; ch < rows; ++ch)
                    for (int t = 0; t < len; ++t)
                        if ((t < a || t >= bnd) && buf[((size_t)b * rows + ch) * len + t] != 0.25f) {
                            std::fprintf(stderr, "EMU: chunk [%d, %d) wrote %s frame %d\n", a, bnd, what, t);
                            rc = 3;
                            return;
                        }
        };
        if (!c.head) check(y, C, T, f0, f1, "y");
        if (c.cond) check(d.cond_out, C, T, f0, f1, "cond_out");
        if (c.head) check(d.head.out, 1, T, f0, f1, "head out");
        if (c.rate) {
            const int TE = (T + c.rate - 1) / c.rate;
            check(d.e, 2 * C, TE, f0 / c.rate, (f1 + c.rate - 1) / c.rate, "e");
        }
    }
    for (void* p : own) std::free(p);
    return rc;
}

}  // namespace

int main(int argc, char** argv)
{
    std::vector<Case> cases;
    for (int prec : {0, 1, 2})
        for (int C : {32, 64, 128, 48, 96, 192}) {
            const int F = ou_block_frames(C);
            // ragged lengths: shorter than a workgroup, just past one, not a multiple
            for (int T : {7, F + 1, 3 * F - 5}) {
                cases.push_back({C, T, 2, prec, false, false, false, false, false, false, 0, 0});
                cases.push_back({C, T, 2, prec, true, false, false, false, false, false, 0, 0});
                cases.push_back({C, T, 1, prec, true, true, false, false, false, false, 0, 0});
                cases.push_back({C, T, 2, prec, false, false, true, false, false, false, 0, 0});
                cases.push_back({C, T, 1, prec, false, false, false, true, false, false, 0, 0});
                if (C == 32 || C == 48) {   // the score network's ends
                    cases.push_back({C, T, 2, prec, true, false, false, false, true, false, 0, 0});
                    cases.push_back({C, T, 1, prec, false, false, false, false, true, false, 0, 0});
                    cases.push_back({C, T, 2, prec, true, true, false, false, false, true, 0, 0});
                    cases.push_back({C, T, 1, prec, false, false, false, false, false, true, 0, 0});
                }
                if (C == 32) {   // the encoder rate changes
                    for (int kt : {3, 1}) {
                        cases.push_back({C, T, 2, prec, false, false, false, false, false, false, 2, kt});
                        cases.push_back({C, T, 1, prec, true, false, false, false, false, false, 2, kt});
                        cases.push_back({C, T, 2, prec, true, false, false, false, true, false, 2, kt});
                    }
                }
                if (C == 64) {
                    cases.push_back({C, T, 2, prec, false, false, false, false, false, false, 4, 1});
                    cases.push_back({C, T, 1, prec, true, false, false, false, false, false, 4, 1});
                }
            }
        }
    const int only = argc > 1 ? std::atoi(argv[1]) : -1;
    int n = 0;
    for (int i = 0; i < (int)cases.size(); ++i) {
        if (only >= 0 && i != only) continue;
        const Case& c = cases[i];
        if (std::getenv("OUHIP_EMU_VERBOSE"))
            std::fprintf(stderr, "case %d: C %d T %d B %d prec %d film %d sc %d cond %d res2 %d in %d head %d rate %d kt %d\n",
                         i, c.C, c.T, c.B, c.prec, c.film, c.sc, c.cond, c.res2, c.in, c.head, c.rate, c.down_kt);
        for (int chunk = 0; chunk < 2; ++chunk) {
            const int rc = run(c, chunk);
            if (rc != 0) {
                std::fprintf(stderr, "case %d%s: ou_block returned %d: %s\n", i, chunk ? " (frame range)" : "", rc,
                             ouhip_detail::err_buf());
                return 2;
            }
            ++n;
        }
    }
    std::printf("ok: %d fused-block launches bounds-checked\n", n);
    return 0;
}
