// Replay the conv descriptors of a recorded enhance program (dump from
// tests/emu/dump_plan_convs.py) through the bounds emulator, every tile shape
// x tiles-per-workgroup, with every buffer an exact-size heap block (ASan).
#include "../../open_universe_amd/csrc/ou_conv.hip"

#include <fstream>
#include <sstream>
#include <string>

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    std::ifstream in(argv[1]);
    std::vector<char*> bufs;
    std::vector<size_t> sizes;
    std::string line;
    int nconv = 0, nl = 0;
    std::vector<std::string> convs;
    while (std::getline(in, line)) {
        std::istringstream ss(line);
        std::string tag;
        ss >> tag;
        if (tag == "BUF") {
            int id;
            size_t n;
            ss >> id >> n;
            if ((int)bufs.size() <= id) bufs.resize(id + 1), sizes.resize(id + 1);
            bufs[id] = (char*)std::calloc(n ? n : 1, 1);
            sizes[id] = n;
        } else if (tag == "CONV") {
            convs.push_back(line.substr(5));
        }
    }
    auto ptr = [&](long b, long off) -> float* { return b < 0 ? nullptr : (float*)(bufs[b] + off); };
    const int only = argc > 2 ? std::atoi(argv[2]) : -1;
    int shard = 0, nshards = 1;   // OUHIP_EMU_SHARD="i/n": descriptors ci % n == i
    if (const char* s = std::getenv("OUHIP_EMU_SHARD")) std::sscanf(s, "%d/%d", &shard, &nshards);
    for (size_t ci = 0; ci < convs.size(); ++ci) {
        if (only >= 0 && (int)ci != only) continue;
        if ((int)(ci % nshards) != shard) continue;
        std::istringstream ss(convs[ci]);
        long xb, xo, ib, io, wb, wo, yb, yo, bb, bo, r1b, r1o, fb, fo, r2b, r2o;
        ou_conv_desc d{};
        long long xbs, xcs, ybs, ycs, r1bs, r1cs, fbs, r2bs, r2cs;
        ss >> xb >> xo >> xbs >> xcs >> d.cin >> d.in_len >> d.frame >> d.shift >> ib >> io >> d.slope >> wb >> wo >>
            d.m >> d.kt >> d.pad >> d.cc >> d.n_frames >> d.batch >> yb >> yo >> ybs >> ycs >> d.rout >> d.out_len >>
            d.valid_len >> bb >> bo >> r1b >> r1o >> r1bs >> r1cs >> d.s1 >> fb >> fo >> fbs >> r2b >> r2o >> r2bs >>
            r2cs >> d.s2;
        d.x = ptr(xb, xo); d.x_bstride = xbs; d.x_cstride = xcs; d.in_scale = ptr(ib, io); d.w = ptr(wb, wo);
        d.y = ptr(yb, yo); d.y_bstride = ybs; d.y_cstride = ycs; d.bias = ptr(bb, bo);
        d.res1 = ptr(r1b, r1o); d.r1_bstride = r1bs; d.r1_cstride = r1cs;
        d.film = ptr(fb, fo); d.film_bstride = fbs;
        d.res2 = ptr(r2b, r2o); d.r2_bstride = r2bs; d.r2_cstride = r2cs;
        if (std::getenv("OUHIP_EMU_FRAMED") && d.frame == 1) continue;
        for (int t = 0; t < ou_conv_num_tiles(); ++t) {
            if (!ou_conv_tile_ok(d.kt, t)) continue;
            for (int tpw = 0; tpw < 5; ++tpw) {   // 3: warp-specialised, 4: split-f16 (same weight bytes)
                if (tpw == 3 && d.rout != 1) continue;   // warp-specialised: plain convs only
                const int v = tpw == 4 ? 2048 : tpw == 3 ? 1024 : tpw << 8;
                if (!ou_conv_tile_ok(d.kt, t | v)) continue;
                if (std::getenv("OUHIP_EMU_VERBOSE"))
                    std::fprintf(stderr, "conv %zu (m %d cin %d frame %d kt %d n %d rout %d) tile %d tpw %d\n", ci, d.m,
                                 d.cin, d.frame, d.kt, d.n_frames, d.rout, t, tpw);
                d.tile = t | (tpw == 4 ? 0 : v);
                d.prec = tpw == 4 ? 1 : 0;
                d.w_unscale = 1.f;
                const int rc_ = ou_conv(&d, nullptr);
                if (rc_ == -2 && tpw == 3) continue;   // warp-specialised form refused for this geometry
                if (rc_ != 0) {
                    std::fprintf(stderr, "conv %zu tile %d: error %s\n", ci, t, ouhip_detail::err_buf());
                    return 3;
                }
                ++nl;
            }
        }
        ++nconv;
    }
    for (char* b : bufs) std::free(b);
    std::printf("ok: %d descriptors, %d launches bounds-checked\n", nconv, nl);
    return 0;
}
