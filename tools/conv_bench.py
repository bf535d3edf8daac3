#!/usr/bin/env python
"""Time ou_conv tiles on representative UNIVERSE++ 16 kHz layer shapes.

    python tools/conv_bench.py                       # every layer, every valid tile
    python tools/conv_bench.py --layer L2k3 --tile 11 --reps 50   # one config (for rocprofv3 --pmc)

Random weights/inputs (timing does not depend on values).  Prints ms per
launch and algorithmic TFLOP/s per (layer, tile).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from open_universe_amd import _lib as L
from open_universe_amd import engine as E

# name: (m, cin, frame, kt, n_frames, rout, residual)
LAYERS = {
    "L0k3": (32, 32, 1, 3, 128000, 1, True),
    "L0k5": (32, 32, 1, 5, 128000, 1, False),
    "L1k3": (64, 64, 1, 3, 64000, 1, True),
    "L1k5": (64, 64, 1, 5, 64000, 1, False),
    "L2k3": (128, 128, 1, 3, 16000, 1, True),
    "L2k5": (128, 128, 1, 5, 16000, 1, False),
    "L3k3": (256, 256, 1, 3, 4000, 1, True),
    "L3k5": (256, 256, 1, 5, 4000, 1, False),
    "L4k3": (512, 512, 1, 3, 800, 1, True),
    "L4k5": (512, 512, 1, 5, 800, 1, False),
    "D3": (512, 256, 5, 3, 800, 1, False),     # down-sampling conv, rate 5 (polyphase)
    "D1": (128, 64, 4, 3, 16000, 1, False),    # down-sampling conv, rate 4 (level 1 -> 2)
    "D2": (256, 128, 4, 3, 4000, 1, False),    # down-sampling conv, rate 4 (level 2 -> 3)
    "CD1": (128, 64, 4, 1, 16000, 1, False),   # conditioner down conv (no FIR), rate 4
    "ST0": (512, 32, 160, 1, 800, 1, False),   # conditioner st_convs (level -> bottleneck)
    "ST1": (512, 64, 80, 1, 800, 1, False),
    "ST2": (512, 128, 20, 1, 800, 1, False),
    "U3": (1280, 512, 1, 3, 800, 5, True),     # up-sampling conv, rate 5
    "GI": (1536, 512, 1, 1, 800, 1, False),    # GRU input projection
    "U2": (512, 256, 1, 3, 4000, 4, True),     # up-sampling conv, rate 4 (level 3 -> 2)
    "U1": (256, 128, 1, 3, 16000, 4, True),    # up-sampling conv, rate 4 (level 2 -> 1)
    # PP24 at C4 (B = 32, 10 s) as one long item: the batch's frames back to back
    "P3k3": (384, 384, 1, 3, 256256, 1, True),    # 384-channel level, k3
    "P4k3": (768, 768, 1, 3, 32032, 1, True),     # 768-channel level, k3
    "PD5": (384, 192, 5, 3, 256256, 1, False),    # down conv rate 5 (192 -> 384 channels)
}


def make(name, dev, seed=0):
    m, cin, frame, kt, n, rout, res = LAYERS[name]
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(m, cin * frame, kt, generator=g) * 0.05).numpy()
    spec = E.ConvSpec(w, cin, frame, (kt - 1) // 2, rout, 0.25, np.zeros(m // rout, np.float32),
                      ref_macs=float(w.size))
    cw = E.make_conv(spec, dev)
    x = E.Act(torch.randn(1, cin, n * frame, device=dev))
    y = E.new_act(1, m // rout, n * rout, dev)
    r = E.Act(torch.randn(1, m // rout, n * rout, device=dev)) if res else None
    d = E.conv_desc(cw, x, y, res1=r, s1=0.7, n_frames=n)
    ws = torch.empty(E.KSWS_BYTES // 4, dtype=torch.float32, device=dev)   # K-slice workspace
    d.ks_ws, d.ks_ws_bytes = ws.data_ptr(), E.KSWS_BYTES
    return d, (cw, x, y, r, ws)


GRAPH_COPIES = 20


def split_image(x, slope, shift, rows=None):
    """Host-side (torch) split image of prelu(x) * 2^-shift, include/ouhip.h
    layout [B][C / 32][rows][hi | lo][32] as int16 (tools and tests only)."""
    B, C, T = x.shape
    rows = T if rows is None else rows
    p = x.float() * 2.0 ** -shift
    p = torch.where(p >= 0, p, p * slope)
    hi = p.half()
    lo = ((p - hi.float()) * 2048.0).half()
    img = torch.zeros(B, C // 32, rows, 2, 32, dtype=torch.float16, device=x.device)
    img[:, :, :T, 0, :] = hi.reshape(B, C // 32, 32, T).transpose(2, 3)
    img[:, :, :T, 1, :] = lo.reshape(B, C // 32, 32, T).transpose(2, 3)
    return img.view(torch.int16).reshape(-1)


def split_variant(d, keep, shift=6):
    """The same layer reading a split image of its input (tile bit 15)."""
    cw, x = keep[0], keep[1]
    img = split_image(x.t, cw.slope, shift)
    ds = L.ConvDesc.from_buffer_copy(d)
    ds._flops = d._flops
    ds.xs, ds.xs_bstride, ds.xs_rows, ds.xs_shift = img.data_ptr(), img.numel() * 2 // x.B, x.T, shift
    ds.w, ds.w_unscale = cw.w_nat.data_ptr(), cw.w_unscale_nat
    return ds, img


def time_tile_graph(d, tile, reps, stream):
    """Device time per launch: GRAPH_COPIES copies of the op captured in one
    hipGraph (no host launch cost in the figure; K-slice tiles pay their
    second launch as a graph node, as in the recorded plans)."""
    import ctypes

    lib = L.load()
    d.tile = tile
    if lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream)) != 0:
        return None
    prog = L.Program()
    for _ in range(GRAPH_COPIES):
        prog.add(L.OP_CONV, d)
    prog.capture()
    prog.launch(stream)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(max(2, reps // 10)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        prog.launch(stream)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / GRAPH_COPIES)
    return best


def time_tile(d, tile, reps, stream):
    import ctypes

    if os.environ.get("CONV_BENCH_GRAPH", "1") == "1":
        return time_tile_graph(d, tile, reps, stream)
    lib = L.load()
    d.tile = tile
    if lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream)) != 0:
        return None
    for _ in range(2):
        lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream))
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default=None)
    ap.add_argument("--tile", type=int, default=None)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rdiag", action="store_true",
                    help="register-streamed tiles: also time without input loads (bit 8) / without the K loop (bit 9)")
    ap.add_argument("--stamps", action="store_true", help="diag library: per-phase cycles")
    ap.add_argument("--wstamps", action="store_true", help="diag library: warp-specialised kernel phases")
    ap.add_argument("--sstamps", action="store_true",
                    help="with --split, a library built with -DOU_SK_STAMPS: per-wave phase cycles of the best "
                         "split-image tile")
    ap.add_argument("--split", action="store_true",
                    help="also time the split-image kernel (tile bit 15) on a split image of the input, check its "
                         "output against the best tile's, and re-time the best tile storing a split image (sy)")
    a = ap.parse_args()
    dev = "cuda:0"
    stream = torch.cuda.current_stream().cuda_stream
    lib = L.load()
    names = a.layer.split(",") if a.layer else list(LAYERS)
    for name in names:
        d, keep = make(name, dev)
        if d.prec == 1:
            tiles = [a.tile] if a.tile is not None else [t | k for t in range(lib.ou_conv_num_tiles())
                                                          if lib.ou_conv_tile_ok(d.kt, t | (1 << 11))
                                                          for k in (0, 1 << 12, 2 << 12, 3 << 12)]
            if a.tile is None and d.cin % 16 == 0:   # register-streamed kernel
                tiles += [t | E.RS_BIT for t in range(16) if lib.ou_conv_tile_ok(d.kt, t | E.RS_BIT)]
                if a.rdiag:
                    tiles += [t | v for t in tiles if t & E.RS_BIT for v in (1 << 8, 2 << 8, 3 << 8)]
        else:
            tiles = [a.tile] if a.tile is not None else [t | v for t in range(lib.ou_conv_num_tiles())
                                                          for v in (0, 1 << 8, 2 << 8, 1 << 10)
                                                          if lib.ou_conv_tile_ok(d.kt, t | v)]
        res = []
        for t in tiles:
            ms = time_tile(d, t, a.reps, stream)
            if ms is not None:
                res.append((ms, t))
        res.sort()
        fl = d._flops
        def nm(t):
            if t & E.RS_BIT:
                return f"r{t & 0xff}" + ("" if not (t >> 8) & 3 else f"d{(t >> 8) & 3}")
            return (f"t{t & 0xff}" + ("w" if (t >> 10) & 1 else (f"p{1 << ((t >> 8) & 3)}" if (t >> 8) & 3 else ""))
                    + (f"k{1 << (t >> 12)}" if t >> 12 else ""))
        line = "  ".join(f"{nm(t)}:{ms * 1e3:.1f}us" for ms, t in res[:40 if a.rdiag else 12])
        print(f"{name:5s} {fl / 1e9:6.2f} GFLOP  best {nm(res[0][1])} {res[0][0] * 1e3:.1f} us "
              f"{fl / res[0][0] / 1e9:.1f} TF/s | {line}", flush=True)
        if a.split and keep[0].w_nat is not None:
            import ctypes

            y = keep[2].t
            d.tile = res[0][1]
            lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream))
            torch.cuda.synchronize()
            yref = y.clone()
            ds, img = split_variant(d, keep)
            sres = []
            for t in range(6):
                for mj in (0, 1 << 16):
                    ms = time_tile(ds, L.SS_BIT | t | mj, a.reps, stream)
                    if ms is not None:
                        sres.append((ms, L.SS_BIT | t | mj))
            sres.sort()
            ds.tile = sres[0][1]
            y.fill_(float("nan"))
            assert lib.ou_conv(ctypes.byref(ds), ctypes.c_void_p(stream)) == 0
            torch.cuda.synchronize()
            err = ((y - yref).norm() / yref.norm()).item()
            # the producer side: the best tile storing a split image of its output
            m_out = keep[0].cout
            sy = torch.zeros(m_out // 32 * y.shape[-1] * 64 * y.shape[0], dtype=torch.int16, device=dev) \
                if keep[0].rout == 1 and m_out % 32 == 0 else None
            t_sy = None
            if sy is not None:
                d.sy, d.sy_bstride, d.sy_rows, d.sy_shift, d.sy_slope = sy.data_ptr(), m_out // 32 * y.shape[-1] * 128, \
                    y.shape[-1], 6, 0.25
                t_sy = time_tile(d, res[0][1], a.reps, stream)
                d.sy = None
            if a.sstamps:
                st_buf = torch.zeros(1024 * 4 * 8, dtype=torch.int64, device=dev)
                ds.ks_ws = st_buf.data_ptr()
                assert lib.ou_conv(ctypes.byref(ds), ctypes.c_void_p(stream)) == 0
                torch.cuda.synchronize()
                ds.ks_ws = None
                st = st_buf.view(1024, 4, 8).cpu().numpy().astype(np.float64)
                st = st[st[:, :, :4].sum(axis=(1, 2)) > 0]
                if len(st):
                    ph = st[:, :, :4].mean(axis=(0, 1))
                    skew = (st[:, :, 1].max(1) - st[:, :, 1].min(1)).mean()   # main-loop spread within a WG
                    life = (st[:, :, 7] - st[:, :, 6]).mean() / 100.0
                    t0 = st[:, :, 6].min()
                    print(f"      stamps ({len(st)} WGs, cycles per wave): prologue={ph[0]:.0f} main={ph[1]:.0f} "
                          f"reduce={ph[2]:.0f} epilogue={ph[3]:.0f} (main-loop skew in a WG {skew:.0f}); "
                          f"wave lifetime {life:.2f} us; starts "
                          f"0..{(st[:, :, 6].max() - t0) / 100:.2f} us, last end {(st[:, :, 7].max() - t0) / 100:.2f} us",
                          flush=True)
            sl = "  ".join(f"s{t & 0xff}{'m' if t & (1 << 16) else ''}:{ms * 1e3:.1f}us" for ms, t in sres)
            print(f"      split image: best {sres[0][0] * 1e3:.1f} us {fl / sres[0][0] / 1e9:.1f} TF/s "
                  f"(rel diff vs best tile {err:.2e}) | {sl}" +
                  (f" | best tile storing sy: {t_sy * 1e3:.1f} us" if t_sy else ""), flush=True)
        if a.wstamps:
            import ctypes

            n = 4096 * 8
            buf = (ctypes.c_uint64 * n)()
            lib.ou_conv_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
            assert lib.ou_conv_read_stamps(ctypes.cast(buf, ctypes.c_void_p), n) == 0
            st = np.frombuffer(buf, dtype=np.uint64).reshape(2048, 16).astype(np.float64)
            st = st[st[:, :5].sum(1) > 0]
            c, l = st[:, :8], st[:, 8:]
            print(f"      {len(st)} WGs; MFMA wave cycles: mfma={c[:, 1].mean():.0f} acc-image={c[:, 2].mean():.0f} "
                  f"tick-barrier={c[:, 3].mean():.0f} first-barrier={c[:, 4].mean():.0f}; staging wave: "
                  f"dma-issue={l[:, 0].mean():.0f} vmcnt-wait={l[:, 1].mean():.0f} prelu={l[:, 3].mean():.0f} "
                  f"epilogue={l[:, 4].mean():.0f} res+other={l[:, 5].mean():.0f} barrier={l[:, 2].mean():.0f}",
                  flush=True)
            t0 = c[:, 6].min()
            print(f"      realtime (us): MFMA wave start {(c[:, 6].max() - t0) / 100:.2f} max, end {(c[:, 7] - t0).min() / 100:.2f}.."
                  f"{(c[:, 7] - t0).max() / 100:.2f}", flush=True)
        if a.stamps:
            import ctypes

            n = 4096 * 8
            buf = (ctypes.c_uint64 * n)()
            lib.ou_conv_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
            assert lib.ou_conv_read_stamps(ctypes.cast(buf, ctypes.c_void_p), n) == 0
            st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.float64)
            st = st[st.sum(1) > 0]
            names = ("prologue", "load_issue", "mfma", "store", "barrier", "epilogue")
            if (res[0][1] if a.tile is None else a.tile) & E.RS_BIT:
                names = ("ring_issue", "staging", "barrier", "mfma", "reduce", "epilogue")
            mean = st.mean(0)
            rt0, rt1 = st[:, 6], st[:, 7]
            print(f"      realtime (us, 100 MHz): WG duration mean {(rt1 - rt0).mean() / 100:.2f} "
                  f"min {(rt1 - rt0).min() / 100:.2f} max {(rt1 - rt0).max() / 100:.2f}; starts spread "
                  f"{(rt0.max() - rt0.min()) / 100:.2f}, first start -> last end {(rt1.max() - rt0.min()) / 100:.2f}",
                  flush=True)
            print(f"      stamps over {len(st)} WGs (cycles): " +
                  " ".join(f"{nm}={mean[i]:.0f}" for i, nm in enumerate(names)) +
                  f" total={mean[:6].sum():.0f} (min {st[:, :6].sum(1).min():.0f} max {st[:, :6].sum(1).max():.0f})",
                  flush=True)
            t0 = st[:, 6].min()
            s0, s1 = (st[:, 6] - t0) / 100.0, (st[:, 7] - t0) / 100.0   # s_memrealtime: 100 MHz -> us
            dur = s1 - s0
            print(f"      realtime: starts 0..{s0.max():.2f} us, ends {s1.min():.2f}..{s1.max():.2f} us, "
                  f"WG lifetime mean {dur.mean():.2f} max {dur.max():.2f} us; span {s1.max():.2f} us; "
                  f"start quantiles {np.quantile(s0, [0.25, 0.5, 0.75, 0.95]).round(2).tolist()}", flush=True)


if __name__ == "__main__":
    main()
