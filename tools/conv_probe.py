#!/usr/bin/env python
"""Probe single ou_conv tiles on one geometry against torch (fp32), one launch
at a time with a sync after each; stops at the first launch error."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from open_universe_amd import _lib as L
from open_universe_amd import engine as E


def main():
    cout, cin, kt, T, B = [int(v) for v in sys.argv[1].split(",")]
    tiles = [int(t, 0) for t in sys.argv[2].split(",")]
    lib = L.load()
    req, opt = ctypes.c_int(), ctypes.c_int()
    dev = "cuda:0"
    g = torch.Generator().manual_seed(0)
    w = torch.randn(cout, cin, kt, generator=g) * 0.1
    bias = torch.randn(cout, generator=g) * 0.1
    cw = E.make_conv(E.ConvSpec(w.numpy(), cin, 1, (kt - 1) // 2, 1, 0.25, bias.numpy()), dev)
    x = torch.randn(B, cin, T, generator=g)
    ref = F.conv1d(torch.where(x >= 0, x, 0.25 * x), w, bias, padding=(kt - 1) // 2)
    xa = E.Act(x.to(dev))
    for t in tiles:
        lib.ou_conv_lds_info(kt, t, ctypes.byref(req), ctypes.byref(opt))
        y = E.new_act(B, cout, T, dev)
        d = E.conv_desc(cw, xa, y)
        d.tile = t
        rc = lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        err = ((y.t.cpu() - ref).norm() / ref.norm()).item()
        print(f"tile {t & 0xff} tpw {1 << (t >> 8)}: rc {rc} lds {req.value} (optin max {opt.value}) rel err {err:.3g}",
              flush=True)


if __name__ == "__main__":
    main()
