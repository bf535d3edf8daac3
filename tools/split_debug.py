"""Diagnostics: replay a recorded enhance() op by op (one-op programs, same
descriptors and tiles) and report the first op whose output is non-finite,
with the input/output magnitudes of every conv on the way."""
import ctypes
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import torch

from open_universe_amd import _lib as L
from open_universe_amd import engine as E
from open_universe_amd import plan as P

acts = []
_orig = E.new_act


def _rec(B, C, T, dev):
    a = _orig(B, C, T, dev)
    acts.append(a)
    return a


E.new_act = _rec
P.new_act = _rec
ops = []
_add = L.Program.add


def _radd(self, op, desc):
    _add(self, op, desc)
    c = type(desc)()
    ctypes.memmove(ctypes.addressof(c), ctypes.addressof(desc), ctypes.sizeof(desc))
    ops.append((op, c))


L.Program.add = _radd


def owner(ptr):
    for a in acts:
        base = a.t.data_ptr()
        if base <= ptr < base + a.t.numel() * 4:
            return a.t
    return None


def main():
    from conftest import golden_state_dict, load_golden
    from open_universe_amd.configs import get_config
    from open_universe_amd.networks.universe import UniverseGAN

    import os

    arch = os.environ.get("ARCH", "pp16")
    if arch == "pp16":
        d = load_golden("pp16")
        cfg = get_config("pp16", None)
        m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
        m.load_state_dict(golden_state_dict(d), strict=False)
        m = m.to("cuda:0").eval()
    else:   # bench.py's synthetic model of that architecture
        import bench

        cfg, m = bench.build_model("cuda:0", arch=arch)
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 128000
    mix = (0.1 * torch.randn(1, T, generator=torch.Generator().manual_seed(3))).to("cuda:0")
    from open_universe_amd.plan import EnhancePlan

    eng = m._get_engine()
    plan = EnhancePlan(eng, 1, T, 8, 1.3)
    plan.MIX.copy_(mix[:, None])
    plan.draw_noise(torch.Generator(device="cuda:0").manual_seed(2))
    plan._launch(torch.cuda.current_stream().cuda_stream, False)
    torch.cuda.synchronize()
    print("prec", eng.conv_prec, "status", eng.status.tolist(), "finite", bool(torch.isfinite(plan.OUT).all()),
          "ops", len(ops), flush=True)
    eng.status.zero_()
    for a in acts:
        a.t.zero_()
    stream = torch.cuda.current_stream().cuda_stream
    for i, (op, desc) in enumerate(ops):
        p = L.Program()
        _add(p, op, desc)
        p.run(stream)
        torch.cuda.synchronize()
        if op == L.OP_CONV:
            x, y = owner(desc.x), owner(desc.y)
            xm = float(x.abs().max()) if x is not None else -1
            ym = float(y.abs().max()) if y is not None else -1
            fin = y is None or bool(torch.isfinite(y).all())
            st = eng.status[:4 + len(eng.range_owners)].tolist()
            print(f"{i} conv m={desc.m} cin={desc.cin} fr={desc.frame} kt={desc.kt} n={desc.n_frames} "
                  f"rout={desc.rout} tile={desc.tile} prec={desc.prec} xs_shift={desc.xs_shift} |x|max={xm:.4g} "
                  f"|y|max={ym:.4g} finite={fin} status={st}", flush=True)
            if any(st[1:]):
                print("RANGE FLAG at op", i)
                return
            if not fin:
                print("FIRST NON-FINITE at op", i)
                return
        elif op == L.OP_GRU:
            y = owner(desc.y)
            fin = y is None or bool(torch.isfinite(y).all())
            print(f"{i} gru finite={fin}", flush=True)
            if not fin:
                print("FIRST NON-FINITE at op", i)
                return


main()
