"""Which buffers of a sub-batched plan differ between its first and second
replay (golden pp16_c4, B = 2): the first stage that differs names a missing
dependency."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
from conftest import golden_state_dict, load_golden  # noqa: E402
from open_universe_amd.configs import get_config  # noqa: E402
from open_universe_amd.networks.universe import UniverseGAN  # noqa: E402
from open_universe_amd.plan import EnhancePlan  # noqa: E402

DEV = "cuda:0"
d = load_golden("pp16_c4")
cfg = get_config("pp16", 4)
m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
m.load_state_dict(golden_state_dict(d), strict=False)
m = m.to(DEV).eval()
mix = torch.from_numpy(d["enh_mix"]).to(DEV)
B, T = mix.shape[0], mix.shape[-1]
eng = m._get_engine()
n_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
os.environ["OUHIP_SUB_BATCH"] = sys.argv[2] if len(sys.argv) > 2 else "1"
p = EnhancePlan(eng, B, T, n_steps, 1.3)


def snap():
    out = {}
    for name, bufs in [("cb", p.cb)] + [(f"sb{k}", sb) for k, sb in enumerate(getattr(p, "score_bufs", [p.sb]))]:
        for k, v in bufs.items():
            t = getattr(v, "t", v)
            if isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32:
                out[f"{name}.{k}"] = t.clone()
            elif isinstance(v, list):
                for i, a in enumerate(v):
                    if hasattr(a, "t"):
                        out[f"{name}.{k}{i}"] = a.t.clone()
    for i, a in enumerate(p.SC):
        out[f"SC{i}"] = a.t.clone()
    out["X"], out["OUT"] = p.X.t.clone(), p.OUT.clone()
    return out


def poison():
    """NaN into every activation and split-image buffer of the plan (not the
    GRU workspaces, which a replay zeroes itself): a read of a value this
    replay did not write shows as a NaN output."""
    for name, bufs in [("cb", p.cb)] + [(f"sb{k}", sb) for k, sb in enumerate(getattr(p, "score_bufs", [p.sb]))]:
        for k, v in bufs.items():
            if k == "gran":
                continue
            for a in (v if isinstance(v, list) else [v]):
                t = getattr(a, "t", a)
                if isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32:
                    t.fill_(float("nan"))
    for a in p.SC:
        a.t.fill_(float("nan"))
    for buf in getattr(p.prog, "split_bufs", {}).values():
        buf.fill_(0x7E00)
    torch.cuda.synchronize()


def nan_bufs(s):
    return {k for k, v in s.items() if torch.isnan(v).any()}


if os.environ.get("DBG_POISON_FIRST", "1") == "1":
    poison()
y1 = p(mix, torch.Generator(device=DEV).manual_seed(5), use_graph=False).clone()
s1 = snap()
print(f"first replay: finite {bool(torch.isfinite(y1).all())}", flush=True)
unused = None
for i, graph in enumerate((False, False, True, True)):
    poison()
    y2 = p(mix, torch.Generator(device=DEV).manual_seed(5), use_graph=graph).clone()
    print(f"poisoned replay {i} graph {int(graph)}: finite {bool(torch.isfinite(y2).all())} "
          f"diff vs first {(y1 - y2).abs().nan_to_num(1e9).max().item():.3g}", flush=True)
    nb = nan_bufs(snap())
    unused = nb if unused is None else unused & nb
s2 = snap()
print("NaN after the first replay only:", sorted(nan_bufs(s1) - unused))
for k in s1:
    a, b = s1[k], s2[k]
    if not torch.equal(a, b):
        per = [(a[i] - b[i]).abs().max().item() for i in range(a.shape[0])] if a.dim() >= 2 else []
        print(f"{k} {tuple(a.shape)}: max diff {(a - b).abs().max().item():.3g} per item {per}")
