"""Diagnostics for the sub-batched score pass: the same enhance as the
whole-batch plan and the sub-batched plan, eager and captured, with and
without split-image links; prints max |diff| against the first run.
  python tools/sub_debug.py B N_STEPS [NCH|golden:TAG] [T]"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
from open_universe_amd.configs import get_config  # noqa: E402
from open_universe_amd.networks.universe import UniverseGAN  # noqa: E402
from open_universe_amd.plan import EnhancePlan  # noqa: E402
from open_universe_amd.utils.synthetic import synth_state_dict  # noqa: E402

DEV = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
src = sys.argv[3] if len(sys.argv) > 3 else ""
T = int(sys.argv[4]) if len(sys.argv) > 4 else 16000
if src.startswith("golden:"):
    from conftest import golden_state_dict, load_golden

    d = load_golden(src[7:])
    cfg = get_config("pp16", 4)
    m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(golden_state_dict(d), strict=False)
    mix = torch.from_numpy(d["enh_mix"]).to(DEV)
    B, T = mix.shape[0], mix.shape[-1]
else:
    cfg = get_config("pp16", int(src) if src else None)
    m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()]), strict=False)
    mix = (0.1 * torch.randn(B, 1, T, generator=torch.Generator().manual_seed(3))).to(DEV)
m = m.to(DEV).eval()
eng = m._get_engine()
ref = None
for split in os.environ.get("DBG_SPLIT", "1,0").split(","):
    for sub in os.environ.get("DBG_SUB", "1,0").split(","):
        os.environ["OUHIP_SPLIT_IMAGES"], os.environ["OUHIP_SUB_BATCH"] = split, sub
        p = EnhancePlan(eng, B, T, n_steps, 1.3)
        for graph in (False, False, True, True):
            y = p(mix, torch.Generator(device=DEV).manual_seed(5), use_graph=graph).clone()
            if ref is None:
                ref = y
            d = (y - ref).abs().max().item()
            per = [(y[b] - ref[b]).abs().max().item() for b in range(B)]
            print(f"split {split} sub {sub} graph {int(graph)}: max diff {d:.3g} per item {per}", flush=True)
