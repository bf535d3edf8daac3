"""Diagnostics for the sub-batched score pass: the same B = 2 enhance as the
whole-batch plan and the sub-batched plan, eager and captured, with and
without split-image links; prints max |diff| against the whole-batch eager run."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from open_universe_amd.configs import get_config  # noqa: E402
from open_universe_amd.networks.universe import UniverseGAN  # noqa: E402
from open_universe_amd.plan import EnhancePlan  # noqa: E402
from open_universe_amd.utils.synthetic import synth_state_dict  # noqa: E402

DEV = "cuda:0"
nch = int(sys.argv[3]) if len(sys.argv) > 3 else None
cfg = get_config("pp16", nch)
m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
m.load_state_dict(synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()]), strict=False)
m = m.to(DEV).eval()
eng = m._get_engine()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
T = int(sys.argv[4]) if len(sys.argv) > 4 else 16000
n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
mix = (0.1 * torch.randn(B, 1, T, generator=torch.Generator().manual_seed(3))).to(DEV)
ref = None
for split in ("1", "0"):
    for sub in ("0", "1"):
        os.environ["OUHIP_SPLIT_IMAGES"], os.environ["OUHIP_SUB_BATCH"] = split, sub
        p = EnhancePlan(eng, B, T, n_steps, 1.3)
        for graph in (False, False, True, True):
            y = p(mix, torch.Generator(device=DEV).manual_seed(5), use_graph=graph).clone()
            if ref is None:
                ref = y
            d = (y - ref).abs().max().item()
            per = [(y[b] - ref[b]).abs().max().item() for b in range(B)]
            print(f"split {split} sub {sub} graph {int(graph)}: max diff {d:.3g} per item {per}", flush=True)
