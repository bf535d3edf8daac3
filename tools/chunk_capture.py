"""Diagnostics: record a chunked EnhancePlan, replay it eagerly, then capture
it as a hipGraph and replay that (argv: batch, samples, n_steps)."""
import faulthandler
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.enable()
import torch

from open_universe_amd.configs import get_config
from open_universe_amd.networks.universe import UniverseGAN
from open_universe_amd.plan import EnhancePlan
from open_universe_amd.utils.synthetic import synth_state_dict


def main():
    B, T, n = (int(a) for a in (sys.argv[1:] + ["1", "64000", "8"])[:3]) if len(sys.argv) > 1 else (1, 64000, 8)
    dev = "cuda:0"
    cfg = get_config("pp16")
    m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()]), strict=False)
    m = m.to(dev).eval()
    eng = m._get_engine()
    p = EnhancePlan(eng, B, T, n, 1.3)
    kinds = p.prog.op_kinds()
    print("chunks", p.chunks, "ops", len(kinds), "events", getattr(p.prog, "n_events", 0), flush=True)
    mix = (0.1 * torch.randn(B, 1, T)).to(dev)
    a = p(mix, torch.Generator(device=dev).manual_seed(1), use_graph=False).clone()
    torch.cuda.synchronize()
    print("eager ok", flush=True)
    p.prog.capture()
    print("captured", flush=True)
    b = p(mix, torch.Generator(device=dev).manual_seed(1), use_graph=True).clone()
    torch.cuda.synchronize()
    print("graph ok, equal:", torch.equal(a, b), flush=True)


if __name__ == "__main__":
    main()
