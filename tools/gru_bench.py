"""Time the GRU recurrence variants (ou_gru_desc.flags) at score-network
shape (H = 256, T = 801) for a few batch sizes; prints us per time step."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from open_universe_amd import _lib as L
from open_universe_amd import engine as E
from open_universe_amd.configs import get_config
from open_universe_amd.networks.universe import UniverseGAN
from open_universe_amd.utils.synthetic import synth_state_dict


def main():
    dev = "cuda:0"
    cfg = get_config("pp16")
    m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()]), strict=False)
    m = m.to(dev).eval()
    eng = m._get_engine()
    T = int(os.environ.get("GRU_T", "801"))
    stream = torch.cuda.current_stream().cuda_stream
    gw = eng.s_gru
    for B in (1, 4, 8):
        x = E.Act(torch.randn(B, 512, T, device=dev) * 0.5)
        gi, y = E.new_act(B, 1536, T, dev), E.new_act(B, 512, T, dev)
        gran = torch.zeros(L.load().ou_gru_workspace_bytes(256, B) // 8, dtype=torch.int64, device=dev)
        ref = None
        for flags in [int(f) for f in os.environ.get("GRU_FLAGS", "5,7,9,11,21,25").split(",")]:
            E.GRU_FLAGS = flags
            prog = L.Program()
            E.rec_gru(prog, gw, 0, x, gi, y, gran, eng.status)
            prog.run(stream)
            torch.cuda.synchronize()
            ms = []
            for _ in range(5):
                t = prog.profile(stream)
                ms.append(t[1])
            out = y.t.clone()
            if ref is None:
                ref = out
            ok = torch.equal(out, ref) and int(eng.status.max()) == 0
            eng.status.zero_()
            print(f"B={B} flags={flags}: {1000 * min(ms) / T:.3f} us/step "
                  f"(median {1000 * sorted(ms)[2] / T:.3f}) identical={ok}", flush=True)
            if os.environ.get("OUHIP_LIB", "").endswith("_diag.so"):
                # phase stamps (OU_GRU_STAMPS build): cycles per step per workgroup
                st = gran[B * 4 * 256 + B * 256 // 4:].view(-1, 8).cpu()
                rows = [r for r in st.tolist() if r[5] > 0]
                names = (("poll", "lds+bar1", "dot", "gate+store", "bar2") if flags & 32 else
                         ("poll", "fma", "reduce", "gate+store", "local_l2x"))
                for w, r in enumerate(rows[:4]):
                    print("   wg%d " % w + " ".join(f"{n}={r[i] / r[5]:.0f}" for i, n in enumerate(names[:4])) + f" {names[4]}={r[4]}",
                          f"total={sum(r[:5]) / r[5]:.0f} cyc/step", flush=True)


if __name__ == "__main__":
    main()
