#!/usr/bin/env python
"""Record an enhance program on CPU memory (never launched) and write every
ou_conv descriptor it holds, with each pointer resolved to (tensor storage,
byte offset) and every storage's size, for tests/emu/conv_emu_plan.cpp.

    python tests/emu/dump_plan_convs.py OUT.txt [config] [n_channels] [B] [T]
"""
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from open_universe_amd import _lib as L
from open_universe_amd.configs import get_config
from open_universe_amd.engine import Engine
from open_universe_amd.networks.universe import Universe, UniverseGAN
from open_universe_amd.plan import EnhancePlan
from open_universe_amd.utils.synthetic import synth_state_dict

PTRS = ("x", "in_scale", "w", "y", "bias", "res1", "film", "res2")


def main():
    out = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "pp16"
    nch = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    T = int(sys.argv[5]) if len(sys.argv) > 5 else 4000
    cfg = get_config(name, nch)
    cls = UniverseGAN if cfg["_target_"].endswith("UniverseGAN") else Universe
    m = cls(**{k: v for k, v in cfg.items() if k != "_target_"})
    sd = synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()], 0)
    descs = []

    orig_add = L.Program.add

    def add(self, op, desc):
        if op == L.OP_CONV:
            c = L.ConvDesc()
            ctypes_copy(c, desc)
            descs.append(c)
        return orig_add(self, op, desc)

    L.Program.add = add
    try:
        eng = Engine(cfg, sd, "cpu", _record_only=True)
        plans = [EnhancePlan(eng, B, T, 8, 1.3)]
        if name != "orig16":
            plans.append(EnhancePlan(eng, B, T, 8, 1.3, use_aux_signal=True))
    finally:
        L.Program.add = orig_add
    spans = {}
    for o in gc.get_objects():
        if torch.is_tensor(o) and o.device.type == "cpu":
            st = o.untyped_storage()
            spans[st.data_ptr()] = max(spans.get(st.data_ptr(), 0), st.nbytes())
    bases = sorted(spans)
    ids = {b: i for i, b in enumerate(bases)}

    def where(p):
        if not p:
            return (-1, 0)
        for b in bases:
            if b <= p < b + spans[b]:
                return (ids[b], p - b)
        raise RuntimeError(f"pointer {p:#x} is in no CPU tensor")

    # one descriptor per distinct (geometry, buffer sizes, offsets): the
    # diffusion steps repeat the same layers on the same buffers
    seen, uniq = set(), []
    for d in descs:
        v = tuple(getattr(d, k) if k not in PTRS else (lambda w: (spans[bases[w[0]]] if w[0] >= 0 else -1, w[1]))(
            where(getattr(d, k))) for k, _ in L.ConvDesc._fields_ if k != "tile")
        if v not in seen:
            seen.add(v)
            uniq.append(d)
    descs = uniq
    with open(out, "w") as fh:
        for b in bases:
            fh.write(f"BUF {ids[b]} {spans[b]}\n")
        for d in descs:
            v = {k: getattr(d, k) for k, _ in L.ConvDesc._fields_}
            loc = {k: where(v[k]) for k in PTRS}
            f = [*loc["x"], v["x_bstride"], v["x_cstride"], v["cin"], v["in_len"], v["frame"], v["shift"],
                 *loc["in_scale"], v["slope"], *loc["w"], v["m"], v["kt"], v["pad"], v["cc"], v["n_frames"],
                 v["batch"], *loc["y"], v["y_bstride"], v["y_cstride"], v["rout"], v["out_len"], v["valid_len"],
                 *loc["bias"], *loc["res1"], v["r1_bstride"], v["r1_cstride"], v["s1"], *loc["film"],
                 v["film_bstride"], *loc["res2"], v["r2_bstride"], v["r2_cstride"], v["s2"]]
            fh.write("CONV " + " ".join(str(x) for x in f) + "\n")
    print(f"{len(descs)} conv descriptors, {len(bases)} buffers -> {out}")


def ctypes_copy(dst, src):
    import ctypes

    ctypes.memmove(ctypes.byref(dst), ctypes.byref(src), ctypes.sizeof(dst))


if __name__ == "__main__":
    main()
