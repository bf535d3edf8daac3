#!/usr/bin/env python
"""Benchmark: seconds of audio enhanced per second, UNIVERSE++ 16 kHz, 8 s clips.

    python bench.py [--gpus N] [--steps K] [--warmup W]

One step = one ``model.enhance()`` of one synthetic 8 s clip at batch 1
(BASELINE.json configs[1]: "UNIVERSE++ 16 kHz, batch=1, 8 s clips"), run as
the production path does it: one hipGraph replay of the recorded sampler
(conditioner + 8 score-network passes + sampler updates).  Every rank (one
process per GPU, torchrun) enhances its own clips -- utterances shard across
GPUs with no collective on the data path -- so scaling is weak; ``value`` is
the whole-job audio-seconds per second: N * K * 8 s / max-over-ranks time.

Extra fields:
  roofline      the dominant kernel (ou_conv, every launch of one enhance):
                algorithmic FLOPs of the reference ops it replaces and
                algorithmic bytes (activations once, f32 weights) over its
                device time, measured with HIP events per launch in an
                instrumented eager replay of the same enhance on the same
                stream; the bound is whichever of FLOPs/MFMA peak and
                bytes/HBM peak is larger.
  cpu_baseline  the CPU restatement of the reference op sequence (oracle/,
                plain PyTorch) on this host's cores, bounded sample.
Weights are synthetic (no trained checkpoint offline); timing does not depend
on weight values.
"""
import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

FS = 16000
CLIP_S = 8.0
FP32_PEAK_TF = 157.3   # MI355X dense FP32 matrix peak (MI355X_MICROARCH.md)
F16_PEAK_TF = 2516.6   # dense F16/BF16 MFMA peak; split-f16 spends 3 MFMAs per f32 MAC
HBM_PEAK = 8000.0      # GB/s


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# BASELINE.json configs: c2 is the headline (default); the others are measured
# on request (--config) with the same harness.  Batch is per GPU for c3 and the
# whole-node batch for c4 (32 clips sharded over the ranks: 32/N per rank).
CONFIGS = {
    "c2": dict(arch="pp16", batch=1, seconds=8.0, n_steps=None,
               workload="UNIVERSE++ 16 kHz enhance(), batch=1, 8 s clip, 8 diffusion steps (BASELINE.json configs[1])"),
    "c3": dict(arch="orig16", batch=8, seconds=8.0, n_steps=60,
               workload="UNIVERSE (original) 16 kHz enhance(), batch=8, 8 s clips, 60 diffusion steps "
                        "(BASELINE.json configs[2])"),
    "c4": dict(arch="pp24", batch=32, seconds=10.0, n_steps=None, node_batch=True,
               workload="UNIVERSE++ 24 kHz enhance(), batch=32 per node sharded over the GPUs, 10 s clips, "
                        "8 diffusion steps (BASELINE.json configs[3])"),
    "c5": dict(arch="pp16", batch=1, seconds=60.0, n_steps=None, conv_prec="f16",
               workload="UNIVERSE++ 16 kHz enhance(), batch=1, 60 s long-form clip, 8 diffusion steps, fp16 conv "
                        "operands, whole sampler captured in one hipGraph (BASELINE.json configs[4])"),
}


def build_model(device, nch=None, seed=0, arch="pp16"):
    import torch

    from open_universe_amd.configs import get_config
    from open_universe_amd.networks.universe import Universe, UniverseGAN
    from open_universe_amd.utils.synthetic import synth_state_dict

    cfg = get_config(arch, nch)
    cls = Universe if cfg["_target_"].endswith(".Universe") else UniverseGAN
    m = cls(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()], seed),
                      strict=False)
    return cfg, m.to(device).eval()


def cpu_baseline(model, cfg, seconds):
    """Oracle (CPU restatement of the reference ops) on a bounded sample:
    one 8 s clip, 1 warm-up + best of 3."""
    import numpy as np
    import torch

    from oracle import ou_oracle
    from open_universe_amd.utils.synthetic import synth_audio

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    torch.set_num_threads(threads)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    orc = ou_oracle.Oracle(sd, cfg)
    T = int(seconds * FS)
    mix = torch.from_numpy(synth_audio(T, FS, 99)[0])[None]
    best = float("inf")
    with torch.no_grad():
        for i in range(4):
            t0 = time.perf_counter()
            orc.enhance(mix, rng=torch.Generator().manual_seed(1028282))
            dt = time.perf_counter() - t0
            if i > 0:
                best = min(best, dt)
    return {"value": round(seconds / best, 4), "unit": "audio-s/s", "cores": threads,
            "kind": "port",
            "sample": f"oracle/ou_oracle.py Oracle.enhance, UNIVERSE++ 16 kHz, one {seconds:g} s clip, "
                      f"B=1, 8 steps, fp32, best of 3 after 1 warm-up ({best:.3f} s), {cpu_model()}"}


def profile_roofline(plan, stream, dump=None):
    """Per-op device time of one instrumented eager replay of the plan."""
    from open_universe_amd import _lib as L

    ms = plan.prog.profile(stream)
    if dump:
        rows = []
        for i, (t, k, f) in enumerate(zip(ms, plan.prog.op_kinds(), plan.prog.flops)):
            info = plan.prog.info[i] if i < len(plan.prog.info) else {}
            rows.append({"i": i, "kind": k, "ms": t, "gflop": f / 1e9, **info})
        with open(dump, "w") as fh:
            json.dump(rows, fh)
    kinds = plan.prog.op_kinds()
    flops = plan.prog.flops
    conv_ms = sum(t for t, k in zip(ms, kinds) if k == L.OP_CONV)
    conv_fl = sum(f for f, k in zip(flops, kinds) if k == L.OP_CONV)
    conv_by = sum(b for b, k in zip(plan.prog.bytes, kinds) if k == L.OP_CONV)
    n_conv = sum(1 for k in kinds if k == L.OP_CONV)
    gru_ms = sum(t for t, k in zip(ms, kinds) if k == L.OP_GRU)
    return {
        "conv_ms": conv_ms, "conv_flops": conv_fl, "conv_bytes": conv_by, "n_conv": n_conv, "gru_ms": gru_ms,
        "total_ms": sum(ms), "total_flops": sum(flops), "n_ops": len(ms),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="BASELINE.json config (c2 = configs[1], the headline)")
    ap.add_argument("--seconds", type=float, default=None, help="override the config's clip length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--dump-ops", default=None, help="write per-op profile rows (JSON)")
    ap.add_argument("--traffic-json", default=os.path.join(HERE, "profiles", "pmc_latest.json"),
                    help="per-kernel HBM traffic from tools/pmc_summary.py (rocprofv3 PMC passes)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    from open_universe_amd.utils.synthetic import synth_audio

    from open_universe_amd.sharding import dist_env, max_over_ranks

    rank, local, world = dist_env()
    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    C = CONFIGS[args.config]
    if C.get("conv_prec") and "OUHIP_CONV_PREC" not in os.environ:
        os.environ["OUHIP_CONV_PREC"] = C["conv_prec"]
    if args.seconds is None:
        args.seconds = C["seconds"]
    B = C["batch"] // world if C.get("node_batch") else C["batch"]
    assert B >= 1, "c4 shards 32 clips over at most 32 ranks"
    cfg, model = build_model(dev, arch=C["arch"])
    fs = int(cfg["fs"])
    T = int(args.seconds * fs)
    n_clips = args.warmup + args.steps
    clips = [torch.from_numpy(np.stack([synth_audio(T, fs, rank * 100003 + i * 97 + j)[0] for j in range(B)]))
             .to(dev) for i in range(min(n_clips, 4))]
    rng = torch.Generator(device=dev).manual_seed(1028282 + rank)
    ekw = {"n_steps": C["n_steps"]} if C["n_steps"] else {}

    with torch.no_grad():
        for i in range(args.warmup):
            model.enhance(clips[i % len(clips)], rng=rng, **ekw)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            model.enhance(clips[(args.warmup + i) % len(clips)], rng=rng, **ekw)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed)

    prof = None
    if not args.no_profile:
        plan = next(iter(model._plans.values()))
        with torch.no_grad():
            plan.MIX.copy_(clips[0].reshape(plan.MIX.shape))
            plan.draw_noise(rng)
            prof = profile_roofline(plan, torch.cuda.current_stream(dev).cuda_stream, args.dump_ops)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c2":
        cpu = cpu_baseline(model, cfg, args.seconds)

    prec = model._get_engine().conv_prec
    if prec == 1:
        dtype = "f32 (conv operands split into f16 hi/lo: 3 f16 MFMA passes, f32 accumulation)"
        peak, peak_basis = round(F16_PEAK_TF / 3, 1), "dense f16 MFMA peak / 3 passes per f32 MAC"
    elif prec == 2:
        dtype = "f16 (conv operands f16, f32 accumulation; GRU, sampler and STFT/mel in f32)"
        peak, peak_basis = F16_PEAK_TF, "dense f16 MFMA peak"
    else:
        dtype, peak, peak_basis = "f32", FP32_PEAK_TF, "dense f32 MFMA peak"
    if rank == 0:
        audio_s = world * B * args.steps * args.seconds
        value = audio_s / elapsed
        ms_per_step = 1000.0 * elapsed / args.steps
        out = {
            "metric": "sec-audio enhanced/sec/GPU + xRT, UNIVERSE++ 16 kHz 8 s clips @1/2/4/8 GPU",
            "bench_config": args.config,
            "value": round(value, 3),
            "unit": "audio-s/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (16 kHz harmonic+noise clips, seeded synthetic weights)",
            "config": {"workload": C["workload"],
                       "model": {"pp16": "UniverseGAN PP16 (42.85 M params)", "orig16": "Universe ORIG16 (43.0 M params)",
                                 "pp24": "UniverseGAN PP24 (107.5 M params)"}[C["arch"]],
                       "global_batch": world * B, "batch_per_gpu": B,
                       "clip_s": args.seconds, "n_steps": C["n_steps"] or 8,
                       "parallelism": f"utterance-shard x{world}"},
            "xrt_per_gpu": round(value / world, 3),
        }
        if prof is not None:
            # the roofline that binds ou_conv over one enhance: the larger of
            # FLOPs / MFMA peak and algorithmic bytes / HBM peak
            t_mfma = prof["conv_flops"] / (peak * 1e12)
            t_hbm = prof["conv_bytes"] / (HBM_PEAK * 1e9)
            sec = prof["conv_ms"] * 1e-3
            tflops, gbps = prof["conv_flops"] / sec / 1e12, prof["conv_bytes"] / sec / 1e9
            traffic, tsrc = None, None
            if args.traffic_json and os.path.exists(args.traffic_json):
                with open(args.traffic_json) as fh:
                    pmc = json.load(fh)
                row = pmc.get("kernels", {}).get("conv_kernel")
                if row:
                    traffic = row["traffic_bytes_per_launch"]
                    per = "kernel dispatch"
                    if pmc.get("enhances_profiled"):
                        # per recorded conv op (K-slice ops dispatch twice)
                        traffic = round(traffic * row["dispatches"] / pmc["enhances_profiled"] / prof["n_conv"])
                        per = "ou_conv op (both launches of K-slice ops)"
                    tsrc = (f"{os.path.relpath(args.traffic_json, HERE)} ({pmc.get('tag', '')}): "
                            f"rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, bytes per {per}")
            if t_hbm > t_mfma:
                rl = {"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM_PEAK, "peak_basis": "HBM3E",
                      "unit": "GB/s", "frac": round(gbps / HBM_PEAK, 4),
                      "mfma": {"achieved": round(tflops, 3), "peak": peak, "unit": "TFLOP/s",
                               "frac": round(tflops / peak, 4), "peak_basis": peak_basis}}
            else:
                rl = {"bound": "mfma", "achieved": round(tflops, 3), "peak": peak, "peak_basis": peak_basis,
                      "unit": "TFLOP/s", "frac": round(tflops / peak, 4),
                      "hbm": {"achieved": round(gbps, 1), "peak": HBM_PEAK, "unit": "GB/s",
                              "frac": round(gbps / HBM_PEAK, 4)}}
            out["roofline"] = {
                **rl, "traffic": traffic,
                "traffic_source": tsrc,
                "kernel": "ou_conv (conv_kernel, all launches of one enhance)",
                "launches": prof["n_conv"],
                "avg_launch_ms": round(prof["conv_ms"] / prof["n_conv"], 5),
                "flops_per_launch": round(prof["conv_flops"] / prof["n_conv"]),
                "algorithmic_bytes_per_launch": round(prof["conv_bytes"] / prof["n_conv"]),
            }
            out["profile"] = {
                "enhance_device_ms": round(prof["total_ms"], 3),
                "conv_ms": round(prof["conv_ms"], 3),
                "gru_ms": round(prof["gru_ms"], 3),
                "other_ms": round(prof["total_ms"] - prof["conv_ms"] - prof["gru_ms"], 3),
                "algorithmic_gflop_per_clip": round(prof["total_flops"] / 1e9, 2),
                "e2e_tflops": round(prof["total_flops"] / (ms_per_step * 1e-3) / 1e12, 3),
                "ops": prof["n_ops"],
            }
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
