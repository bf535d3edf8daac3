#!/usr/bin/env python
"""Benchmark: seconds of audio enhanced per second, UNIVERSE++ 16 kHz, 8 s clips.

    python bench.py [--gpus N] [--steps K] [--warmup W]

One step = one ``model.enhance()`` of one synthetic 8 s clip at batch 1
(BASELINE.json configs[1]: "UNIVERSE++ 16 kHz, batch=1, 8 s clips"), run as
the production path does it: one hipGraph replay of the recorded sampler
(conditioner + 8 score-network passes + sampler updates).  Every rank (one
process per GPU) enhances its own clips -- utterances shard across GPUs with
no collective on the data path -- so scaling is weak; ``value`` is the
whole-job audio-seconds per second: N * K * 8 s / max-over-ranks time
(``value_per_gpu`` = value / N, the per-GPU figure the metric names).

Ranks: under torchrun (WORLD_SIZE set) this process is one rank.  Without it,
``--gpus N`` (N > 1) starts the N rank processes itself before touching the
GPU (``launch_ranks``), each with the torchrun environment, and waits for them.

Extra fields:
  roofline      the dominant kernel (ou_conv, every launch of one enhance):
                algorithmic FLOPs of the reference ops it replaces and
                algorithmic bytes (activations once, f32 weights) over its
                device time, measured with HIP events per launch in an
                instrumented eager replay of the same enhance on the same
                stream; the bound is whichever of FLOPs/MFMA peak and
                bytes/HBM peak is larger.
  cpu_baseline  the CPU restatement of the reference op sequence (oracle/,
                plain PyTorch) on this host's cores, bounded sample, B = 1
                and the config's B.
  f32_value     (c2) a second timed pass with f32 conv operands, beside the
                default split-f16 operand build.
  queued_value  (c2) the same batch-1 clips with two enhances in flight on
                two streams (a queue of batch-1 requests); not the headline.
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
# the kernels of the conv stack (roofline.traffic sums their PMC bytes)
CONV_STACK_KERNELS = ("conv_kernel", "conv_rkernel", "conv_skernel", "conv_rreduce", "conv_fdkernel", "conv_fukernel",
                      "block_kernel")
HBM_PEAK = 8000.0      # GB/s


def lib_sha16():
    """Hash of the libouhip.so this process loads (ties PMC counters to a build)."""
    import hashlib

    from open_universe_amd import _lib as L

    with open(L.LIB_PATH, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


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
    "c1": dict(arch="pp16", batch=1, seconds=4.0, n_steps=None,
               workload="UNIVERSE++ 16 kHz enhance(), batch=1, one 4 s clip, 8 diffusion steps (BASELINE.json "
                        "configs[0]: the reference's CPU-only case; here on the GPU, the oracle's CPU time beside it)"),
    "c2": dict(arch="pp16", batch=1, seconds=8.0, n_steps=None,
               workload="UNIVERSE++ 16 kHz enhance(), batch=1, 8 s clip, 8 diffusion steps (BASELINE.json configs[1])"),
    "c3": dict(arch="orig16", batch=8, seconds=8.0, n_steps=60,
               workload="UNIVERSE (original) 16 kHz enhance(), batch=8, 8 s clips, 60 diffusion steps "
                        "(BASELINE.json configs[2])"),
    # c4 runs the damped synthetic family (utils/synthetic.py RC_DAMP): with
    # g ~ 1 on the anti-aliased rate changes PP24's activations reach 7.7e6 in
    # the reference itself and the split-f16 operands would fall back to f32
    "c4": dict(arch="pp24", batch=32, seconds=10.0, n_steps=None, node_batch=True, damped=True,
               workload="UNIVERSE++ 24 kHz enhance(), batch=32 per node sharded over the GPUs, 10 s clips, "
                        "8 diffusion steps (BASELINE.json configs[3]); damped synthetic weights"),
    "c5": dict(arch="pp16", batch=1, seconds=60.0, n_steps=None, conv_prec="f16",
               workload="UNIVERSE++ 16 kHz enhance(), batch=1, 60 s long-form clip, 8 diffusion steps, fp16 conv "
                        "operands, whole sampler captured in one hipGraph (BASELINE.json configs[4])"),
}


def default_traffic_json(config):
    """The PMC summary bench quotes `traffic` from (tools/gpu_profile.sh):
    profiles/pmc_latest.json for the headline config, pmc_latest_<config>.json
    for the others."""
    return os.path.join(HERE, "profiles", "pmc_latest.json" if config == "c2" else f"pmc_latest_{config}.json")


def build_model(device, nch=None, seed=0, arch="pp16", damped=False):
    import torch

    from open_universe_amd.configs import get_config
    from open_universe_amd.networks.universe import Universe, UniverseGAN
    from open_universe_amd.utils.synthetic import RC_DAMP, synth_state_dict

    cfg = get_config(arch, nch)
    cls = Universe if cfg["_target_"].endswith(".Universe") else UniverseGAN
    m = cls(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()], seed,
                                       RC_DAMP if damped else 1.0), strict=False)
    return cfg, m.to(device).eval()


def available_cpus():
    """CPUs this process may use: os.cpu_count(),
    bounded by the affinity mask and the cgroup CPU quota when either is
    smaller (a GPU box shares its host: os.cpu_count() shows the whole
    machine, the quota is this job's share)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    if quota:
        n = min(n, max(1, int(math.ceil(quota))))
    return n, quota


# CPU sample per config: (clip seconds at B=1, clip seconds at the config's B).
# Bounded so each leg is a few seconds of oracle work (c2: the full 8 s clip).
# clip seconds of the B=1 leg and of the config-B leg (None: no config-B leg;
# C3 / C4 time one full-length clip instead of short clips at the config's B)
CPU_SAMPLE = {"c1": (4.0, 4.0), "c2": (8.0, 8.0), "c3": (8.0, None), "c4": (10.0, None), "c5": (8.0, 8.0)}


def cpu_baseline(model, cfg, C, config_name):
    """The oracle (CPU restatement of the reference ops, oracle/ou_oracle.py)
    on a bounded sample of the workload: B=1 and the config's B, one warm-up
    then best of 3 (best of 2 for the 60-step full-length clip; BASELINE.md
    section 3).  The headline ``value`` is the config-B leg, or for C3 / C4
    the B=1 leg on the config's full clip length (the B=1 leg is reported
    beside it)."""
    import numpy as np
    import torch

    from oracle import ou_oracle
    from open_universe_amd.utils.synthetic import synth_audio

    threads, quota = available_cpus()
    torch.set_num_threads(threads)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    orc = ou_oracle.Oracle(sd, cfg)
    fs = int(cfg["fs"])
    ekw = {"n_steps": C["n_steps"]} if C["n_steps"] else {}
    legs = {}
    s1, sB = CPU_SAMPLE[config_name]
    Bc = C["batch"]
    for B, secs in ((1, s1), (Bc, sB)):
        if B in legs or secs is None:
            continue
        runs = 3 if secs * (C["n_steps"] or 8) >= 400 else 4
        T = int(secs * fs)
        mix = torch.from_numpy(np.stack([synth_audio(T, fs, 99 + j)[0] for j in range(B)]))
        best = float("inf")
        with torch.no_grad():
            for i in range(runs):
                t0 = time.perf_counter()
                orc.enhance(mix, rng=torch.Generator().manual_seed(1028282), **ekw)
                dt = time.perf_counter() - t0
                if i > 0:
                    best = min(best, dt)
        legs[B] = {"value": round(B * secs / best, 4), "batch": B, "clip_s": secs, "best_s": round(best, 3)}
    head = legs[Bc] if sB is not None else legs[1]
    return {"value": head["value"], "unit": "audio-s/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "cpu_quota": quota, "legs": list(legs.values()),
            "sample": f"oracle/ou_oracle.py Oracle.enhance ({C['arch']}, {C['n_steps'] or 8} steps, fp32), "
                      f"torch.set_num_threads({threads}); value = the B={head['batch']} leg ({head['clip_s']:g} s clips)"
                      + (", B=1 leg in legs" if sB is not None else
                         f", the config's full clip length; its B={Bc} batch is not run on the CPU")
                      + f"; 1 warm-up + best of the rest per leg; {cpu_model()}"}


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
    # the conv stack: ou_conv launches and fused ConvBlock (ou_block) launches
    cv = (L.OP_CONV, L.OP_BLOCK)
    conv_ms = sum(t for t, k in zip(ms, kinds) if k in cv)
    conv_fl = sum(f for f, k in zip(flops, kinds) if k in cv)
    conv_by = sum(b for b, k in zip(plan.prog.bytes, kinds) if k in cv)
    n_conv = sum(1 for k in kinds if k in cv)
    n_block = sum(1 for k in kinds if k == L.OP_BLOCK)
    gru_ms = sum(t for t, k in zip(ms, kinds) if k == L.OP_GRU)
    return {
        "conv_ms": conv_ms, "conv_flops": conv_fl, "conv_bytes": conv_by, "n_conv": n_conv, "n_block": n_block,
        "gru_ms": gru_ms,
        "total_ms": sum(ms), "total_flops": sum(flops), "n_ops": len(ms),
    }


def launch_ranks(n, argv):
    """``bench.py --gpus N`` without an outer torchrun: start N rank processes
    (one per GPU) before anything in this parent touches the GPU, wait for
    them and return the worst exit code.  Each child gets the torchrun
    environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1,
    MASTER_PORT) and joins the gloo barrier / max-over-ranks like a torchrun
    rank; rank 0 prints the JSON line."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    try:
        for p in procs:
            rc = max(rc, p.wait())
            if rc:
                break
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    return rc


def rank_batch(C, world):
    """Clips per rank: the config's batch per GPU, or (node_batch configs, C4)
    the whole-node batch split into equal contiguous shards (equal-length clips;
    sharding.shard_utterances gives the same split)."""
    if not C.get("node_batch"):
        return C["batch"]
    if C["batch"] % world:
        raise ValueError(f"{C['batch']} clips do not shard evenly over {world} ranks")
    return C["batch"] // world


def timed_loop(step, warmup, steps, world, sync):
    """W untimed steps, then K steps bracketed by barrier + device sync; the
    elapsed time is the max over ranks."""
    import torch.distributed as dist

    from open_universe_amd.sharding import max_over_ranks

    for i in range(warmup):
        step(i)
    sync()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    sync()
    if world > 1:
        dist.barrier()
    return max_over_ranks(time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="BASELINE.json config (c2 = configs[1], the headline)")
    ap.add_argument("--seconds", type=float, default=None, help="override the config's clip length")
    ap.add_argument("--batch", type=int, default=None,
                    help="clips per rank, overriding the config's (c4 at 16/8/4 on one GPU = the per-rank "
                         "shard at 2/4/8 GPUs)")
    ap.add_argument("--undamped", action="store_true",
                    help="c4: the undamped synthetic weights (activations past the default split-f16 range; "
                         "the warm-up widens the named layers' exponents, the line reports `widenings`)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-queued", action="store_true",
                    help="skip the extra leg with batch-1 enhances in flight on several streams (queued_value)")
    ap.add_argument("--queued-streams", type=int, default=2, help="streams of the queued leg")
    ap.add_argument("--no-f32-pass", action="store_true",
                    help="skip the second timed pass with f32 conv operands (f32_value)")
    ap.add_argument("--dump-ops", default=None, help="write per-op profile rows (JSON)")
    ap.add_argument("--traffic-json", default=None,
                    help="per-kernel HBM traffic from tools/pmc_summary.py (rocprofv3 PMC passes); default "
                         "profiles/pmc_latest.json for c2, profiles/pmc_latest_<config>.json for the others")
    ap.add_argument("--stub-ms", type=float, default=None, help=argparse.SUPPRESS)  # CPU test of the launcher
    args = ap.parse_args()
    if args.traffic_json is None:
        args.traffic_json = default_traffic_json(args.config)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import numpy as np
    import torch
    import torch.distributed as dist

    from open_universe_amd.sharding import dist_env
    from open_universe_amd.utils.synthetic import synth_audio

    rank, local, world = dist_env()
    if world > 1:
        # gloo's C++ side prints its "[Gloo] Rank r is connected ..." lines to
        # stdout; stdout carries only rank 0's JSON line, so they go to stderr
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    if world != args.gpus and rank == 0:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: reporting {world}", file=sys.stderr)
    C = CONFIGS[args.config]
    if args.seconds is None:
        args.seconds = C["seconds"]
    B = rank_batch(C, world) if args.batch is None else args.batch

    if args.stub_ms is not None:
        # launcher/control-plane test without a GPU: a step is a sleep
        elapsed = timed_loop(lambda i: time.sleep(args.stub_ms * 1e-3), args.warmup, args.steps, world,
                             lambda: None)
        if rank == 0:
            print(json.dumps({"metric": "stub", "value": world * B * args.steps * args.seconds / elapsed,
                              "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                              "ms_per_step": 1000.0 * elapsed / args.steps,
                              "config": {"global_batch": world * B, "batch_per_gpu": B}}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    # one rank per GPU; more ranks than GPUs (a rehearsal of the N-rank path on
    # a smaller box) share devices round-robin.  device_count() does not
    # initialise the GPU.
    ndev = torch.cuda.device_count()
    gpu = local % ndev if ndev else local
    if ndev and world > ndev and rank == 0:
        print(f"[bench] {world} ranks on {ndev} GPU(s): ranks share devices round-robin (rehearsal, not a "
              f"scaling measurement)", file=sys.stderr)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if C.get("conv_prec") and "OUHIP_CONV_PREC" not in os.environ:
        os.environ["OUHIP_CONV_PREC"] = C["conv_prec"]
    damped = C.get("damped", False) and not args.undamped
    cfg, model = build_model(dev, arch=C["arch"], damped=damped)
    fs = int(cfg["fs"])
    T = int(args.seconds * fs)
    n_clips = args.warmup + args.steps
    clips = [torch.from_numpy(np.stack([synth_audio(T, fs, rank * 100003 + i * 97 + j)[0] for j in range(B)]))
             .to(dev) for i in range(min(n_clips, 4))]
    rng = torch.Generator(device=dev).manual_seed(1028282 + rank)
    ekw = {"n_steps": C["n_steps"]} if C["n_steps"] else {}
    sync = lambda: torch.cuda.synchronize(dev)

    with torch.no_grad():
        elapsed = timed_loop(lambda i: model.enhance(clips[i % len(clips)], rng=rng, **ekw),
                             args.warmup, args.steps, world, sync)

    prof = None
    if not args.no_profile:
        plan = next(iter(model._plans.values()))
        with torch.no_grad():
            plan.MIX.copy_(clips[0].reshape(plan.MIX.shape))
            plan.draw_noise(rng)
            prof = profile_roofline(plan, torch.cuda.current_stream(dev).cuda_stream, args.dump_ops)

    prec = model._get_engine().conv_prec
    fallbacks = model.range_fallbacks   # timed-loop enhances rerun with f32 operands (OuRangeError)
    # the strictly-f32 figure: a second timed pass with f32 conv operands
    f32 = None
    # (c2 only: at c4 the split-f16 model's arena, split images included, and
    # an f32 model's no longer fit one GPU's 288 GB together)
    if prec != 0 and not args.no_f32_pass and args.config == "c2":
        _, m32 = build_model(dev, arch=C["arch"], damped=damped)
        m32._conv_prec = 0
        with torch.no_grad():
            e32 = timed_loop(lambda i: m32.enhance(clips[i % len(clips)], rng=rng, **ekw),
                             args.warmup, args.steps, world, sync)
        assert m32._get_engine().conv_prec == 0
        f32 = {"value": round(world * B * args.steps * args.seconds / e32, 3),
               "ms_per_step": round(1000.0 * e32 / args.steps, 3)}
        del m32

    # extra leg: the same B=1 clips with two enhances in flight on two streams
    # (Universe.enhance_many) -- the throughput of a queue of batch-1
    # requests; the headline value above stays strictly one clip at a time
    queued = None
    if args.config == "c2" and not args.no_queued and not C["n_steps"]:
        seq = [clips[i % len(clips)] for i in range(args.steps)]
        with torch.no_grad():
            qs = args.queued_streams
            model.enhance_many(seq[: max(2 * qs, args.warmup)], rng=rng, streams=qs)
            eq = timed_loop(lambda i: model.enhance_many(seq, rng=rng, streams=qs), 0, 1, world, sync)
        queued = {"streams": qs, "clips": args.steps,
                  "value": round(world * B * args.steps * args.seconds / eq, 3),
                  "ms_per_clip": round(1000.0 * eq / args.steps, 3)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(model, cfg, C, args.config)

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
            "value_semantics": "whole job: audio-seconds enhanced by all n_gpus ranks / max-over-ranks wall "
                               "time (bench contract); the per-GPU figure the metric names is value_per_gpu",
            "value_per_gpu": round(value / world, 3),
            "n_gpus": world,
            **({"gpus_visible": ndev, "ranks_share_gpus": True} if ndev and world > ndev else {}),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (harmonic+noise clips, seeded synthetic weights%s)"
                    % (", damped family" if damped else (", undamped family" if C.get("damped") else "")),
            "config": {"workload": C["workload"],
                       "model": {"pp16": "UniverseGAN PP16 (42.85 M params)", "orig16": "Universe ORIG16 (43.0 M params)",
                                 "pp24": "UniverseGAN PP24 (107.5 M params)"}[C["arch"]],
                       "global_batch": world * B, "batch_per_gpu": B,
                       "clip_s": args.seconds, "n_steps": C["n_steps"] or 8,
                       "parallelism": f"utterance-shard x{world}"},
            "xrt_per_gpu": round(value / world, 3),
            "fallbacks": fallbacks,
            "widenings": model.range_widenings,
            "fallbacks_note": "widenings: enhance() calls of the timed loop (and warm-up) rerun after a split-f16 "
                              "range flag widened the staging exponents of the layers it named (those layers only; "
                              "they keep the wider exponent); fallbacks: calls rerun with f32 operands because no "
                              "widening fixed the range (after one, the model stays on f32)",
        }
        if args.batch is not None:
            out["config"]["batch_override"] = True
        if queued is not None:
            out["queued_value"] = queued["value"]
            out["queued"] = {**queued, "note": "extra leg: the same batch-1 clips, enhance() calls in flight "
                                               "on several HIP streams (Universe.enhance_many)"}
        if f32 is not None:
            out["f32_value"] = f32["value"]
            out["f32_pass"] = {**f32, "dtype": "f32 (v_mfma_f32_32x32x2_f32 conv operands)",
                               "steps": args.steps, "warmup": args.warmup}
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
                rows = [r for k, r in pmc.get("kernels", {}).items()
                        if k in CONV_STACK_KERNELS]
                lib_now = lib_sha16()
                if pmc.get("lib_sha16") != lib_now:
                    # counters of another build of the kernels: not quoted
                    rows = []
                    tsrc = (f"null: {os.path.relpath(args.traffic_json, HERE)} was counted on libouhip.so "
                            f"{pmc.get('lib_sha16')}, this run loads {lib_now} (re-run tools/gpu_profile.sh)")
                elif pmc.get("config", "c2") != args.config:
                    tsrc = f"null: the PMC passes profiled --config {pmc.get('config', 'c2')}, not {args.config}"
                if rows and pmc.get("config", "c2") == args.config and pmc.get("enhances_profiled"):
                    # bytes of every conv-stack dispatch of one enhance, per
                    # recorded conv op (K-slice ops dispatch twice)
                    tot = sum(r["traffic_bytes_per_launch"] * r["dispatches"] for r in rows)
                    traffic = round(tot / pmc["enhances_profiled"] / prof["n_conv"])
                    per = "conv-stack op (ou_conv incl. both launches of K-slice ops, ou_block)"
                    tsrc = (f"{os.path.relpath(args.traffic_json, HERE)} ({pmc.get('tag', '')}, libouhip.so "
                            f"{lib_now}, the library this run loaded): rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, "
                            f"bytes per {per}")
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
                "kernel": "conv stack: ou_conv (conv_kernel, conv_rkernel + conv_rreduce, conv_skernel, the "
                          "FIR-applied rate-change conv_fdkernel / conv_fukernel) + fused ConvBlock ou_block "
                          "(block_kernel), all launches of one enhance",
                "launches": prof["n_conv"],
                "fused_block_launches": prof["n_block"],
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
