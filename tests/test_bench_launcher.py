"""bench.py's multi-GPU entry point on CPU: ``--gpus 2`` without torchrun
starts two rank processes itself (gloo barrier + max-over-ranks), and the C4
node batch of 32 clips shards 16 + 16.  The workload is a stub (a sleep per
step), so no GPU is touched."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    # the bench contract: stdout is rank 0's one JSON line and nothing else
    # (gloo's connection messages and the ranks' logs go to stderr)
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    return json.loads(lines[0])


def test_two_ranks_self_launched_c4_shards():
    out = _run("--gpus", "2", "--steps", "3", "--warmup", "1", "--stub-ms", "2", "--config", "c4")
    assert out["n_gpus"] == 2
    assert out["config"]["batch_per_gpu"] == 16 and out["config"]["global_batch"] == 32


def test_single_rank_default():
    out = _run("--steps", "2", "--warmup", "1", "--stub-ms", "1")
    assert out["n_gpus"] == 1 and out["config"]["batch_per_gpu"] == 1


def test_rank_batch():
    sys.path.insert(0, REPO)
    import bench

    assert bench.rank_batch(bench.CONFIGS["c4"], 8) == 4
    assert bench.rank_batch(bench.CONFIGS["c3"], 8) == 8
    try:
        bench.rank_batch(bench.CONFIGS["c4"], 3)
    except ValueError:
        pass
    else:
        raise AssertionError("32 clips over 3 ranks must be refused")


def test_default_traffic_json_per_config():
    """bench quotes `traffic` from the PMC summary of its own config: the
    headline's pmc_latest.json, pmc_latest_<config>.json otherwise; the
    committed files carry the library hash they were counted on."""
    sys.path.insert(0, REPO)
    import bench

    assert bench.default_traffic_json("c2").endswith(os.path.join("profiles", "pmc_latest.json"))
    assert bench.default_traffic_json("c4").endswith(os.path.join("profiles", "pmc_latest_c4.json"))
    for cfg in ("c2", "c4"):
        with open(bench.default_traffic_json(cfg)) as fh:
            doc = json.load(fh)
        assert doc["config"] == cfg and len(doc["lib_sha16"]) == 16 and doc["enhances_profiled"] >= 1
