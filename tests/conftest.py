import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    # under pytest-xdist, share the cores between workers (the oracle's torch
    # ops oversubscribe badly otherwise)
    n = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "0") or 0)
    if n > 1:
        import torch

        torch.set_num_threads(max(1, (os.cpu_count() or 1) // n))


def load_golden(tag):
    with np.load(os.path.join(GOLDEN, f"{tag}.npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def golden_state_dict(d, seed=0):
    """Synthetic weights for the golden manifest (same generator the fixture
    script applied to the reference model)."""
    from open_universe_amd.utils.synthetic import synth_state_dict

    spec = [(n, [int(s) for s in sh.split(",") if s != ""])
            for n, sh in zip(d["manifest_names"], d["manifest_shapes"])]
    rc_gain = float(d["synth_rc_gain"]) if "synth_rc_gain" in d else 1.0   # the damped family (pp24d)
    return synth_state_dict([(n, s) for n, s in spec if not n.startswith("loss_")], seed, rc_gain)


def rel_rms(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b**2)), 1e-30))


def si_sdr(est, ref):
    """Scale-invariant SDR in dB (closed form, fast_bss_eval zero_mean=False,
    reference metrics/wrapper.py:197-213), over the flattened signals."""
    est = np.asarray(est, dtype=np.float64).ravel()
    ref = np.asarray(ref, dtype=np.float64).ravel()
    a = np.dot(est, ref) / max(np.dot(ref, ref), 1e-30)
    e = est - a * ref
    return float(10 * np.log10(max(np.dot(a * ref, a * ref), 1e-30) / max(np.dot(e, e), 1e-30)))


@pytest.fixture
def golden():
    return load_golden
