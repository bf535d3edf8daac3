"""CPU emulation of the HIP kernels (tests/emu): the ou_conv source compiled
for the host against a bounds-checking shim and run under AddressSanitizer
(addresses), and under a fiber scheduler that reproduces barriers and the
wave-wide MFMA (values).  No GPU involved: this is how a kernel change is
checked for out-of-bounds accesses before it ever runs on a device."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
EMU = os.path.join(HERE, "emu")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"

pytestmark = pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang++ not present")


def _build(src, out, *flags):
    cmd = [CLANG, "-std=c++17", *flags, "-I", EMU, "-x", "c++", os.path.join(EMU, src), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]


def _run(cmd, env=None, timeout=900):
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", **(env or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


ASAN = ("-O0", "-g0", "-fsanitize=address", "-fno-omit-frame-pointer")


def test_conv_tiles_in_bounds(tmp_path):
    exe = str(tmp_path / "conv_emu")
    _build("conv_emu.cpp", exe, *ASAN)
    assert "ok:" in _run([exe])


def test_recorded_plan_convs_in_bounds(tmp_path):
    """Every conv descriptor of a recorded enhance program (small-channel
    UNIVERSE++ config, batch 2), every tile shape x tiles-per-workgroup."""
    plan = str(tmp_path / "plan.txt")
    r = subprocess.run(["python", os.path.join(EMU, "dump_plan_convs.py"), plan, "pp16", "8", "2", "4000"],
                       capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    exe = str(tmp_path / "conv_emu_plan")
    _build("conv_emu_plan.cpp", exe, *ASAN)
    n = 4   # descriptor shards, one process each, run side by side
    procs = [subprocess.Popen([exe, plan], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0", OUHIP_EMU_BLOCKS="2",
                                       OUHIP_EMU_SHARD=f"{i}/{n}"))
             for i in range(n)]
    for p in procs:
        out, err = p.communicate(timeout=900)
        assert p.returncode == 0 and "ok:" in out, (out[-2000:], err[-4000:])


def test_conv_values_match_reference(tmp_path):
    """Fiber emulation: every tile configuration against a double-precision
    evaluation of the ou_conv_desc formula (include/ouhip.h)."""
    exe = str(tmp_path / "conv_emu_values")
    # -O0: -O1 spends minutes compiling every kernel instantiation for the host
    _build("conv_emu_values.cpp", exe, "-O0", "-DOU_EMU_FIBERS")
    # plain k3 batch 2; 1x1 with FiLM and two residuals; transposed conv -- one
    # process each, run side by side
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    procs = [subprocess.Popen([exe, g], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
             for g in ("0", "4", "7")]
    for p in procs:
        out, err = p.communicate(timeout=900)
        assert p.returncode == 0 and "ok:" in out, (out[-2000:], err[-2000:])
