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
    cmd = [CLANG, "-std=c++17", "-Wno-psabi", *flags, "-I", EMU, "-x", "c++", os.path.join(EMU, src), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]


def _run(cmd, env=None, timeout=900):
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", **(env or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


ASAN = ("-O0", "-g0", "-fsanitize=address", "-fno-omit-frame-pointer")


def test_conv_tiles_in_bounds(tmp_path):
    """Every ou_conv tile of the chunked kernel, and every register-streamed
    (conv_rkernel, tile bit 14) shape on ragged / 1-step / deep / frame-view /
    K-chunked (st_conv) geometries, split-f16 and f16."""
    exe = str(tmp_path / "conv_emu")
    _build("conv_emu.cpp", exe, *ASAN)
    out = _run([exe])
    assert "ok:" in out and "(0 register-streamed)" not in out


def test_fused_block_in_bounds(tmp_path):
    """ou_block at 32 / 64 / 128 channels, split-f16 and f16, every epilogue
    the dispatcher instantiates (FiLM, input_cond, cond_out, res2, kEpiIn,
    kEpiHead, kEpiDown at rates 2 and 4) and ragged lengths."""
    exe = str(tmp_path / "block_emu")
    _build("block_emu.cpp", exe, *ASAN)
    assert "ok:" in _run([exe])


def _mutant(tmp_path, src, old, new):
    """A copy of csrc/<src> with one edit, laid out so its relative includes
    resolve (ou_common.h beside it, include/ouhip.h two levels up)."""
    import shutil

    d = tmp_path / "m" / "a" / "csrc"
    d.mkdir(parents=True)
    (tmp_path / "m" / "include").mkdir()
    shutil.copy(os.path.join(ROOT, "open_universe_amd", "csrc", "ou_common.h"), d)
    shutil.copy(os.path.join(ROOT, "include", "ouhip.h"), tmp_path / "m" / "include")
    text = open(os.path.join(ROOT, "open_universe_amd", "csrc", src)).read()
    assert old in text, old
    (d / src).write_text(text.replace(old, new, 1))
    return str(d / src)


def _must_fail(cmd, env=None):
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", **(env or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=e)
    # raw pointer overruns: AddressSanitizer; buffer-resource overruns: the
    # shim's range check (voffset + soffset past the resource)
    assert r.returncode != 0 and ("AddressSanitizer" in r.stderr or "EMU:" in r.stderr), (r.stdout[-1000:],
                                                                                           r.stderr[-2000:])


def test_emulator_catches_the_reverted_rkernel_clamp(tmp_path):
    """The round-2 GPU fault (commit b31c724): a conv_rkernel wave with no K
    steps read the weight ring below its range.  The K loop now guards its
    prologue with n > 0 (the clamped step index min(j, n - 1) is -1 without
    it); with the guard removed the emulator must report the read."""
    src = _mutant(tmp_path, "ou_conv.hip", "        if (n > 0) {   // uniform; clamped",
                  "        if (true) {   // uniform; clamped")
    exe = str(tmp_path / "conv_emu_rev")
    _build("conv_emu.cpp", exe, *ASAN, f'-DOU_EMU_CONV_SRC="{src}"')
    _must_fail([exe, "12"], env={"OUHIP_EMU_RS_ONLY": "1"})


def test_emulator_catches_an_unclamped_block_read(tmp_path):
    """ou_block stages PReLU(h) through a buffer resource: frames outside the
    clip take the sentinel voffset (range-checked, they load 0), the channel
    rows are scalar soffsets, which the hardware does NOT range-check.  A
    staging read one channel group past the tensor (the last group's rows
    shifted by 8) must be reported by the emulator."""
    src = _mutant(tmp_path, "ou_block.hip", "__builtin_amdgcn_raw_buffer_load_b32(hrs, vo, i * hcs * 4, 0)",
                  "__builtin_amdgcn_raw_buffer_load_b32(hrs, vo, (i + 8) * hcs * 4, 0)")
    exe = str(tmp_path / "block_emu_rev")
    _build("block_emu.cpp", exe, *ASAN, f'-DOU_EMU_BLOCK_SRC="{src}"')
    _must_fail([exe])


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
    # plain k3 batch 2 (and k5: both with the register-streamed kernel);
    # 1x1 with FiLM and two residuals; transposed conv;
    # channel-major rows at 2 / 4 / 8 phases (8-B / 16-B epilogue) -- one
    # process each, run side by side
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    procs = [subprocess.Popen([exe, g], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
             for g in ("0", "2", "4", "7", "8", "9", "11")]
    for p in procs:
        out, err = p.communicate(timeout=900)
        assert p.returncode == 0 and "ok:" in out, (out[-2000:], err[-2000:])


def test_block_values_match_reference(tmp_path):
    """Fiber emulation of ou_block against a double-precision evaluation of
    the ConvBlock formula at 32 / 48 / 64 / 96 / 128 / 192 channels (48:
    padded MFMA rows), split-f16 and f16, FiLM / input_cond / cond_out /
    res2, whole-signal and on frame ranges (garbage h outside [h0, h1))."""
    exe = str(tmp_path / "block_emu_values")
    _build("block_emu_values.cpp", exe, "-O0", "-DOU_EMU_FIBERS")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    procs = [subprocess.Popen([exe, str(g)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
             for g in range(6)]
    for p in procs:
        out, err = p.communicate(timeout=1200)
        assert p.returncode == 0 and "ok:" in out, (out[-2000:], err[-2000:])


def test_split_image_values_match_reference(tmp_path):
    """Fiber emulation of the split-image path, under AddressSanitizer: the
    consumer kernel (tile bit 15) against a double-precision evaluation at
    every NR shape (k1/k3/k5, frame views at rates 4 and 5, a transposed
    channel-major output, a one-chunk layer whose other waves run zero
    chunks), and the split image every producer kernel family stores
    (ou_conv_desc.sy) against prelu(y) * 2^-s element by element."""
    exe = str(tmp_path / "conv_emu_split")
    _build("conv_emu_split.cpp", exe, *ASAN, "-DOU_EMU_FIBERS")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    procs = [subprocess.Popen([exe, g], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
             for g in ("0", "1", "2", "3", "4", "5", "6", "100")]
    for p in procs:
        out, err = p.communicate(timeout=900)
        assert p.returncode == 0 and "ok:" in out, (out[-2000:], err[-2000:])


def test_fir_values_match_reference(tmp_path):
    """Fiber emulation of the FIR-applied rate-change kernels (tile bit 17,
    conv_fdkernel / conv_fukernel), under AddressSanitizer: every OU_FTILES
    shape (and the m-major order), split-f16 and f16, down (FIR before the
    strided conv; ragged lengths, FiLM, the split-image output) and up (FIR
    after the transposed conv; residuals, FiLM, a cropped output, valid_len
    zero-fill) against a double-precision evaluation of the reference's op
    order, at every rate the configs use (2, 3, 4, 5, 8); and the same
    kernel without the FIR for the st_convs (fir 3: kernel = stride = 20, 24,
    40; chunks of 4 / 8 phases)."""
    exe = str(tmp_path / "conv_emu_fir")
    _build("conv_emu_fir.cpp", exe, *ASAN, "-DOU_EMU_FIBERS")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    procs = [subprocess.Popen([exe, r], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
             for r in ("2", "3", "4", "5", "8", "st")]
    for p in procs:
        out, err = p.communicate(timeout=900)
        assert p.returncode == 0 and "ok:" in out, (out[-2000:], err[-2000:])
