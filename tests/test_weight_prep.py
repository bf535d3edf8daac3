"""CPU checks of the weight folding that feeds the HIP conv kernel.

The kernel computes (include/ouhip.h, ou_conv):
    xv[c'][t] = prelu(x[c'/R][t*R + c'%R + shift]);  acc[m][u] = sum W[m][c'][k] xv[c'][u+k-pad]
    then pixel shuffle (m = ph*cout + co -> t = u*rout + ph) and bias.
Here that formulation is emulated in float64 with the engine's logical
weights (ConvSpec) and compared with the oracle's restatement of the reference
op sequence (PReLU -> FIR -> strided conv, PReLU -> ConvTranspose -> FIR, ...).
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden_state_dict, load_golden
from open_universe_amd import engine as E
from open_universe_amd import dsp
from oracle import ou_oracle as O


def emulate(spec, x, n_frames, out_len, valid_len=None, in_scale=None):
    x = x.double()
    B, Cin, T = x.shape
    R, kt = spec.frame, spec.w.shape[2]
    ts = torch.arange(-spec.pad, n_frames - spec.pad + kt - 1)
    xv = torch.zeros(B, Cin * R, len(ts), dtype=torch.float64)
    for c in range(Cin * R):
        ci, p = divmod(c, R)
        pos = ts * R + p + spec.shift
        ok = (pos >= 0) & (pos < T)
        xv[:, c, ok] = x[:, ci, pos[ok]]
    if in_scale is not None:
        xv = xv * in_scale
    xv = torch.where(xv >= 0, xv, xv * spec.slope)
    acc = F.conv1d(xv, torch.from_numpy(np.asarray(spec.w, np.float64)))
    m = acc.shape[1]
    cout = m // spec.rout
    if spec.cm:   # channel-major rows m = co * rout + ph
        y = acc.reshape(B, cout, spec.rout, n_frames).permute(0, 1, 3, 2).reshape(B, cout, -1)
    else:         # phase-major rows m = ph * cout + co
        y = acc.reshape(B, spec.rout, cout, n_frames).permute(0, 2, 3, 1).reshape(B, cout, -1)
    if spec.bias is not None:
        y = y + torch.from_numpy(np.asarray(spec.bias, np.float64))[None, :, None]
    if valid_len is not None and valid_len < y.shape[-1]:
        y[..., valid_len:] = 0
    if y.shape[-1] < out_len:
        y = F.pad(y, (0, out_len - y.shape[-1]))
    return y[..., :out_len]


@pytest.fixture(scope="module")
def sd():
    d = load_golden("pp16_c4")
    return {k: v.double() for k, v in golden_state_dict(d).items()}


def _x(B, C, T, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, C, T, generator=g, dtype=torch.float64)


def test_binomial_taps_match_reference_values():
    # SURVEY.md 8(a) A9 (values from the reference's get_binomial_filter)
    np.testing.assert_allclose(dsp.binomial_taps(5)[:3], [0.267261, 1.069045, 1.603567], atol=1e-6)
    np.testing.assert_allclose(dsp.binomial_taps(11)[:4], [0.007716, 0.077161, 0.347224, 0.92593],
                               atol=1e-6)
    for k in (5, 7, 9, 11, 17):
        np.testing.assert_allclose(dsp.binomial_taps(k), O.get_binomial_filter(k).numpy(), rtol=1e-6)


@pytest.mark.parametrize("k,name", [(5, "conv1"), (3, "conv2")])
def test_same_conv(sd, k, name):
    p = f"_edm_model.encoder.ds_modules.1.{name}"
    x = _x(2, 8, 37)
    spec = E.spec_same(sd, p, k)
    y = emulate(spec, x, 37, 37)
    ref = O.prelu_conv(sd, p, x, k, padding="same")
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("lvl,r", [(0, 2), (1, 4), (3, 5)])
@pytest.mark.parametrize("T", [40, 43])
def test_down_conv_with_fir(sd, lvl, r, T):
    p = f"_edm_model.encoder.ds_modules.{lvl}.rate_change_conv"
    C = 4 * 2**lvl
    x = _x(2, C, T, seed=lvl)
    spec = E.spec_down(sd, p, r, True)
    U = -(-T // r)
    y = emulate(spec, x, U, U)
    ref = O.prelu_conv(sd, p, x, r, stride=r, antialias=True)
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("lvl,r", [(1, 5), (2, 4), (4, 2)])
@pytest.mark.parametrize("extra_len", [0, -3])
def test_up_conv_with_fir(sd, lvl, r, extra_len):
    p = f"_edm_model.decoder.up_modules.{lvl}.rate_change_conv"
    Cin = 2 * sd[p + ".conv.weight_v"].shape[1]
    Tin = 11
    x = _x(2, sd[p + ".conv.weight_v"].shape[0], Tin, seed=lvl)
    spec = E.spec_up(sd, p, r, True)
    length = r * Tin + extra_len
    y = emulate(spec, x, Tin, length, valid_len=r * Tin)
    ref = O.prelu_conv(sd, p, x, r, stride=r, transpose=True, antialias=True)
    ref = F.pad(ref, (0, length - ref.shape[-1]))
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-6)


def test_up_conv_plain(sd):
    p = "condition_model.decoder.up_modules.2.rate_change_conv"
    x = _x(1, sd[p + ".conv.weight_v"].shape[0], 9)
    spec = E.spec_up(sd, p, 4, False)
    y = emulate(spec, x, 9, 36)
    ref = O.prelu_conv(sd, p, x, 4, stride=4, transpose=True)
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("i,r", [(0, 160), (1, 80), (2, 20)])
def test_st_convs(sd, i, r):
    p = f"condition_model.encoder.st_convs.{i}"
    C = 4 * 2**i
    T = 3 * r + 7
    x = _x(1, C, T)
    spec = E.spec_down(sd, p, r, False)
    U = -(-T // r)
    y = emulate(spec, x, U, U)
    ref = O.prelu_conv(sd, p, x, r, stride=r)
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-6)


def test_mel_front_end_as_gemm():
    """STFT as a framed GEMM (R = hop, 4 frames) + |.|^2 + filterbank GEMM equals
    the (restated) torchaudio MelSpectrogram on the padded signal
    (condition.py:85-102)."""
    hop, nfft, nmels = 160, 640, 80
    T = 160 * 12
    x = _x(2, 1, T)
    pl = (nfft - hop) // 2
    nfreq = nfft // 2 + 1
    win = dsp.hann_periodic(nfft).astype(np.float64)
    n = np.arange(nfft)
    ang = 2 * math.pi * np.outer(np.arange(nfreq), n) / nfft
    dft = np.concatenate([win * np.cos(ang), win * np.sin(ang)], 0)
    wl = dft.reshape(2 * nfreq, nfft // hop, hop).transpose(0, 2, 1)
    spec = E.ConvSpec(wl, 1, hop, 0, 1, 1.0, None, shift=-pl)
    U = T // hop
    s = emulate(spec, x, U, U)
    power = s[:, :nfreq] ** 2 + s[:, nfreq:] ** 2
    fb = torch.from_numpy(dsp.melscale_fbanks(nfreq, 0.0, 12000.0, nmels, 24000).astype(np.float64))
    mel = torch.einsum("bft,fm->bmt", power, fb)
    xp = F.pad(x, (pl, nfft - hop - pl))
    ref = O.mel_spectrogram(xp, nfft, hop, nmels).squeeze(1)
    torch.testing.assert_close(mel, ref, rtol=5e-5, atol=1e-6)


def test_mel_fbank_matches_oracle():
    np.testing.assert_allclose(dsp.melscale_fbanks(321, 0.0, 12000.0, 80, 24000),
                               O.melscale_fbanks(321, 0.0, 12000.0, 80, 24000).numpy(),
                               rtol=1e-5, atol=1e-7)


def test_resample_kernels_match_oracle():
    for o, n in ((1, 2), (2, 1)):
        k, w = dsp.sinc_resample_kernel(o, n)
        k2, w2, _, _ = O._sinc_resample_kernel(o, n)
        assert w == w2
        np.testing.assert_allclose(k, k2.reshape(k.shape).numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("m,cin,kt", [(32, 32, 5), (64, 160, 3), (1536, 512, 1), (642, 160, 4), (50, 70, 3)])
def test_numpy_split_packing_matches_c(m, cin, kt):
    """The numpy restatements the engine uses are byte-identical to the C ABI
    packers (ou_conv_pack_split, ou_block_pack)."""
    import numpy as np

    from open_universe_amd import _lib as L

    g = np.random.default_rng(m + cin + kt)
    w = (g.standard_normal((m, cin, kt)) * 0.05).astype(np.float32)
    a, ua = L.conv_pack_split(w)
    b, ub = L.conv_pack_split_np(w)
    assert ua == ub and a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    if m == cin and m % 32 == 0:
        a, ua = L.block_pack(w)
        b, ub = L.block_pack_np(w)
        assert ua == ub and np.array_equal(a, b)


def test_numpy_block_packing_matches_c():
    import numpy as np

    from open_universe_amd import _lib as L

    # square block convs and the fused rate-change convs (2C x C x kt * rate)
    for m, c, kt in ((32, 32, 5), (64, 64, 3), (128, 128, 5), (64, 32, 6), (128, 64, 12), (64, 32, 2)):
        w = (np.random.default_rng(m + c + kt).standard_normal((m, c, kt)) * 0.03).astype(np.float32)
        a, ua = L.block_pack(w)
        b, ub = L.block_pack_np(w)
        assert ua == ub and np.array_equal(a, b)


@pytest.mark.parametrize("C,kt", [(32, 5), (48, 3), (64, 3), (96, 5), (192, 3)])
def test_numpy_block_f32_packing_matches_c(C, kt):
    """ou_block's f32-operand layout (prec 0): the numpy restatement the
    engine uses is byte-identical to ou_block_pack_f32 (48 channels: rows
    padded to 64 with zeros)."""
    from open_universe_amd import _lib as L

    w = np.random.default_rng(C * 10 + kt).standard_normal((C, C, kt)).astype(np.float32)
    c, uc = L.block_pack_f32(w)
    wp = np.concatenate([w, np.zeros((-C % 32, C, kt), np.float32)]) if C % 32 else w
    n, un = L.block_pack_f32_np(wp)
    assert uc == un == 64.0
    assert c.shape == n.shape and np.array_equal(c, n)


@pytest.mark.parametrize("m,cin,kt", [(32, 32, 5), (64, 160, 3), (1536, 512, 1), (50, 96, 3)])
def test_numpy_natural_split_packing_matches_c(m, cin, kt):
    """conv_pack_split_nat_np (what the engine packs for the split-image
    kernel) is byte-identical to ou_conv_pack_split_nat, and holds the same
    hi / lo halves as the pair-ordered packing, only permuted."""
    import numpy as np

    from open_universe_amd import _lib as L

    g = np.random.default_rng(m * cin + kt)
    w = (g.standard_normal((m, cin, kt)) * 0.05).astype(np.float32)
    a, ua = L.conv_pack_split(w, natural=True)
    b, ub = L.conv_pack_split_nat_np(w)
    assert ua == ub and a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    c, uc = L.conv_pack_split_np(w)
    assert uc == ua and np.array_equal(np.sort(a.view(np.uint16)), np.sort(c.view(np.uint16)))


def emulate_fir(spec, x, n_frames, out_len, valid_len=None):
    """The FIR-applied form (ou_conv_desc.fir, include/ouhip.h) from its
    unfolded weights in the kernels' K / row order, float64."""
    mode, r, wu, taps = spec.fir
    x = torch.where(x.double() >= 0, x.double(), x.double() * spec.slope)
    B, Cin, T = x.shape
    t = torch.from_numpy(np.asarray(taps, np.float64))
    fir = lambda v: F.conv1d(v, t[None, None].expand(v.shape[1], 1, -1), padding="same", groups=v.shape[1])
    wu = torch.from_numpy(np.asarray(wu, np.float64))
    if mode in (1, 3):   # k = ((cb r / R + sub) 16 + c) R + p, phase sub R + p (mode 3: no FIR)
        R = 8 if mode == 3 and r % 8 == 0 else 4 if mode == 3 else r
        f = F.pad(x, (0, n_frames * r - T))
        f = fir(f) if mode == 1 else f
        bv = f.reshape(B, Cin // 16, 16, n_frames, r // R, R).permute(0, 1, 4, 2, 5, 3).reshape(B, Cin * r, n_frames)
        y = torch.einsum("mk,bku->bmu", wu, bv)
    else:           # row 32 (co // P) + (co % P) r + ph
        P = 32 // r
        z = torch.einsum("mk,bku->bmu", wu, x)
        cout = spec.w.shape[0] // r
        co = torch.arange(cout)
        rows = 32 * (co // P) + (co % P) * r
        pre = torch.stack([z[:, rows + ph] for ph in range(r)], -1)   # (B, cout, U, r)
        y = fir(pre.reshape(B, cout, n_frames * r))
    if spec.bias is not None:
        y = y + torch.from_numpy(np.asarray(spec.bias, np.float64))[None, :, None]
    if valid_len is not None and valid_len < y.shape[-1]:
        y[..., valid_len:] = 0
    if y.shape[-1] < out_len:
        y = F.pad(y, (0, out_len - y.shape[-1]))
    return y[..., :out_len]


def _sd_rc(direction, cin, cout, r, seed=0):
    g = torch.Generator().manual_seed(seed)
    shape = (cout, cin, r) if direction == "down" else (cin, cout, r)
    return {"p.conv.weight": torch.randn(shape, generator=g, dtype=torch.float64),
            "p.prelu.weight": torch.tensor([0.25], dtype=torch.float64),
            "p.bias": torch.randn(cout, generator=g, dtype=torch.float64)}


@pytest.mark.parametrize("r", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("T", [40, 43])
def test_fir_form_down_matches_folded(r, T):
    """The unfolded K order of the FIR-applied down conv computes what the
    folded 3-frame weights do (both = PReLU -> FIR -> strided conv)."""
    sd = _sd_rc("down", 32, 48, r, seed=r)
    spec = E.spec_down(sd, "p", r, True)
    assert spec.fir is not None and spec.fir[0] == 1
    x = _x(2, 32, T, seed=r)
    U = -(-T // r)
    torch.testing.assert_close(emulate_fir(spec, x, U, U), emulate(spec, x, U, U), rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("r", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("extra_len", [0, -3])
def test_fir_form_up_matches_folded(r, extra_len):
    """The padded whole-channel row order of the FIR-applied up conv
    (32 // r channels per 32-row m-tile) computes what the folded weights do."""
    sd = _sd_rc("up", 64, 40, r, seed=r)
    spec = E.spec_up(sd, "p", r, True)
    assert spec.fir is not None and spec.fir[0] == 2
    x = _x(2, 64, 13, seed=r)
    length = r * 13 + extra_len
    torch.testing.assert_close(emulate_fir(spec, x, 13, length, valid_len=r * 13),
                               emulate(spec, x, 13, length, valid_len=r * 13), rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("r", [4, 20, 40, 120])
def test_st_conv_form_matches_plain(r):
    """The st_convs' blocked K order (ou_conv_desc.fir 3, no FIR) computes
    what the plain frame-view weights do."""
    sd = _sd_rc("down", 32, 48, r, seed=r)
    spec = E.spec_down(sd, "p", r, False)
    assert spec.fir is not None and spec.fir[0] == 3
    T = 5 * r + 3
    x = _x(2, 32, T, seed=r)
    U = -(-T // r)
    torch.testing.assert_close(emulate_fir(spec, x, U, U), emulate(spec, x, U, U), rtol=1e-9, atol=1e-9)


def test_fir_form_only_where_the_kernels_apply():
    """No FIR form where the FIR kernels do not run: channel counts off the
    16 / 32 grid, rates outside 2 / 3 / 4 / 5 / 8, no anti-aliasing."""
    assert E.spec_down(_sd_rc("down", 24, 48, 2), "p", 2, True).fir is None
    assert E.spec_down(_sd_rc("down", 32, 64, 6), "p", 6, True).fir is None
    assert E.spec_down(_sd_rc("down", 32, 64, 2), "p", 2, False).fir is None
    assert E.spec_up(_sd_rc("up", 48, 24, 2), "p", 2, True).fir is None
    assert E.spec_up(_sd_rc("up", 64, 32, 2), "p", 2, False).fir is None
