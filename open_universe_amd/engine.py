"""MI355X execution engine for the UNIVERSE / UNIVERSE++ enhancement path.

The engine turns a reference-named state dict into device-resident, pre-packed
weights (weight norm folded, anti-alias FIRs folded into the rate-change
convolutions, GEMM operands packed in MFMA fragment order) and records the
whole ``enhance()`` launch sequence for one (batch, length, options) shape as
an ``ou_program`` that is replayed natively or as one hipGraph.

The layer walk mirrors the reference modules it replaces:
  ConvBlock                networks/universe/blocks.py:234-416
  ScoreNetwork / enc / dec networks/universe/score.py:27-298
  ConditionerNetwork       networks/universe/condition.py:68-377
  Universe.enhance         networks/universe/universe.py:231-375
"""
import ctypes
import os
import math
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from . import _lib as L
from . import dsp

NF2 = np.float32(1.0 / math.sqrt(2.0))

# Operand precision of ou_conv (ConvDesc.prec): 1 = split-f16 (three f16 MFMA
# passes on hi/lo operand halves, f32 accumulation, f32-class accuracy: see
# csrc/ou_conv.hip), 0 = f32 MFMA, 2 = plain f16 operands (f32 accumulation;
# BASELINE configs[4] "fp16").  OUHIP_CONV_PREC=f32|split|f16 picks the default
# of every Engine; Engine(conv_prec=...) overrides it per model.
_PREC_NAMES = {"f32": 0, "fp32": 0, "0": 0, "split": 1, "split16": 1, "1": 1, "f16": 2, "fp16": 2, "2": 2}


def default_conv_prec():
    import os

    v = os.environ.get("OUHIP_CONV_PREC", "split").strip().lower()
    if v not in _PREC_NAMES:
        raise ValueError(f"OUHIP_CONV_PREC={v!r}: expected f32, split or f16")
    return _PREC_NAMES[v]


_PREP_PREC = None     # set by Engine while it packs its weights
_PREP_STATUS = 0      # device int32* the split-f16 convs flag range errors into (outside an Engine)
_PREP_ENGINE = None   # the Engine packing its weights: hands out per-layer range slots
RANGE_SLOTS = 1024    # per-layer range-flag words after the engine's 4 status words
MAX_SHIFT = 40        # staging exponents past this fall back to f32 operands
_PREP_KSWS = (0, 0)   # (device float*, bytes): the engine's K-slice workspace
KSWS_BYTES = 64 << 20
RS_BIT = 1 << 14      # ConvDesc.tile bit: the register-streamed conv kernel (conv_rkernel)

_REC = None   # set while a plan records (begin_record)
# lane the recorder is on (plan lanes run concurrently) and the plan slot
# (plans of one model that may run at the same time on different streams,
# Universe.enhance_many): convs recorded on (slot, lane) use K-slice workspace
# slot * MAX_LANES + lane of their engine
_LANE = 0
_SLOT = 0
MAX_LANES = 4   # 0 main (score network), 1 conditioner, 2 mel front end + signal_cond_proj convs, 3 spare
MAX_SLOTS = 2   # a third stream measured slower: the box gives a process 4 hardware queues


def set_lane(prog, i):
    """Switch the recording program (and conv_desc's K-slice workspace) to lane i."""
    global _LANE
    assert 0 <= i < MAX_LANES
    prog.lane(i)
    _LANE = i


SC_LANE = 2    # the conditions' signal_cond_proj convs (after the mel front end on the same lane)


def overlap_enabled():
    import os

    return os.environ.get("OUHIP_OVERLAP", "1") != "0"


def split_images_enabled():
    """OUHIP_SPLIT_IMAGES=0 keeps every conv and block on its own f32 staging.
    (Fused blocks as consumers measured neutral at C2 against conv consumers
    only, 731-740 vs 735-737x on one box, `ab_r05m`; they stay linked.)"""
    import os

    return os.environ.get("OUHIP_SPLIT_IMAGES", "1") != "0"


_REC_DEVICE = None   # the recording engine's device (split-image buffers outside an arena)

# Anti-aliased rate-change convs (PReLU_Conv with use_antialiasing,
# blocks.py:214-226) have two forms: the (2r+1)-tap binomial FIR folded into
# 3-frame weights (any kernel; three times the reference's dense MACs) and the
# FIR applied by conv_fdkernel / conv_fukernel (tile bit 17, ou_conv_desc.fir;
# the reference's MACs).  OUHIP_FIR=auto (default) times both per layer and
# records the faster, 1 always the FIR-applied form, 0 always the folded one.
FIR_RATES = (2, 3, 4, 5, 8)
FIR_BIT = 1 << 17
FIR_EARLY = 1 << 8   # with FIR_BIT: the up kernel's residual / bias loads issued before its main loop
FIR_DEEP = 1 << 9    # with FIR_BIT: two input chunks in flight per thread (lean down, up)


def fir_mode():
    v = os.environ.get("OUHIP_FIR", "auto").strip().lower()
    if v not in ("auto", "0", "1"):
        raise ValueError(f"OUHIP_FIR={v!r}: expected auto, 0 or 1")
    return v


def fir_enabled():
    return fir_mode() != "0"


def begin_record(prec, device=None):
    global _REC, _REC_DEVICE
    _REC = {"prec": prec}
    _REC_DEVICE = device
    L.ADD_HOOK = split_hook if prec == 1 and split_images_enabled() else None



def end_record():
    global _REC
    _REC = None
    L.ADD_HOOK = None


# Split images (include/ouhip.h, ou_conv_desc.sy / xs).  A conv whose input
# is the output of the conv recorded just before it on the same lane reads
# that producer's split image -- the PReLU'd, scaled, f16 hi / lo operand the
# producer's epilogue stores beside y -- through the split-image kernel (tile
# bit 15), whose staging is then a plain copy.  The staging exponent of that
# consumer (ou_conv_desc.xs_shift) defaults to the fixed 2^-6 of the f32
# staging path.
SPLIT_SHIFT = 6


def _split_consumer(op, d):
    """(x ptr, bstride, cstride, in_len, channels, slope, shift, owner) of an
    op that can read its operand from a split image, or None."""
    if op == L.OP_CONV:
        wn = getattr(d, "_w_nat", None)
        if wn is None or getattr(d, "_no_split", False) or d.prec != 1 or d.xs or d.in_scale or d.f0 or d.cin % 32:
            return None
        return (d.x, d.x_bstride, d.x_cstride, d.in_len, d.cin, d.slope, d.xs_shift, ("c", getattr(d, "_cw", None), 0))
    fw = getattr(d, "_fw", None)
    if (fw is None or d.prec != 1 or d.xs or d.x or d.f0 or d.f1 or d.h0 or d.h1 or d.channels % 32):
        return None
    return (d.h, d.h_bstride, d.h_cstride, d.length, d.channels, d.slope[0], d.shift[0], ("f", fw, 0))


def _split_producer(op, p):
    """(y ptr, bstride, cstride, out_len, channels, batch) of an op whose
    epilogue can store a split image, or None."""
    if op == L.OP_CONV:
        if p.prec != 1 or p.rout != 1 or p.m % 32 or p.sy or p.f0:
            return None
        return (p.y, p.y_bstride, p.y_cstride, p.out_len, p.m, p.batch)
    if (p.prec != 1 or p.head.w or p.sy or p.channels % 32 or p.f0 or p.f1):
        return None
    return (p.y, p.y_bstride, p.y_cstride, p.length, p.channels, p.batch)


SPLIT_STORE_BPMS = 4e9   # bytes per ms a producer's epilogue adds for its image (~4 TB/s)


def _split_ms(d, per_item, rows, shift, batch):
    """Tuned ms per launch of conv ``d`` reading a split image, plus the
    producer's extra image store (~ bytes / 4 TB/s), or None without a tuner.
    The trial reads the image from d's own input (the same or more bytes:
    timing only reads it), so no image memory is taken to decide."""
    tuner = L.TUNER
    if not hasattr(tuner, "pick"):
        return None
    trial = L.ConvDesc.from_buffer_copy(d)
    trial.xs, trial.xs_bstride, trial.xs_rows, trial.xs_shift = d.x, per_item, rows, shift
    trial.w, trial.w_unscale = d._w_nat
    trial.tile = -1
    _, ms_s = tuner.pick(trial)
    return None if ms_s is None else ms_s + batch * per_item / SPLIT_STORE_BPMS


def _split_pays(d, per_item, rows, shift, batch):
    """A conv consumer takes the split image only where the split-image
    kernel's best tile, plus the producer's extra image store, beats its best
    plain tile (both timed by the tuner; without one, always)."""
    tuner = L.TUNER
    if not hasattr(tuner, "pick"):
        return True
    plain = L.ConvDesc.from_buffer_copy(d)
    plain.tile = -1
    _, ms_p = tuner.pick(plain)
    ms_s = _split_ms(d, per_item, rows, shift, batch)
    if ms_p is None or ms_s is None:
        return True
    return ms_s < ms_p


def _split_note(prog, idx, op, d):
    """Every op added while a split-f16 plan records: forget the producers
    whose output it overwrites, then record it if it is a producer (a conv or
    fused block whose epilogue can store a split image)."""
    from .hazards import footprint, overlap

    writers = prog.__dict__.setdefault("split_writers", {})
    if op in (L.OP_LANE, L.OP_SIGNAL, L.OP_WAIT):
        return
    W = footprint(op, d)[1]
    for k in [k for k, (_, _, _, box) in writers.items() if any(overlap(w, box) for w in W)]:
        del writers[k]
    if op in (L.OP_CONV, L.OP_BLOCK) and _split_producer(op, d) is not None:
        y = [w for w in W if w.base == d.y]
        if y:
            writers[d.y] = (idx, op, d, y[0])


def _split_link(prog, op, d):
    """The split-image link op ``d`` would take (see split_hook), or None:
    (producer index, producer op, producer desc, rows, batch, per-item
    bytes, consumer tuple)."""
    cons = _split_consumer(op, d)
    pv = prog.__dict__.get("split_writers", {}).get(d.x if op == L.OP_CONV else d.h)
    if cons is None or pv is None:
        return None
    idx, pop, p, _ = pv
    prod = _split_producer(pop, p)
    x, xb, xc, in_len, C, slope, shift, owner = cons
    if (p is d or prod is None or prod[0] != x or prod[1] != xb or prod[2] != xc or prod[3] < in_len
            or prod[4] != C or prod[5] < d.batch):
        return None
    rows, batch = prod[3], prod[5]
    return idx, pop, p, rows, batch, (C // 32) * rows * 128, cons


def split_hook(prog, op, d):
    """Program.add hook (split-f16 plans): link op ``d`` (a conv, or a fused
    block's conv1) to the split image of the op that last wrote d's input,
    when that op is a conv or a fused block (any lane: d reads that output,
    so the program already orders d after it).  The pairing follows the data,
    not the lanes, so plans that place unrelated ops differently (enhance and
    enhance_many's) link the same pairs and compute the same bits.  A conv
    consumer is linked only where that pays (_split_pays, decided before any
    image memory is taken)."""
    link = _split_link(prog, op, d)
    if link is None:
        return
    idx, pop, p, rows, batch, per_item, cons = link
    x, xb, xc, in_len, C, slope, shift, owner = cons
    if op == L.OP_CONV and not _split_pays(d, per_item, rows, shift, batch):
        return
    # one image per activation buffer: every step of the score loop rewrites
    # the same activations in the same order, so their images too
    key = (x, xb, xc, rows, C, batch)
    cache = prog.__dict__.setdefault("split_bufs", {})
    buf = cache.get(key)
    if buf is None:
        buf = cache[key] = empty((batch * per_item // 2,), dtype=torch.int16, device=_REC_DEVICE)
        prog.keep.append(buf)
    prog.__dict__.setdefault("split_links", []).append((idx, len(prog.flops)))
    if p.status and owner[1] is not None:
        # a split-image range code (2 / 32) of p widens d's operand: kept per
        # program, so a plan's error resolves against the pairs it recorded
        prog.__dict__.setdefault("split_consumers", {})[p.status] = owner
    p.sy, p.sy_bstride, p.sy_rows, p.sy_shift, p.sy_slope = buf.data_ptr(), per_item, rows, shift, slope
    prog.patch(idx, pop, p)
    d.xs, d.xs_bstride, d.xs_rows = p.sy, per_item, rows
    if op == L.OP_CONV:
        d.xs_shift = shift
        d.w, d.w_unscale = d._w_nat
        if d.tile >= 0 and not d.tile & L.SS_BIT:
            d.tile = -1


split_hook.note = _split_note


# ---------------------------------------------------------------------------
# weights
# ---------------------------------------------------------------------------
def _np(t):
    return t.detach().to("cpu", torch.float32).numpy()


def fold_weight(sd, prefix):
    """weight_norm(dim=0): w = v * (g / ||v||), norm over all dims but 0,
    in float32 as torch._weight_norm does (blocks.py:40-46)."""
    if prefix + ".weight_g" in sd:
        g = sd[prefix + ".weight_g"].detach().to("cpu", torch.float32)
        v = sd[prefix + ".weight_v"].detach().to("cpu", torch.float32)
        n = v.reshape(v.shape[0], -1).norm(dim=1).reshape((-1,) + (1,) * (v.dim() - 1))
        return (v * (g / n)).numpy()
    return _np(sd[prefix + ".weight"])


@dataclass
class ConvW:
    """A prepared convolution: packed weights + geometry (see ou_conv_desc)."""
    m: int
    cin: int
    kt: int
    frame: int
    pad: int
    rout: int
    slope: float
    cc: int
    w: torch.Tensor
    bias: Optional[torch.Tensor]
    shift: int = 0
    ref_macs: float = 0.0
    prec: int = 0            # ConvDesc.prec the weights were packed for
    w_unscale: float = 1.0   # split-f16 weight scale (ou_conv_pack_split)
    status: int = 0          # device int32* for the split-f16 range flag (0 = none)
    ks_ws: tuple = (0, 0)    # K-slice workspace (ptr, bytes) shared by the engine's convs
    cm: bool = False         # rout > 1: channel-major rows (m = co * rout + ph; ConvDesc.rout < 0)
    w_nat: Optional[torch.Tensor] = None   # prec 1, cin % 32 == 0: ou_conv_pack_split_nat (split-image kernel)
    w_unscale_nat: float = 1.0
    xshift: int = 6          # split-f16 staging exponent of this conv's input (ConvDesc.xs_shift)
    fir: Optional["FirW"] = None   # the FIR-applied form of an anti-aliased rate-change conv

    @property
    def cout(self):
        return self.m // self.rout


@dataclass
class FirW:
    """The FIR-applied form of an anti-aliased rate-change conv (ou_conv_desc.fir,
    tile bit 17): unfolded weights (K = cin * rate down, cin up; one tap) in
    the kernels' order (include/ouhip.h), packed by ou_conv_pack_split_nat,
    and the (2 rate + 1)-tap binomial FIR on the device."""
    mode: int                # 1: FIR before a strided conv, 2: after a transposed conv, 3: no FIR (st_convs)
    rate: int
    w: torch.Tensor
    unscale: float
    taps: torch.Tensor


@dataclass
class ConvSpec:
    """Logical (unpacked) convolution in the ou_conv formulation:
    w[m][cin*frame][kt] over the frame view, plus geometry and epilogue bias."""
    w: np.ndarray
    cin: int
    frame: int
    pad: int
    rout: int
    slope: float
    bias: Optional[np.ndarray]
    shift: int = 0
    ref_macs: float = 0.0   # MACs of the replaced reference ops per output frame
    cm: bool = False        # rout > 1: rows ordered m = co * rout + ph (else ph * cout + co)
    fir: Optional[tuple] = None   # (mode 1 down / 2 up / 3 plain strided, rate, unfolded weights, taps): FirW


def make_conv(spec, device, prec=None):
    """prec: 0 f32 operands, 1 split-f16, 2 f16; None = the packing Engine's choice
    (or OUHIP_CONV_PREC outside an Engine)."""
    if prec is None:
        prec = _PREP_PREC if _PREP_PREC is not None else default_conv_prec()
    w_logical = np.ascontiguousarray(spec.w, dtype=np.float32)
    m, cin_eff, kt = w_logical.shape
    assert cin_eff == spec.cin * spec.frame, (cin_eff, spec.cin, spec.frame)
    if spec.frame > 1:
        # logical frame-view channel ci*R + ph -> the kernel's phase-major ph*cin + ci
        w_logical = np.ascontiguousarray(
            w_logical.reshape(m, spec.cin, spec.frame, kt).transpose(0, 2, 1, 3).reshape(m, cin_eff, kt))
    cc = L.conv_chunk(kt, spec.frame)
    if prec in (1, 2):   # f16 uses the hi halves of the split packing
        packed_np, unscale = L.conv_pack_split_np(w_logical)
    else:
        packed_np, unscale = L.conv_pack(w_logical, cc), 1.0
    packed = torch.from_numpy(packed_np).to(device)
    b = None if spec.bias is None else torch.from_numpy(np.ascontiguousarray(spec.bias, np.float32)).to(device)
    w_nat, unscale_nat = None, 1.0
    if prec == 1 and spec.cin % 32 == 0 and kt in (1, 3, 5) and split_images_enabled():
        nat_np, unscale_nat = L.conv_pack_split_nat_np(w_logical)
        w_nat = torch.from_numpy(nat_np).to(device)
    fir = None
    if spec.fir is not None and prec in (1, 2) and fir_enabled():
        mode, rate, wf, taps = spec.fir
        fp_np, fun = L.conv_pack_split_nat_np(np.ascontiguousarray(wf, np.float32)[:, :, None])
        fir = FirW(int(mode), int(rate), torch.from_numpy(fp_np).to(device), float(fun),
                   torch.from_numpy(np.ascontiguousarray(taps, np.float32)).to(device))
    cw = ConvW(m, spec.cin, kt, spec.frame, spec.pad, spec.rout, float(spec.slope), cc, packed, b,
               spec.shift, spec.ref_macs, int(prec), float(unscale), _PREP_STATUS if prec else 0,
               _PREP_KSWS, cm=bool(spec.cm), w_nat=w_nat, w_unscale_nat=float(unscale_nat), fir=fir)
    if prec:
        cw.status = _range_slot(cw) or cw.status
    return cw


def _range_slot(owner):
    """A range-flag word of its own for a split-f16 layer of the packing
    Engine (its device address), so that a range error names the layer."""
    eng = _PREP_ENGINE
    if eng is None or len(eng.range_owners) >= RANGE_SLOTS:
        return 0
    eng.range_owners.append(owner)
    return eng.status.data_ptr() + 4 * (3 + len(eng.range_owners))


def _slope(sd, p):
    return float(sd[p + ".prelu.weight"].reshape(-1)[0])


def _bias(sd, key):
    b = sd.get(key)
    return None if b is None else _np(b)


def spec_same(sd, p, k):
    """PReLU_Conv(C, C, k, padding='same') (blocks.py:293-316)."""
    w = fold_weight(sd, p + ".conv")
    return ConvSpec(w, w.shape[1], 1, (k - 1) // 2, 1, _slope(sd, p), _bias(sd, p + ".conv.bias"),
                    ref_macs=float(w.size))


def spec_plain(sd, p, k, slope=1.0):
    """Plain Conv1d (no activation): input_conv, 1x1 signal_cond_proj, mel conv."""
    w = fold_weight(sd, p)
    return ConvSpec(w, w.shape[1], 1, (k - 1) // 2, 1, slope, _bias(sd, p + ".bias"),
                    ref_macs=float(w.size))


def fir_chunk(mode, r):
    """Phases per K chunk of the down-type FIR kernels (conv_fdkernel): the
    whole frame for mode 1, 8 (or 4) of the st_convs' r phases for mode 3 --
    the device's choice in ou_conv (ou_conv.hip)."""
    return r if mode == 1 else (8 if r % 8 == 0 else 4)


def fir_k_order(w, mode, r):
    """(cout, cin, r) strided-conv weights -> (cout, cin r) in conv_fdkernel's
    K order (include/ouhip.h): chunks of 16 channels x R = fir_chunk(mode, r)
    phases, channel-major inside a chunk, k = ((cb r / R + sub) 16 + c) R + p
    for ci = 16 cb + c, phase sub R + p.  Mode 1 (R = r): k = ci r + ph."""
    cout, cin, _ = w.shape
    R = fir_chunk(mode, r)
    return w.reshape(cout, cin // 16, 16, r // R, R).transpose(0, 1, 3, 2, 4).reshape(cout, cin * r)


def spec_down(sd, p, r, antialias):
    """Strided PReLU_Conv(C, 2C, r, stride=r) (blocks.py:203-231, 268-275).
    Frame view: channel c' = ci*r + p.  With anti-aliasing the 2r+1-tap
    binomial FIR (applied before the conv, blocks.py:217-218) is folded into a
    3r-tap kernel = 3 frames (-1, 0, +1)."""
    w = fold_weight(sd, p + ".conv")  # (Cout, Cin, r)
    cout, cin, _ = w.shape
    if antialias:
        fir = dsp.binomial_taps(2 * r + 1).astype(np.float64)
        wf = np.zeros((cout, cin, 3 * r), dtype=np.float64)
        for kk in range(r):
            wf[:, :, kk:kk + 2 * r + 1] += w[:, :, kk:kk + 1].astype(np.float64) * fir[None, None, :]
        wl = wf.reshape(cout, cin, 3, r).transpose(0, 1, 3, 2).reshape(cout, cin * r, 3)
        fir = None
        if cin % 16 == 0 and r in FIR_RATES:
            # unfolded, in the frame view's K order k = ci r + ph (include/ouhip.h)
            fir = (1, r, fir_k_order(w, 1, r), dsp.binomial_taps(2 * r + 1))
        return ConvSpec(wl, cin, r, 1, 1, _slope(sd, p), _bias(sd, p + ".bias"),
                        ref_macs=float(cout * cin * r + cin * (2 * r + 1) * r), fir=fir)
    fir = None
    if cin % 16 == 0 and r % 4 == 0:
        # the wide strided convs (st_convs, rates 20 .. 240) in the FIR kernels'
        # K order without a FIR (ou_conv_desc.fir 3): each input sample read once
        fir = (3, r, fir_k_order(w, 3, r), np.ones(1, np.float32))
    return ConvSpec(w.reshape(cout, cin * r, 1), cin, r, 0, 1, _slope(sd, p),
                    _bias(sd, p + ".conv.bias"), ref_macs=float(cout * cin * r), fir=fir)


def spec_up(sd, p, r, antialias):
    """Transposed PReLU_Conv(2C, C, r, stride=r) (+ FIR after, blocks.py:221-225)
    as a polyphase convolution over input frames producing r*C rows that the
    kernel's epilogue pixel-shuffles.  weight_norm dim 0 of a ConvTranspose1d
    weight (Cin, Cout, r) is per input channel; fold_weight handles it.  The
    rows are channel-major (m = co * r + ph, ConvDesc.rout = -r): a lane's
    consecutive accumulator rows are consecutive output samples, stored as
    one 16-B access at r = 4 and completing whole output lines within one
    wave at r = 5 (faster at rate 2 too: profiles/bench_ab_upcm_rate_r03p.txt)."""
    w = fold_weight(sd, p + ".conv").astype(np.float64)  # (Cin, Cout, r)
    cin, cout, _ = w.shape
    if antialias:
        fir = dsp.binomial_taps(2 * r + 1).astype(np.float64)
        wl = np.zeros((r, cout, cin, 3), dtype=np.float64)
        for ph in range(r):
            for j in range(2 * r + 1):
                s_ = ph + j - r
                d = s_ // r
                e = s_ - d * r
                wl[ph, :, :, d + 1] += fir[j] * w[:, :, e].T
        cm = r >= 2
        if cm:
            wl = wl.transpose(1, 0, 2, 3)
        fir = None
        if cin % 32 == 0 and r in FIR_RATES and cm:
            # unfolded: every 32-row m-tile holds P = 32 // r whole channels,
            # row 32 (co // P) + (co % P) r + ph (include/ouhip.h)
            P = 32 // r
            wu = np.zeros((-(-cout // P) * 32, cin), dtype=np.float64)
            co = np.arange(cout)
            for ph in range(r):
                wu[32 * (co // P) + (co % P) * r + ph] = w[:, :, ph].T
            fir = (2, r, wu, dsp.binomial_taps(2 * r + 1))
        return ConvSpec(np.ascontiguousarray(wl).reshape(r * cout, cin, 3), cin, 1, 1, r, _slope(sd, p),
                        _bias(sd, p + ".bias"), ref_macs=float(cin * cout * r + cout * (2 * r + 1) * r), cm=cm,
                        fir=fir)
    wl = w.transpose(2, 1, 0)   # (r, cout, cin)
    cm = r >= 2
    if cm:
        wl = wl.transpose(1, 0, 2)
    return ConvSpec(np.ascontiguousarray(wl).reshape(r * cout, cin, 1), cin, 1, 0, r, _slope(sd, p),
                    _bias(sd, p + ".conv.bias"), ref_macs=float(cin * cout * r), cm=cm)


def prep_same(sd, p, k, device):
    return make_conv(spec_same(sd, p, k), device)


def prep_plain(sd, p, k, device, slope=1.0):
    return make_conv(spec_plain(sd, p, k, slope), device)


def prep_down(sd, p, r, antialias, device):
    return make_conv(spec_down(sd, p, r, antialias), device)


def prep_strided(sd, p, r, device):
    """st_convs: PReLU_Conv(Ci, Co, r, stride=r), no FIR (condition.py:53-59)."""
    return make_conv(spec_down(sd, p, r, False), device)


def prep_up(sd, p, r, antialias, device):
    return make_conv(spec_up(sd, p, r, antialias), device)


@dataclass
class FusedW:
    """The three convs of a ConvBlock packed for ou_block (one launch)."""
    w: torch.Tensor          # packed conv1 | conv2 | conv3 (f16 halves as int16, or f32 for prec 0)
    offs: tuple              # byte offsets of the three packed convs in w
    unscale: tuple
    prec: int
    shifts: list = field(default_factory=lambda: [6, 6, 6, 6])   # conv1 / 2 / 3 / down staging exponents
    status: int = 0          # its range-flag word (ou_block codes 1 / 2 / 8 / 16)


@dataclass
class DownW:
    """An encoder block's strided rate-change conv packed for ou_block's fused
    fourth stage (ou_block_desc.w_down): [2C][C][kt * rate] tap-major."""
    w: torch.Tensor
    unscale: float
    bias: Optional[torch.Tensor]
    slope: float
    rate: int
    kt: int


@dataclass
class BlockW:
    """ConvBlock weights (blocks.py:234-351)."""
    C: int
    kind: str
    rate: Optional[int]
    conv1: ConvW
    conv2: ConvW
    conv3: ConvW
    rate_conv: Optional[ConvW] = None
    fused: Optional[FusedW] = None
    down: Optional[DownW] = None


def fuse_blocks_enabled():
    import os

    return os.environ.get("OUHIP_FUSE_BLOCKS", "1") != "0"


# channel counts of the score network's level-0 blocks whose ou_block
# instantiations take the input conv (kEpiIn) and the head (kEpiHead)
ENDS_C = (32, 48)


def fuse_ends_enabled():
    """OUHIP_FUSE_ENDS=0 keeps the score input conv and head as their own launches."""
    import os

    return os.environ.get("OUHIP_FUSE_ENDS", "1") != "0"


def prep_fused(specs, C, prec, device):
    """ou_block weights for a ConvBlock whose channel count one workgroup
    covers (ou_block_supported), else None."""
    if not (fuse_blocks_enabled() and L.load().ou_block_supported(C, prec)):
        return None
    parts, offs, uns, off = [], [], [], 0
    for sp in specs:
        w = sp.w
        if w.shape[0] % 32:   # 48 channels: zero rows up to the next 32 (computed, never stored)
            w = np.concatenate([w, np.zeros((-w.shape[0] % 32,) + w.shape[1:], w.dtype)])
        # f32 operands (prec 0): ou_block_pack_f32's layout; else split / f16 halves
        packed, un = L.block_pack_f32_np(w) if prec == 0 else L.block_pack_np(w)
        parts.append(packed)
        offs.append(off)
        uns.append(un)
        off += packed.nbytes
    w = torch.from_numpy(np.concatenate(parts)).to(device)
    fw = FusedW(w, tuple(offs), tuple(uns), prec)
    if prec:
        fw.status = _range_slot(fw) or _PREP_STATUS
    return fw


def fuse_down_enabled():
    """OUHIP_FUSE_DOWN=0 keeps the encoder's rate-change convs as their own launches."""
    import os

    return os.environ.get("OUHIP_FUSE_DOWN", "1") != "0"


def prep_down_fused(spec, C, prec, bias, device):
    """The rate-change conv in ou_block's layout (DownW), or None where the
    fused block has no such stage."""
    m, cr, kt = spec.w.shape
    r = spec.frame
    if not (fuse_down_enabled() and m == 2 * C and cr == C * r
            and L.load().ou_block_down_supported(C, r, kt, prec)):
        return None
    # frame-view channel ci*r + ph at frame k -> tap k*r + ph of channel ci
    w4 = np.ascontiguousarray(spec.w.reshape(m, C, r, kt).transpose(0, 1, 3, 2).reshape(m, C, kt * r))
    packed, un = L.block_pack_np(w4)
    return DownW(torch.from_numpy(packed).to(device), un, bias, float(spec.slope), r, kt)


def prep_block(sd, p, kind, rate, antialias, device):
    specs = [spec_same(sd, p + ".conv1", 5), spec_same(sd, p + ".conv2", 3), spec_same(sd, p + ".conv3", 3)]
    c1, c2, c3 = (make_conv(sp, device) for sp in specs)
    rc, rc_spec = None, None
    if kind == "down":
        rc_spec = spec_down(sd, p + ".rate_change_conv", rate, antialias)
        rc = make_conv(rc_spec, device)
    elif kind == "up":
        rc = prep_up(sd, p + ".rate_change_conv", rate, antialias, device)
    fused = prep_fused(specs, c1.m, c1.prec, device) if c1.prec in (1, 2) else None
    down = prep_down_fused(rc_spec, c1.m, c1.prec, rc.bias, device) if (fused and rc_spec) else None
    return BlockW(c1.m, kind, rate, c1, c2, c3, rc, fused, down)


@dataclass
class GruW:
    hidden: int
    layers: List  # per layer: (ConvW input projection, w_hh dev [2][3H][H], b_hh dev [2][3H])


def prep_gru(sd, p, num_layers, device):
    layers = []
    for l in range(num_layers):
        s, sr = f"_l{l}", f"_l{l}_reverse"
        w_ih = np.concatenate([_np(sd[p + ".weight_ih" + s]), _np(sd[p + ".weight_ih" + sr])], 0)
        b_ih = np.concatenate([_np(sd[p + ".bias_ih" + s]), _np(sd[p + ".bias_ih" + sr])], 0)
        proj = make_conv(ConvSpec(w_ih[:, :, None], w_ih.shape[1], 1, 0, 1, 1.0, b_ih,
                                  ref_macs=float(w_ih.size)), device)
        w_hh = torch.stack([sd[p + ".weight_hh" + s], sd[p + ".weight_hh" + sr]]).detach().to(
            "cpu", torch.float32).contiguous()
        b_hh = torch.stack([sd[p + ".bias_hh" + s], sd[p + ".bias_hh" + sr]]).float().contiguous().to(device)
        layers.append((proj, w_hh.to(device), b_hh))
    H = int(sd[p + ".weight_hh_l0"].shape[1])
    return GruW(H, layers)


# ---------------------------------------------------------------------------
# activations
# ---------------------------------------------------------------------------
class Act:
    """A (B, C, T) fp32 device tensor viewed as pointer + strides."""

    def __init__(self, t):
        assert t.dtype == torch.float32 and t.dim() == 3
        self.t = t
        self.ptr = t.data_ptr()
        self.bs, self.cs = t.stride(0), t.stride(1)
        self.B, self.C, self.T = t.shape


class ArenaFull(Exception):
    pass


class Arena:
    """One device buffer the plans of one slot carve their buffers from.

    Every buffer of an EnhancePlan is scratch for one replay (outputs are
    copied out right after it; constants live outside), and the plans of one
    slot replay one after another on one stream, so all of them can start at
    offset 0 of the same memory: a stream of clips of many lengths keeps one
    arena sized for the largest recorded length instead of one allocation set
    per length."""

    def __init__(self, device, nbytes):
        self.buf = torch.empty(int(nbytes), dtype=torch.uint8, device=device)
        self.off = 0

    @property
    def nbytes(self):
        return self.buf.numel()

    def take(self, shape, dtype):
        n = math.prod(shape) * torch.empty((), dtype=dtype).element_size()
        off = (self.off + 255) // 256 * 256
        if off + n > self.buf.numel():
            raise ArenaFull(off + n)
        self.off = off + n
        return self.buf[off:off + n].view(dtype).view(shape)


_ARENA = None   # set while an EnhancePlan records onto an arena


def empty(shape, dtype=torch.float32, device=None):
    return _ARENA.take(tuple(shape), dtype) if _ARENA is not None else torch.empty(shape, dtype=dtype, device=device)


def zeros(shape, dtype=torch.float32, device=None):
    return empty(shape, dtype, device).zero_()


def new_act(B, C, T, device):
    return Act(empty((B, C, T), dtype=torch.float32, device=device))


def conv_desc(cw: ConvW, x: Act, y: Act, *, in_len=None, n_frames=None, out_len=None,
              valid_len=None, in_scale=0, res1: Act = None, s1=1.0, film=0, film_bs=0,
              res2: Act = None, s2=1.0, batch=None):
    """ou_conv descriptor of conv ``cw`` from x to y (include/ouhip.h), with
    its shape guards and its algorithmic FLOP / byte counts (d._flops,
    d._bytes: the roofline accounting)."""
    d = L.ConvDesc()
    d.x, d.x_bstride, d.x_cstride = x.ptr, x.bs, x.cs
    d.cin, d.in_len = cw.cin, x.T if in_len is None else in_len
    d.frame, d.shift = cw.frame, cw.shift
    d.in_scale, d.slope = in_scale or 0, cw.slope
    d.w, d.m, d.kt, d.pad, d.cc = cw.w.data_ptr(), cw.m, cw.kt, cw.pad, cw.cc
    d.prec, d.w_unscale, d.status = cw.prec, cw.w_unscale, cw.status
    d.xs_shift = cw.xshift
    d._w_nat = (cw.w_nat.data_ptr(), cw.w_unscale_nat) if cw.w_nat is not None else None
    d._cw = cw
    d._fir = cw.fir
    d.ks_ws, d.ks_ws_bytes = cw.ks_ws
    if (_LANE or _SLOT) and d.ks_ws:   # the engine allocates MAX_SLOTS x MAX_LANES workspaces
        d.ks_ws += (_SLOT * MAX_LANES + _LANE) * d.ks_ws_bytes
    if n_frames is None:
        n_frames = -(-d.in_len // cw.frame) if cw.rout == 1 else x.T
    d.n_frames = n_frames
    d.f0 = 0
    d.batch = x.B if batch is None else batch
    d.y, d.y_bstride, d.y_cstride = y.ptr, y.bs, y.cs
    d.rout = -cw.rout if (cw.cm and cw.rout > 1) else cw.rout
    d.out_len = y.T if out_len is None else out_len
    d.valid_len = (1 << 30) if valid_len is None else valid_len
    d.bias = cw.bias.data_ptr() if cw.bias is not None else 0
    if res1 is not None:
        d.res1, d.r1_bstride, d.r1_cstride, d.s1 = res1.ptr, res1.bs, res1.cs, s1
    d.film, d.film_bstride = film or 0, film_bs
    if res2 is not None:
        d.res2, d.r2_bstride, d.r2_cstride, d.s2 = res2.ptr, res2.bs, res2.cs, s2
    d.tile = -1
    d._flops = 2.0 * cw.ref_macs * n_frames * d.batch
    assert d.n_frames > 0
    # algorithmic HBM bytes: input, output and residuals once each (f32), plus
    # the logical f32 weights -- no halo or tile re-reads
    act = cw.cin * d.in_len + cw.cout * d.out_len * (1 + (res1 is not None) + (res2 is not None))
    d._bytes = 4.0 * (act * d.batch + cw.m * cw.cin * cw.frame * cw.kt)
    # shape guards: the kernel trusts these (an out-of-bounds store faults the GPU)
    assert x.C == cw.cin, ("conv input channels", x.C, cw.cin)
    assert y.C == cw.cout, ("conv output channels", y.C, cw.cout)
    assert 0 < d.in_len <= x.T, ("conv in_len", d.in_len, x.T)
    assert 0 < d.out_len <= y.T, ("conv out_len", d.out_len, y.T)
    assert d.batch <= min(x.B, y.B)
    for r in (res1, res2):
        if r is not None:
            assert r.C == cw.cout and r.T >= d.out_len and r.B >= d.batch, ("residual", r.t.shape)
    return d


def rec_block(prog, bw: BlockW, h: Act, out: Act, tA: Act, tB: Act, film=0, film_bs=0,
              sc: Act = None, res2: Act = None, s2=1.0, cond_out: Act = None, skip_tail=False,
              x_in=None, head=None, e_out: Act = None, after_c1=None):
    """ConvBlock main stage (blocks.py:393-407):
       cond_out = conv1(h); c = (cond_out + sc)/sqrt2; c = film(c); c = conv3(conv2(c));
       out = (h + c)/sqrt2 [; out = (out + res2) * s2]
    and, for a down block given ``e_out``, its rate-change conv e_out =
    rate_conv(out) (blocks.py:268-275): fused into the block where ou_block
    has the stage, else its own launch.  after_c1(): recorded as soon as
    conv1 (cond_out) is done -- right after conv1's launch in the unfused
    form, after the block in the fused one."""
    c1_out = cond_out if cond_out is not None else tA
    d1 = conv_desc(bw.conv1, h, c1_out, res1=sc, s1=NF2, film=film, film_bs=film_bs)
    if skip_tail:
        add_conv(prog, d1)
        if after_c1 is not None:
            after_c1()
        return
    d2 = conv_desc(bw.conv2, c1_out, tB)
    d3 = conv_desc(bw.conv3, tB, out, res1=h, s1=NF2, res2=res2, s2=s2)
    d_rc = conv_desc(bw.rate_conv, out, e_out) if e_out is not None else None
    if bw.fused is not None and out.ptr != h.ptr:
        fuse_rc = d_rc is not None and bw.down is not None
        descs = (d1, d2, d3) + ((x_in[4],) if x_in is not None else ()) + ((d_rc,) if fuse_rc else ())
        bd = block_desc(bw, h, out, descs, sc=sc, film=film, film_bs=film_bs,
                        cond_out=cond_out, res2=res2, s2=s2,
                        x_in=x_in[:4] if x_in is not None else None, head=head,
                        e_out=e_out if fuse_rc else None)
        prog.add(L.OP_BLOCK, bd)
        if after_c1 is not None:
            after_c1()
        if d_rc is not None and not fuse_rc:
            add_conv(prog, d_rc)
        return
    assert x_in is None and head is None, "input / head fusion needs the fused block"
    add_conv(prog, d1)
    if after_c1 is not None:
        after_c1()
    add_conv(prog, d2)
    add_conv(prog, d3)
    if d_rc is not None:
        add_conv(prog, d_rc)


def fir_desc(d):
    """The FIR-applied form (tile bit 17) of an anti-aliased rate-change
    conv's folded descriptor ``d``: one tap, the unfolded weights and taps
    of its FirW, the same buffers, geometry and epilogue."""
    fw = d._fir
    f = L.ConvDesc.from_buffer_copy(d)
    f.kt, f.pad, f.tile = 1, 0, -1
    f.w, f.w_unscale = fw.w.data_ptr(), fw.unscale
    f.fir, f.fir_taps = fw.mode, fw.taps.data_ptr()
    f._flops, f._bytes, f._cw, f._w_nat = d._flops, d._bytes, getattr(d, "_cw", None), None
    return f


def choose_fir(prog, d):
    """The form an anti-aliased rate-change conv is recorded in (OUHIP_FIR):
    with a tuner, the FIR-applied one where its best tile beats the folded
    form's best tile and, where the conv would read a producer's split image,
    that link's time too; without one, the FIR-applied form."""
    mode = fir_mode()
    if getattr(d, "_fir", None) is None or mode == "0" or d.prec not in (1, 2) or d.f0 or d.xs:
        return d
    f = fir_desc(d)
    tuner = L.TUNER
    if mode == "1" or not hasattr(tuner, "pick"):
        return f
    _, ms_f = tuner.pick(f)
    _, ms_p = tuner.pick(d)
    folded = [ms_p]
    if L.ADD_HOOK is split_hook:
        link = _split_link(prog, L.OP_CONV, d)
        if link is not None:
            _, _, _, rows, batch, per_item, cons = link
            folded.append(_split_ms(d, per_item, rows, cons[6], batch))
    folded = [t for t in folded if t is not None]
    return f if ms_f is not None and (not folded or ms_f < min(folded)) else d


def add_conv(prog, d):
    """Record an ou_conv (an anti-aliased rate-change conv in the form
    choose_fir picks)."""
    prog.add(L.OP_CONV, choose_fir(prog, d))


def block_desc(bw: BlockW, h: Act, out: Act, descs, sc: Act = None, film=0, film_bs=0, cond_out: Act = None,
               res2: Act = None, s2=1.0, x_in=None, head=None, e_out: Act = None):
    """ou_block descriptor of a ConvBlock's main path; ``descs`` are the
    equivalent ou_conv descriptors (their shape checks have run; their
    algorithmic FLOPs and bytes -- the unfused reference ops -- are kept).
    x_in = (x Act, in_scale ptr, w_in, b_in): compute h from the score input
    conv instead of reading it; head: an ou_head descriptor run on the block
    output instead of storing it."""
    fw = bw.fused
    d = L.BlockDesc()
    d.h, d.h_bstride, d.h_cstride = h.ptr, h.bs, h.cs
    d.channels, d.length, d.batch, d.prec = bw.C, h.T, h.B, fw.prec
    assert out.C == bw.C and out.T == h.T and out.B >= h.B, ("block output", out.t.shape, h.t.shape)
    for i, cw in enumerate((bw.conv1, bw.conv2, bw.conv3)):
        d.w[i] = fw.w.data_ptr() + fw.offs[i]
        d.bias[i] = cw.bias.data_ptr() if cw.bias is not None else 0
        d.slope[i] = cw.slope
        d.w_unscale[i] = fw.unscale[i]
    if sc is not None:
        assert sc.C == bw.C and sc.T >= h.T and sc.ptr != out.ptr
        d.sc, d.sc_bstride, d.sc_cstride, d.s_sc = sc.ptr, sc.bs, sc.cs, float(NF2)
    d.film, d.film_bstride = film or 0, film_bs
    if cond_out is not None:
        assert cond_out.C == bw.C and cond_out.T >= h.T and cond_out.ptr != out.ptr
        d.cond_out, d.co_bstride, d.co_cstride = cond_out.ptr, cond_out.bs, cond_out.cs
    d.y, d.y_bstride, d.y_cstride = out.ptr, out.bs, out.cs
    d.s_res, d.s2 = float(NF2), float(s2)
    if res2 is not None:
        assert res2.C == bw.C and res2.T >= h.T and res2.ptr != out.ptr
        d.res2, d.r2_bstride, d.r2_cstride = res2.ptr, res2.bs, res2.cs
    d.status = fw.status or bw.conv1.status or 0
    for i in range(4):
        d.shift[i] = fw.shifts[i]
    d._fw = fw   # split-image linking (split_hook)
    if x_in is not None:
        xa, scale, w_in, b_in = x_in
        assert bw.C in ENDS_C and xa.C == 1 and xa.T == h.T and xa.B >= h.B
        d.x, d.x_bstride, d.in_scale = xa.ptr, xa.bs, scale or 0
        d.w_in, d.b_in = w_in.data_ptr(), b_in.data_ptr()
    if head is not None:
        assert bw.C in ENDS_C and head.length == h.T and head.channels == bw.C
        d.head = head
    if e_out is not None:
        dn = bw.down
        assert e_out.C == 2 * bw.C and e_out.T == -(-h.T // dn.rate) and e_out.B >= h.B, ("block e", e_out.t.shape)
        assert e_out.ptr not in (h.ptr, out.ptr)
        d.w_down, d.w_down_unscale = dn.w.data_ptr(), dn.unscale
        d.b_down = dn.bias.data_ptr() if dn.bias is not None else 0
        d.slope_down, d.rate, d.down_kt = dn.slope, dn.rate, dn.kt
        d.e, d.e_bstride, d.e_cstride = e_out.ptr, e_out.bs, e_out.cs
    d._flops = sum(x._flops for x in descs) + (head._flops if head is not None else 0.0)
    d._bytes = sum(x._bytes for x in descs)
    return d


GRU_FLAGS = int(os.environ.get("OUHIP_GRU_FLAGS", "-1"))   # -1: kernel default; see ou_gru_desc.flags
_GRU_WS_ZEROED = False   # set by EnhancePlan: it zeroes the GRU workspaces once per replay


def rec_gru_ws_zero(prog, granules):
    """Zero a GRU hand-off workspace once per replay (OP_MEMSET); the GRU
    launches recorded after it (with _GRU_WS_ZEROED) then skip their own
    memset (ou_gru_desc.ws_zeroed)."""
    prog.add(L.OP_MEMSET, L.MemsetArgs(ptr=granules.data_ptr(), bytes=granules.numel() * granules.element_size()))


def rec_gru(prog, gw: GruW, layer, x: Act, gi: Act, y: Act, granules, status, res: Act = None,
            res_scale=1.0, xcd=0):
    """Bidirectional GRU layer (input projection + recurrence, gru.py via
    score.py:117-125)."""
    proj, w_hh, b_hh = gw.layers[layer]
    H = gw.hidden
    assert gi.C == 6 * H and gi.T == x.T and y.C == 2 * H and y.T == x.T and y.B == x.B
    if res is not None:
        assert res.C == 2 * H and res.T == x.T
    assert granules.numel() * 8 >= L.load().ou_gru_workspace_bytes(H, x.B)
    prog.add(L.OP_CONV, conv_desc(proj, x, gi))
    d = L.GruDesc()
    d.gi, d.gi_bstride = gi.ptr, gi.bs
    d.w_hh, d.b_hh = w_hh.data_ptr(), b_hh.data_ptr()
    d.y, d.y_bstride, d.y_cstride = y.ptr, y.bs, y.cs
    if res is not None:
        d.res, d.res_bstride, d.res_cstride, d.res_scale = res.ptr, res.bs, res.cs, res_scale
    d.hidden, d.steps, d.batch = gw.hidden, x.T, x.B
    d.granules, d.status = granules.data_ptr(), status.data_ptr()
    d.flags = GRU_FLAGS if not xcd else (GRU_FLAGS if GRU_FLAGS >= 0 else 0x8000) | ((xcd & 7) << 12)
    d.ws_zeroed = 1 if _GRU_WS_ZEROED else 0
    d._flops = 2.0 * 2 * 3 * H * H * x.T * x.B
    prog.add(L.OP_GRU, d)


def level_lengths(T, rates):
    Ts = [T]
    for r in rates:
        Ts.append(-(-Ts[-1] // r))
    return Ts


# ---------------------------------------------------------------------------
# per-layer tile autotuning
# ---------------------------------------------------------------------------
class ConvTuner:
    """Times every tile configuration that fits LDS for a conv geometry (on the
    current stream, with HIP events) and keeps the fastest.  Plans are built
    once per input shape, so this runs once per distinct layer geometry.
    With ``path`` (env OUHIP_TUNE_CACHE) the choices persist across processes
    as JSON; a cached geometry launches nothing at plan build."""

    def __init__(self, reps=4, path=None):
        import json
        import os

        self.cache = {}
        self.times = {}   # key -> the chosen tile's ms per launch (split_hook weighs a split-image link by it)
        self.reps = reps
        self.graph = os.environ.get("OUHIP_TUNE_GRAPH", "1") != "0"   # time candidates inside a hipGraph
        if self.graph:
            self.reps = max(reps, 8)
        self.path = path
        self.timed = 0   # geometries tuned by timing (not reused from another length)
        self.by_geom = {}   # geometry -> frame-count buckets cached
        if path and os.path.exists(path):
            with open(path) as fh:
                raw = json.load(fh)
            times = raw.pop("__ms__", {})
            self.cache = {tuple(json.loads(k)): v for k, v in raw.items()}
            self.times = {tuple(json.loads(k)): v for k, v in times.items()}
        # persisted geometries seed the nearest-length reuse too
        for kk in self.cache:
            self.by_geom.setdefault(kk[:-1], set()).add(kk[-1])

    def _save(self):
        import json

        if self.path:
            out = {json.dumps(list(k)): v for k, v in self.cache.items()}
            out["__ms__"] = {json.dumps(list(k)): v for k, v in self.times.items()}
            with open(self.path, "w") as fh:
                json.dump(out, fh)

    @staticmethod
    def bucket(n):
        """Octave bucket of a frame count: plans for clips of other lengths
        reuse the tiles tuned for the same geometry at a similar length."""
        return int(n).bit_length()

    @staticmethod
    def geometry(d):
        # bool(ks_ws): K-slice tiles are only valid with a workspace
        b = d.batch
        return (d.m, d.cin, d.frame, d.kt, d.pad, b, d.rout, bool(d.res1), bool(d.film), bool(d.res2),
                bool(d.in_scale), d.prec, bool(d.ks_ws), bool(d.xs), d.fir)

    @classmethod
    def key(cls, d):
        return cls.geometry(d) + (cls.bucket(d.n_frames),)

    @staticmethod
    def fit_workspace(d, tile):
        """Drop the K-slice bits of a tile whose partial sums might not fit the
        workspace at this frame count (bound with generous tile padding)."""
        S = 1 << ((tile >> 12) & 3)
        if S > 1 and S * (d.n_frames + 256) * (d.m + 256) * d.batch * 4 > d.ks_ws_bytes:
            return tile & ~(3 << 12)
        return tile

    def __call__(self, d):
        import ctypes
        import os

        k = self.key(d)
        if k in self.cache:
            return self.fit_workspace(d, self.cache[k])
        # the same geometry tuned at another length: reuse its tile (nearest
        # bucket) instead of timing every candidate again
        g, b = self.geometry(d), self.bucket(d.n_frames)
        near = self.by_geom.get(g)
        if near and os.environ.get("OUHIP_TUNE_EVERY_LENGTH", "0") != "1":
            bb = min(near, key=lambda x: (abs(x - b), x))
            self.cache[k] = self.cache[g + (bb,)]
            if g + (bb,) in self.times:   # another length's time: a rough figure, scaled by the frames
                self.times[k] = self.times[g + (bb,)] * 2.0 ** (b - bb)
            near.add(b)
            return self.fit_workspace(d, self.cache[k])
        lib = L.load()
        stream = torch.cuda.current_stream().cuda_stream
        best, best_ms = -1, float("inf")
        self.timed += 1
        # tile shape x log2(output tiles per workgroup); > 0 = persistent kernel
        # (bit 10: the warp-specialised persistent kernel)
        # (split-f16, bit 11 in the query only: one-tile workgroups)
        # K slices (bits 12-13) for one-tile shapes when the engine has a
        # workspace; ou_conv refuses slices beyond the chunk count or workspace
        # only where the grid is small (about 64 x 64 output tiles: under ~4
        # workgroups per CU); elsewhere slices only add traffic
        small = -(-d.n_frames // 64) * -(-d.m // 64) * d.batch <= 1024
        ksl = (0, 1 << 12, 2 << 12, 3 << 12) if d.ks_ws and small else (0,)
        if d.fir:   # the FIR-applied rate-change kernels' shapes only
            cands = [t | FIR_BIT for t in range(16) if lib.ou_conv_tile_ok(d.kt, t | FIR_BIT)]
            if d.fir == 2:   # up: early epilogue loads (tile bit 8) or two chunks in flight (bit 9)
                cands += [t | FIR_EARLY for t in cands] + [t | FIR_DEEP for t in cands]
            elif d.fir == 1 and not (d.res1 or d.res2 or d.film):   # lean down: two chunks in flight
                cands += [t | FIR_DEEP for t in cands]
        elif d.xs:   # a split-image input: the split-image kernel's shapes only
            cands = [t | L.SS_BIT for t in range(16) if lib.ou_conv_tile_ok(d.kt, t | L.SS_BIT)]
        elif d.prec in (1, 2):
            cands = [t | k for t in range(lib.ou_conv_num_tiles()) if lib.ou_conv_tile_ok(d.kt, t | (1 << 11))
                     for k in ksl]
            # register-streamed kernel (tile bit 14): whole input windows
            # staged once; ou_conv refuses the shapes whose window exceeds LDS
            if d.cin % 16 == 0:
                cands += [t | RS_BIT | k for t in range(16) if lib.ou_conv_tile_ok(d.kt, t | RS_BIT) for k in ksl]
        else:
            cands = [t | v for t in range(lib.ou_conv_num_tiles()) for v in (0, 1 << 8, 2 << 8, 1 << 10)
                     if lib.ou_conv_tile_ok(d.kt, t | v)]
            cands += [t | k for t in range(lib.ou_conv_num_tiles()) if lib.ou_conv_tile_ok(d.kt, t)
                      for k in ksl[1:]]
        log = os.environ.get("OUHIP_TUNE_LOG")
        # candidates run on whatever the buffers hold at record time: keep
        # their split-f16 range flags out of the engine's status word (and
        # the timing programs out of the recorder's split-image linking)
        status, d.status = d.status, None
        hook, L.ADD_HOOK = L.ADD_HOOK, None
        try:
            best, best_ms = self._time(d, cands, lib, stream, log)
        finally:   # a candidate that raises leaves the recorder as it was
            d.tile = -1
            d.status = status
            L.ADD_HOOK = hook
        self.cache[k] = best
        self.times[k] = best_ms
        self.by_geom.setdefault(k[:-1], set()).add(k[-1])
        if os.environ.get("OUHIP_TUNE_VERBOSE", "1") != "0":   # progress (long plan builds)
            import sys

            print(f"[ou tune] m={d.m} cin={d.cin} frame={d.frame} kt={d.kt} n={d.n_frames} b={d.batch} "
                  f"rout={d.rout} prec={d.prec} fir={d.fir}: tile 0x{best:x} {best_ms * 1e3:.1f} us "
                  f"({len(cands)} candidates)", file=sys.stderr, flush=True)
        self._save()
        return best

    def _time(self, d, cands, lib, stream, log):
        """(best tile, its ms per launch) over the candidate tiles of ``d``."""
        import ctypes
        import os

        best, best_ms = -1, float("inf")
        for t in cands:
            d.tile = t
            if log:   # diagnostics: name every candidate before it runs
                with open(log, "a") as fh:
                    fh.write(f"m={d.m} cin={d.cin} frame={d.frame} kt={d.kt} n={d.n_frames} b={d.batch} "
                             f"rout={d.rout} res1={bool(d.res1)} tile={t & 0xff} tpw={1 << ((t >> 8) & 3)} ws={t >> 10}\n")
                    fh.flush()
                    os.fsync(fh.fileno())
            if lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream)) != 0:
                continue
            lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream))   # second warm-up (code object load)
            if log:
                torch.cuda.synchronize()
            # best of two timed batches: a single short batch is noisy enough
            # to prefer a 35 % slower tile
            ms = float("inf")
            if self.graph:
                # device time as the plans run it: copies of the op in one
                # hipGraph (eager back-to-back launches are host-bound below
                # ~10 us and charge K-slice tiles a second host launch)
                prog = L.Program()
                for _ in range(self.reps):
                    prog.add(L.OP_CONV, d)
                prog.capture()
                prog.launch(stream)
                for _ in range(2):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    prog.launch(stream)
                    e1.record()
                    e1.synchronize()
                    ms = min(ms, e0.elapsed_time(e1) / self.reps)
                del prog
            else:
                for _ in range(2):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(self.reps):
                        lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream))
                    e1.record()
                    e1.synchronize()
                    ms = min(ms, e0.elapsed_time(e1) / self.reps)
            if ms < best_ms:
                best, best_ms = t, ms
        return best, best_ms


    def pick(self, d):
        """(tile, ms per launch or None) for a descriptor, tuning it if new."""
        tile = self(d)
        return tile, self.times.get(self.key(d))


_TUNER = None


def enable_autotune(flag=True):
    global _TUNER
    import os

    if flag and os.environ.get("OUHIP_AUTOTUNE", "1") != "0":
        if _TUNER is None:
            _TUNER = ConvTuner(path=os.environ.get("OUHIP_TUNE_CACHE") or None)
        L.TUNER = _TUNER
    else:
        L.TUNER = None


# ---------------------------------------------------------------------------
# engine
# ---------------------------------------------------------------------------
class Engine:
    def __init__(self, model_cfg, sd, device, parts=("score", "cond", "sdl"), _record_only=False,
                 conv_prec=None):
        global _PREP_PREC, _PREP_STATUS, _PREP_KSWS, _PREP_ENGINE
        self.device = torch.device(device)
        self.conv_prec = default_conv_prec() if conv_prec is None else int(conv_prec)
        if self.device.type != "cuda" and not _record_only:
            raise L.OuHipError("open_universe_amd runs on a HIP device (got %s)" % device)
        L.load()
        self.cfg = model_cfg
        self.scfg = model_cfg.get("score_model")
        self.ccfg = model_cfg.get("condition_model")
        self.edm = model_cfg.get("edm")
        self.level_db = (model_cfg.get("normalization_kwargs") or {}).get("level_db", 0.0)
        base = self.scfg if self.scfg is not None else self.ccfg
        self.rates = list(base["rate_factors"])
        self.nch = base["n_channels"]
        self.extra = base.get("extra_conv_block", False)
        if not self.extra:
            raise NotImplementedError("the HIP engine targets extra_conv_block=True configs")
        self.tot_ds = math.prod(self.rates)
        sp = "_edm_model" if self.edm is not None else "score_model"
        dev = self.device
        self.has_sdl = False
        # [0] GRU hand-off timeout, [1] split-f16 range error of a layer
        # without a slot of its own; [4 + i] the range codes of layer i
        # (range_owners[i]: a ConvW or FusedW), see plan.check / widen_ranges
        self.status = torch.zeros(4 + RANGE_SLOTS, dtype=torch.int32, device=dev)
        self.range_owners = []
        # K-slice partial sums (ou_conv tile bits 12-13): ops of one lane run
        # one after another, so the convs of a lane share one buffer (one per
        # plan lane: conv_desc offsets by the recording lane)
        self.ks_ws = torch.empty(MAX_SLOTS * MAX_LANES * KSWS_BYTES // 4, dtype=torch.float32, device=dev)
        saved = _PREP_PREC, _PREP_STATUS, _PREP_KSWS, _PREP_ENGINE
        _PREP_PREC, _PREP_STATUS, _PREP_ENGINE = self.conv_prec, self.status.data_ptr() + 4, self
        _PREP_KSWS = (self.ks_ws.data_ptr(), KSWS_BYTES)
        try:
            with torch.no_grad():
                if "score" in parts:
                    self._prep_score(sd, sp, dev)
                if "cond" in parts:
                    self._prep_cond(sd, "condition_model", dev)
                if "sdl" in parts:
                    self._prep_sdl(sd, "signal_decoupling_layer", dev)
        finally:
            _PREP_PREC, _PREP_STATUS, _PREP_KSWS, _PREP_ENGINE = saved
        enable_autotune(self.device.type == "cuda")

    def widen_ranges(self, flags, step=8, consumers=None):
        """A range error's per-layer codes [(slot, code)] (plan.check): widen
        the staging exponent of every operand whose finite values left the
        split-f16 range by 2^step -- the conv's own input (code 1), a fused
        block's conv1 / conv2 / conv3 / down input (1 / 2 / 8 / 16), the
        operand of the op a conv (2) or block (32) stores a split image for.  Codes 4 alone (an
        infinite value: an overflow upstream) widen nothing.  Bits 8-10 (a
        thermometer of how far the values went: 2^23 / 2^31 / 2^39) widen by
        2 / 3 / 4 steps at once, so one rerun fixes what one replay saw.  Returns the
        number of exponents widened; 0 (nothing to widen, or an exponent past
        MAX_SHIFT) means the caller falls back to f32 operands.  Plans must
        be recorded again: the exponents are read at record time.
        ``consumers``: the failing plan's split-image pairs (producer range
        word -> consumer operand; Program.split_consumers)."""
        n = 0
        for slot, code in flags:
            if slot < 0 or slot >= len(self.range_owners):
                return 0
            own = self.range_owners[slot]
            w = step * (1 + bin((code >> 8) & 7).count("1"))
            targets = []
            if isinstance(own, FusedW):
                targets = [("f", own, i) for i, bit in enumerate((1, 2, 8, 16)) if code & bit]
            elif code & 1:
                targets.append(("c", own, 0))
            if code & (32 if isinstance(own, FusedW) else 2):   # its split image: the consumer's operand
                cons = (consumers or {}).get(own.status)
                if cons is None:
                    return 0
                targets.append(cons)
            for kind, o, i in targets:
                if kind == "f":
                    o.shifts[i] += w
                    if o.shifts[i] > MAX_SHIFT:
                        return 0
                else:
                    o.xshift += w
                    if o.xshift > MAX_SHIFT:
                        return 0
                n += 1
        return n

    # -------------------------------------------------------------- weights
    def _prep_score(self, sd, p, dev):
        cfg = self.scfg
        aa = cfg.get("use_antialiasing", False)
        rates = self.rates
        n_lvl = len(rates) + (1 if self.extra else 0)
        self.s_input = prep_plain(sd, p + ".input_conv", cfg.get("fb_kernel_size", 3), dev)
        # raw input-conv weights for the fused first block (ou_block kEpiIn)
        w_in = fold_weight(sd, p + ".input_conv")
        b_in = _bias(sd, p + ".input_conv.bias")
        self.s_in_w = torch.from_numpy(np.ascontiguousarray(w_in.reshape(w_in.shape[0], -1), np.float32)).to(dev)
        self.s_in_b = torch.from_numpy(np.ascontiguousarray(
            b_in if b_in is not None else np.zeros(w_in.shape[0]), np.float32)).to(dev)
        self.s_in_fusable = w_in.shape[1] == 1 and w_in.shape[2] == 3
        self.s_enc = []
        for i in range(n_lvl):
            q = f"{p}.encoder.ds_modules.{i}"
            if i < len(rates):
                self.s_enc.append(prep_block(sd, q, "down", rates[i], aa, dev))
            else:
                self.s_enc.append(prep_block(sd, q, "none", None, aa, dev))
        self.s_gru = prep_gru(sd, p + ".encoder.gru", 1, dev)
        ups = rates[::-1]
        self.s_dec, self.s_sc = [], []
        for l in range(n_lvl):
            q = f"{p}.decoder.up_modules.{l}"
            if self.extra and l == 0:
                self.s_dec.append(prep_block(sd, q, "none", None, aa, dev))
            else:
                self.s_dec.append(prep_block(sd, q, "up", ups[l - (1 if self.extra else 0)], aa, dev))
            self.s_sc.append(prep_plain(sd, f"{p}.decoder.signal_cond_proj.{l}", 1, dev))
        # FiLM projections, concatenated: encoder levels then decoder levels
        ws, bs, self.film_off = [], [], []
        off = 0
        for name in [f"{p}.encoder.cond_proj.{i}" for i in range(n_lvl)] + \
                    [f"{p}.decoder.noise_cond_proj.{l}" for l in range(n_lvl)]:
            w = fold_weight(sd, name)
            ws.append(w)
            bs.append(_np(sd[name + ".bias"]))
            self.film_off.append(off)
            off += w.shape[0]
        self.film_rows = off
        self.emb_w = torch.from_numpy(np.concatenate(ws, 0)).to(dev).contiguous()
        self.emb_b = torch.from_numpy(np.concatenate(bs, 0)).to(dev).contiguous()
        self.emb_dim = self.emb_w.shape[1]
        te = cfg.get("time_embedding")
        self.emb_kind = 0 if te == "simple" else 1
        if self.emb_kind == 0:
            self.te_w = float(sd[p + ".sigma_block.weight"].reshape(-1)[0])
            self.te_b = float(sd[p + ".sigma_block.bias"].reshape(-1)[0])
        else:
            q = p + ".sigma_block"
            self.rff = sd[q + ".freq"].float().contiguous().to(dev)
            self.mlp = [(sd[f"{q}.layer{i}.lin.weight"].float().contiguous().to(dev),
                         sd[f"{q}.layer{i}.lin.bias"].float().contiguous().to(dev),
                         _slope(sd, f"{q}.layer{i}")) for i in (1, 2, 3)]
        # head: score.prelu -> output_conv (PReLU_Conv C -> 1, k3)
        self.head_s1 = float(sd[p + ".prelu.weight"].reshape(-1)[0])
        self.head_s2 = _slope(sd, p + ".output_conv")
        self.head_w = torch.from_numpy(fold_weight(sd, p + ".output_conv.conv").reshape(-1).copy()).to(dev)
        hb = sd.get(p + ".output_conv.conv.bias")
        self.head_b = 0.0 if hb is None else float(hb.reshape(-1)[0])
        assert fold_weight(sd, p + ".output_conv.conv").shape[0] == 1

    def _prep_cond(self, sd, p, dev):
        cfg = self.ccfg
        rates = list(cfg["rate_factors"])
        aa_dec = cfg.get("use_antialiasing", False)
        n_lvl = len(rates) + (1 if cfg.get("extra_conv_block", False) else 0)
        self.c_extra = cfg.get("extra_conv_block", False)
        self.c_gru_res = cfg.get("encoder_gru_residual", False)
        # mel front end (condition.py:68-114)
        ds = math.prod(rates)
        n_fft = cfg.get("n_mel_oversample", 4) * ds
        self.mel_hop, self.mel_nfft = ds, n_fft
        self.mel_nmels = cfg.get("n_mels", 80)
        nfreq = n_fft // 2 + 1
        self.mel_nfreq = nfreq
        self.mel_pl = (n_fft - ds) // 2
        win = dsp.hann_periodic(n_fft).astype(np.float64)
        n = np.arange(n_fft)
        f = np.arange(nfreq)
        ang = 2.0 * math.pi * np.outer(f, n) / n_fft
        dft = np.concatenate([win * np.cos(ang), win * np.sin(ang)], 0)  # (2F, n_fft)
        kt = n_fft // ds
        # w_logical[m][p][kk] = dft[m][kk*hop + p]
        wl = dft.reshape(2 * nfreq, kt, ds).transpose(0, 2, 1)
        # the STFT and the filterbank keep f32 operands: |STFT|^2 is unbounded
        # (split-f16 staging needs |x| < 2^15)
        self.c_stft = make_conv(ConvSpec(wl, 1, ds, 0, 1, 1.0, None, shift=-self.mel_pl), dev, prec=0)
        fb = dsp.melscale_fbanks(nfreq, 0.0, float(24000 // 2), self.mel_nmels, 24000)
        self.c_fb = make_conv(ConvSpec(fb.T[:, :, None], nfreq, 1, 0, 1, 1.0, None), dev, prec=0)
        self.c_melconv = prep_plain(sd, p + ".input_mel.conv", 3, dev)
        self.c_melblock = prep_block(sd, p + ".input_mel.conv_block", "none", None, False, dev)
        self.c_input = prep_plain(sd, p + ".input_conv", cfg.get("fb_kernel_size", 3), dev)
        self.c_enc, self.c_st = [], []
        st_rates = [rates[-1]]
        for r in rates[-2::-1]:
            st_rates.append(st_rates[-1] * r)
        self.c_st_rates = st_rates[::-1]
        for i in range(n_lvl):
            q = f"{p}.encoder.ds_modules.{i}"
            if i < len(rates):
                self.c_enc.append(prep_block(sd, q, "down", rates[i], False, dev))
            else:
                self.c_enc.append(prep_block(sd, q, "none", None, False, dev))
            if i < len(rates) - 1:
                self.c_st.append(prep_strided(sd, f"{p}.encoder.st_convs.{i}", self.c_st_rates[i], dev))
        self.c_cb1 = prep_block(sd, p + ".encoder.conv_block1", "none", None, False, dev)
        self.c_cb2 = prep_block(sd, p + ".encoder.conv_block2", "none", None, False, dev)
        self.c_gru = prep_gru(sd, p + ".encoder.gru", 2, dev)
        self.c_dec_in = prep_block(sd, p + ".decoder.input_conv_block", "none", None, False, dev)
        ups = rates[::-1]
        self.c_dec = []
        for l in range(n_lvl):
            q = f"{p}.decoder.up_modules.{l}"
            if self.c_extra and l == 0:
                self.c_dec.append(prep_block(sd, q, "none", None, False, dev))
            else:
                self.c_dec.append(prep_block(sd, q, "up", ups[l - (1 if self.c_extra else 0)], aa_dec, dev))

    def _prep_sdl(self, sd, p, dev):
        self.has_sdl = (p + ".conv.weight") in sd
        if not self.has_sdl:
            return
        a = sd[p + ".prelu.act.act.alpha"].float()
        self.sdl_alpha = torch.exp(a).contiguous().to(dev)
        ku, wu = dsp.sinc_resample_kernel(1, 2)
        kd, wd = dsp.sinc_resample_kernel(2, 1)
        self.sdl_kup = torch.from_numpy(ku.reshape(-1).copy()).to(dev)
        self.sdl_kdown = torch.from_numpy(kd.reshape(-1).copy()).to(dev)
        self.sdl_taps = (ku.shape[1], wu, kd.shape[1], wd)
        self.sdl_w = sd[p + ".conv.weight"].float().reshape(-1).contiguous().to(dev)
        self.sdl_b = float(sd[p + ".conv.bias"].reshape(-1)[0])

    # -------------------------------------------------------------- buffers
    def alloc_score(self, B, T):
        dev = self.device
        Ts = level_lengths(T, self.rates)
        n_lvl = len(self.s_enc)
        Cs = [self.nch * 2 ** i for i in range(len(self.rates) + 1)]
        bufs = {"T": Ts, "C": Cs}
        for i in range(n_lvl):
            li = min(i, len(self.rates))
            for k in ("E", "A", "B", "V"):
                bufs[f"{k}{i}"] = new_act(B, Cs[li], Ts[li], dev)
        H = self.s_gru.hidden
        bufs["GI"] = new_act(B, 6 * H, Ts[len(self.rates)], dev)
        bufs["gran"] = zeros((L.load().ou_gru_workspace_bytes(H, B) // 8,), dtype=torch.int64, device=dev)
        return bufs

    def score_levels(self):
        """decoder level l -> encoder level index i it mirrors."""
        n = len(self.s_enc)
        return [n - 1 - l for l in range(n)]

    def rec_score(self, prog, bufs, x: Act, film_base, film_bs, in_scale=0, sc_list=None, before_level=None,
                  head=None, after_encoder=None, gru_xcd=0):
        """ScoreNetwork.forward (score.py:278-298).  The encoder and the
        bottleneck GRU do not read the conditions (score.py:284-286), and
        decoder level l reads only condition l: ``before_level(l)`` runs right
        before decoder level l first needs it.  With ``head`` (an ou_head
        descriptor, h unset) the head is recorded too and None is returned;
        otherwise the decoder output Act is returned.  When the 32-channel end
        blocks are fused, the input conv runs inside the first encoder block and
        the head inside the last decoder block (ou_block kEpiIn / kEpiHead).
        ``after_encoder()`` runs between the encoder and the bottleneck GRU;
        ``gru_xcd`` rotates the GRU chains' XCDs (ou_gru_desc.flags bits 12-14:
        the same bits, other L2s than a GRU running beside it)."""
        n_lvl = len(self.s_enc)
        nr = len(self.rates)
        fb = lambda j: film_base + 4 * self.film_off[j]
        # input conv (score.py:244-246, 285)
        prog.label = "score enc"
        d_in = conv_desc(self.s_input, x, bufs["E0"], in_scale=in_scale)
        fuse_in = (self.s_enc[0].fused is not None and self.s_enc[0].C in ENDS_C and self.s_in_fusable
                   and fuse_ends_enabled())
        if not fuse_in:
            prog.add(L.OP_CONV, d_in)
        # encoder (score.py:105-115)
        for i in range(n_lvl):
            bw = self.s_enc[i]
            prog.label = f"score enc L{i}"
            x_in = (x, in_scale, self.s_in_w, self.s_in_b, d_in) if (i == 0 and fuse_in) else None
            rec_block(prog, bw, bufs[f"E{i}"], bufs[f"V{i}"], bufs[f"A{i}"], bufs[f"B{i}"],
                      film=fb(i), film_bs=film_bs, x_in=x_in,
                      e_out=bufs[f"E{i+1}"] if bw.kind == "down" else None)
        if after_encoder is not None:
            after_encoder()
        # bottleneck GRU, fused with the decoder's first residual add
        top = n_lvl - 1
        prog.label = "score gru"
        rec_gru(prog, self.s_gru, 0, bufs[f"V{top}"], bufs["GI"], bufs[f"V{top}"],
                bufs["gran"], self.status, res=bufs[f"V{top}"], res_scale=NF2, xcd=gru_xcd)
        # decoder (score.py:197-211)
        h = None
        for l in range(n_lvl):
            i = top - l
            bw = self.s_dec[l]
            prog.label = f"score dec L{i}"
            if bw.kind == "up":
                li = min(i, nr)
                add_conv(prog, conv_desc(bw.rate_conv, h, bufs[f"V{i}"], n_frames=h.T,
                                         out_len=bufs["T"][li], valid_len=bw.rate * h.T,
                                         res1=bufs[f"V{i}"], s1=NF2))
            # only the block's conv1 reads condition l (its input_cond
            # residual): the up conv above runs before the wait
            if before_level is not None:
                before_level(l)
            last = l == n_lvl - 1
            fuse_head = (last and head is not None and bw.fused is not None and bw.C in ENDS_C
                         and fuse_ends_enabled())
            rec_block(prog, bw, bufs[f"V{i}"], bufs[f"A{i}"], bufs[f"A{i}"], bufs[f"B{i}"],
                      film=fb(n_lvl + l), film_bs=film_bs, sc=sc_list[l], head=head if fuse_head else None)
            h = bufs[f"A{i}"]
            if last and head is not None:
                if not fuse_head:
                    head.h, head.h_bstride = h.ptr, h.bs
                    prog.add(L.OP_HEAD, head)
                return None
        return h

    def rec_sc(self, prog, conds, scs):
        for l, (c, s) in enumerate(zip(conds, scs)):
            prog.add(L.OP_CONV, conv_desc(self.s_sc[l], c, s))

    def alloc_sc(self, B, T):
        Ts = level_lengths(T, self.rates)
        n_lvl = len(self.s_enc)
        out = []
        for l in range(n_lvl):
            i = n_lvl - 1 - l
            li = min(i, len(self.rates))
            out.append(new_act(B, self.s_dec[l].C, Ts[li], self.device))
        return out

    def rec_embed(self, prog, sigma_dev, n, film_out, gbuf):
        d = L.EmbedDesc()
        d.sigma, d.n, d.kind, d.dim = sigma_dev.data_ptr(), n, self.emb_kind, self.emb_dim
        if self.emb_kind == 0:
            d.te_weight, d.te_bias = self.te_w, self.te_b
        else:
            d.rff_freq, d.n_rff = self.rff.data_ptr(), self.rff.numel()
            for k, (w, b, s) in enumerate(self.mlp):
                d.mlp_w[k], d.mlp_b[k], d.mlp_slope[k] = w.data_ptr(), b.data_ptr(), s
        d.rows = self.film_rows
        d.w, d.bias, d.out, d.gbuf = self.emb_w.data_ptr(), self.emb_b.data_ptr(), film_out.data_ptr(), gbuf.data_ptr()
        d._flops = 2.0 * self.film_rows * self.emb_dim * n
        prog.add(L.OP_EMBED, d)

    def head_desc(self, h: Optional[Act], out_ptr, B, T, mode=0, x_ptr=0, z_ptr=0, coef=None):
        """ou_head descriptor; h = None leaves the input unset (rec_score
        fills it in, or fuses the head into the last decoder block)."""
        d = L.HeadDesc()
        C = self.s_dec[-1].C
        if h is not None:
            d.h, d.h_bstride = h.ptr, h.bs
            C = h.C
        d.channels, d.length, d.batch, d.mode = C, T, B, mode
        d.slope1, d.slope2 = self.head_s1, self.head_s2
        d.w, d.bias = self.head_w.data_ptr(), self.head_b
        d.edm = 1 if self.edm is not None else 0
        if coef:
            for k, v in coef.items():
                setattr(d, k, float(v))
        d.x, d.z, d.out = x_ptr, z_ptr, out_ptr
        d._flops = 2.0 * C * 3 * T * B
        return d

    # -------------------------------------------------------------- conditioner
    def alloc_cond(self, B, T, need_aux=False):
        dev = self.device
        rates = list(self.ccfg["rate_factors"])
        Ts = level_lengths(T, rates)
        Cs = [self.ccfg["n_channels"] * 2 ** i for i in range(len(rates) + 1)]
        U = -(-T // self.mel_hop)
        bufs = {"T": Ts, "C": Cs, "U": U}
        bufs["SPEC"] = new_act(B, 2 * self.mel_nfreq, U, dev)
        bufs["POW"] = new_act(B, self.mel_nfreq, U, dev)
        bufs["MEL"] = new_act(B, self.mel_nmels, U, dev)
        bufs["INV"] = empty((B,), dtype=torch.float32, device=dev)
        CL = Cs[-1]
        for k in ("M0", "MA", "MB", "XMEL", "SUM", "OUT", "LA", "LB", "CB1", "G1", "G2", "H", "D0", "Y4"):
            bufs[k] = new_act(B, CL, U, dev)
        n_lvl = len(self.c_enc)
        for i in range(len(rates)):
            for k in ("E", "A", "B", "V"):
                bufs[f"{k}{i}"] = new_act(B, Cs[i], Ts[i], dev)
        bufs[f"E{len(rates)}"] = new_act(B, CL, Ts[len(rates)], dev)
        H = self.c_gru.hidden
        bufs["GI"] = new_act(B, 6 * H, U, dev)
        bufs["gran"] = zeros((L.load().ou_gru_workspace_bytes(H, B) // 8,), dtype=torch.int64, device=dev)
        # decoder: conditions per level + Y (block outputs) per level
        conds, ys = [], []
        for l in range(n_lvl):
            i = n_lvl - 1 - l
            li = min(i, len(rates))
            C = self.c_dec[l].C
            conds.append(new_act(B, C, Ts[li], dev))
            ys.append(new_act(B, C, Ts[li], dev))
        bufs["COND"] = conds
        bufs["Y"] = ys
        bufs["HUP"] = [new_act(B, self.c_dec[l].C, Ts[min(n_lvl - 1 - l, len(rates))], dev) for l in range(n_lvl)]
        bufs["TB"] = [new_act(B, self.c_dec[l].C, Ts[min(n_lvl - 1 - l, len(rates))], dev) for l in range(n_lvl)]
        return bufs

    def rec_cond(self, prog, bufs, x: Act, need_aux=False, after_level=None, st_lane=None):
        """ConditionerNetwork.forward (condition.py:346-377).  ``after_level(l,
        cond_l)`` runs right after decoder level l has produced its condition.
        With ``st_lane`` (recording on a side lane) the strided st_convs, which
        only feed the bottleneck level's residual, are recorded on lane
        ``st_lane`` instead, each behind a signal that its encoder level is
        done, and the bottleneck block waits for their sum: they run beside the
        next encoder levels instead of in line."""
        rates = list(self.ccfg["rate_factors"])
        nr = len(rates)
        n_lvl = len(self.c_enc)
        B, U = x.B, bufs["U"]
        # MelAdapter (condition.py:85-114): |STFT|^2 -> mel -> global norm -> conv -> ConvBlock.
        # Its output is read only by the last st_conv (as a residual), so with
        # ``st_lane`` it runs on a side lane of its own: neither the
        # conditioner's encoder -- the first step's critical path -- nor the
        # earlier st_convs wait for it
        # -- lane 2, so the st_convs do not queue behind it either.  It rejoins
        # through the last st_conv, so without st_convs (one rate factor) it
        # stays in line.
        mel_lane = 2 if st_lane is not None and nr >= 2 else None
        if mel_lane is not None and mel_lane not in (st_lane, 0):
            ev_m = prog.signal()   # a side lane starts by waiting on the conditioner lane
        if mel_lane is not None:
            side = _LANE
            set_lane(prog, mel_lane)
            if mel_lane not in (st_lane, 0):
                prog.wait(ev_m)
        prog.label = "cond mel"
        prog.add(L.OP_CONV, conv_desc(self.c_stft, x, bufs["SPEC"], n_frames=U))
        pa = L.PowerArgs(x=bufs["SPEC"].ptr, y=bufs["POW"].ptr, batch=B, nf=self.mel_nfreq, frames=U)
        prog.add(L.OP_POWER, pa)
        prog.add(L.OP_CONV, conv_desc(self.c_fb, bufs["POW"], bufs["MEL"]))
        ra = L.RmsArgs(x=bufs["MEL"].ptr, out=bufs["INV"].data_ptr(), batch=B,
                       n=self.mel_nmels * U, denom=float(U), eps=1e-5)
        prog.add(L.OP_INV_RMS, ra)
        prog.add(L.OP_CONV, conv_desc(self.c_melconv, bufs["MEL"], bufs["M0"], in_scale=bufs["INV"].data_ptr()))
        rec_block(prog, self.c_melblock, bufs["M0"], bufs["XMEL"], bufs["MA"], bufs["MB"])
        ev_mel = None
        if mel_lane is not None:
            if mel_lane not in (st_lane, 0):
                ev_mel = prog.signal()   # the last st_conv adds XMEL
            set_lane(prog, side)
        # encoder (condition.py:189-220)
        prog.label = "cond enc L0"
        prog.add(L.OP_CONV, conv_desc(self.c_input, x, bufs["E0"]))
        nsum = 0
        for i in range(n_lvl):
            bw = self.c_enc[i]
            prog.label = f"cond enc L{i}"
            if i < nr:
                rec_block(prog, bw, bufs[f"E{i}"], bufs[f"V{i}"], bufs[f"A{i}"], bufs[f"B{i}"],
                          e_out=bufs[f"E{i+1}"])
                if i < nr - 1:
                    # SUM = x_mel + st_0 + st_1 + ... (condition.py:208-215),
                    # accumulated in the st_convs' epilogues.  The mel branch
                    # is added by the LAST st_conv, so the earlier ones run as
                    # soon as their encoder level is done instead of queueing
                    # behind the mel front end (a reassociated fp32 sum)
                    last_st = i == nr - 2
                    if nr - 1 == 1:
                        res_a, res_b = bufs["XMEL"], None
                    elif nsum == 0:
                        res_a, res_b = None, None
                    else:
                        res_a, res_b = bufs["SUM"], (bufs["XMEL"] if last_st else None)
                    if st_lane is not None:
                        side = _LANE
                        ev = prog.signal()
                        set_lane(prog, st_lane)
                        prog.wait(ev)
                        if ev_mel is not None and (res_a is bufs["XMEL"] or res_b is not None):
                            prog.wait(ev_mel)
                    prog.label = f"cond st{i}"
                    dst = conv_desc(self.c_st[i], bufs[f"V{i}"], bufs["SUM"], n_frames=U, res1=res_a, s1=1.0,
                                    res2=res_b, s2=1.0)
                    # never a split-image consumer: where it is recorded (in
                    # line, or on lane 0 behind a wait) must not change its
                    # bits -- enhance_many's plans keep it in line
                    dst._no_split = True
                    add_conv(prog, dst)   # the FIR kernels' st_conv form (fir 3) where it is faster
                    prog.label = f"cond enc L{i}"
                    if st_lane is not None:
                        set_lane(prog, side)
                    nsum += 1
            else:
                if st_lane is not None and nsum:
                    side = _LANE
                    set_lane(prog, st_lane)
                    ev = prog.signal()
                    set_lane(prog, side)
                    prog.wait(ev)
                n_out = nsum + 1
                nf = np.float32(1.0 / math.sqrt(n_out + 1))
                rec_block(prog, bw, bufs[f"E{i}"], bufs["OUT"], bufs["LA"], bufs["LB"],
                          res2=bufs["SUM"], s2=nf)
        if not self.c_extra:
            raise NotImplementedError("conditioner without extra_conv_block")
        prog.label = "cond cb1"
        rec_block(prog, self.c_cb1, bufs["OUT"], bufs["CB1"], bufs["LA"], bufs["LB"])
        prog.label = "cond gru1"
        rec_gru(prog, self.c_gru, 0, bufs["CB1"], bufs["GI"], bufs["G1"], bufs["gran"], self.status)
        res = bufs["CB1"] if self.c_gru_res else None
        prog.label = "cond gru2"
        rec_gru(prog, self.c_gru, 1, bufs["G1"], bufs["GI"], bufs["G2"], bufs["gran"], self.status,
                res=res, res_scale=NF2)
        prog.label = "cond cb2"
        rec_block(prog, self.c_cb2, bufs["G2"], bufs["H"], bufs["LA"], bufs["LB"])
        # decoder (condition.py:264-270)
        prog.label = "cond dec in"
        rec_block(prog, self.c_dec_in, bufs["H"], bufs["D0"], bufs["LA"], bufs["LB"])
        h = bufs["D0"]
        for l in range(n_lvl):
            bw = self.c_dec[l]
            i = n_lvl - 1 - l
            li = min(i, nr)
            prog.label = f"cond dec L{i}"
            if bw.kind == "up":
                hup = bufs["HUP"][l]
                prog.add(L.OP_CONV, conv_desc(bw.rate_conv, h, hup, n_frames=h.T,
                                              out_len=bufs["T"][li], valid_len=bw.rate * h.T))
                h = hup
            last = l == n_lvl - 1
            # condition l is conv1's output (blocks.py:402-407): the consumer
            # hook runs as soon as conv1 is done, before the block's conv2 /
            # conv3 (unfused 256 / 512-channel levels: the first score
            # decoder level starts two launches earlier)
            hook = (lambda l=l: after_level(l, bufs["COND"][l])) if after_level is not None else None
            rec_block(prog, bw, h, bufs["Y"][l], None, bufs["TB"][l], cond_out=bufs["COND"][l],
                      skip_tail=last and not need_aux, after_c1=hook)
            h = bufs["Y"][l]
        return bufs["COND"], bufs["Y"][-1]

    # -------------------------------------------------------------- aux path
    def rec_aux(self, prog, y: Act, tmp: Act, out_ptr, B, T):
        """UniverseGAN.aux_to_wav (universe_gan.py:147-151)."""
        d = L.SnakeDesc()
        d.h, d.h_bstride = y.ptr, y.bs
        d.channels, d.length, d.batch = y.C, T, B
        tu, wu, td, wd = self.sdl_taps
        d.alpha, d.k_up, d.taps_up, d.width_up = self.sdl_alpha.data_ptr(), self.sdl_kup.data_ptr(), tu, wu
        d.k_down, d.taps_down, d.width_down, d.out = self.sdl_kdown.data_ptr(), td, wd, tmp.ptr
        prog.add(L.OP_SNAKE, d)
        h = L.HeadDesc()
        h.h, h.h_bstride, h.channels, h.length, h.batch, h.mode = tmp.ptr, tmp.bs, tmp.C, T, B, 0
        h.slope1 = h.slope2 = 1.0
        h.w, h.bias, h.out = self.sdl_w.data_ptr(), self.sdl_b, out_ptr
        prog.add(L.OP_HEAD, h)
