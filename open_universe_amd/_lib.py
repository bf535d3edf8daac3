"""ctypes binding of libouhip.so (the C ABI declared in include/ouhip.h).

This is the "reference-side binding a maintainer would add": the reference is
pure Python, so the natural FFI is ctypes over the C ABI.  The library is built
in-tree (``__graft_entry__.build()`` / ``open_universe_amd/csrc/build.sh``) and
loaded from ``open_universe_amd/libouhip.so``.  There is no fallback: if the
library is missing, every compute entry point raises.
"""
import ctypes
import os
from ctypes import POINTER, c_float, c_int, c_int32, c_int64, c_size_t, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OUHIP_LIB", os.path.join(_HERE, "libouhip.so"))
ABI_VERSION = 8

fp = c_void_p  # device pointers are passed as integers

# op codes (ouhip.h)
OP_CONV, OP_GRU, OP_EMBED, OP_HEAD = 1, 2, 3, 4
OP_NORMALIZE, OP_INV_RMS, OP_POWER, OP_PAD = 5, 6, 7, 8
OP_SCALE, OP_FINISH, OP_RMS, OP_SNAKE = 9, 10, 11, 12
OP_MEMSET, OP_ENSEMBLE, OP_BLOCK = 13, 14, 15
OP_LANE, OP_SIGNAL, OP_WAIT = 16, 17, 18   # program lanes (side streams) and their events


class ConvDesc(ctypes.Structure):
    _fields_ = [
        ("x", fp), ("x_bstride", c_int64), ("x_cstride", c_int64),
        ("cin", c_int32), ("in_len", c_int32), ("frame", c_int32), ("shift", c_int32),
        ("in_scale", fp), ("slope", c_float), ("w", fp),
        ("m", c_int32), ("kt", c_int32), ("pad", c_int32), ("cc", c_int32),
        ("n_frames", c_int32), ("batch", c_int32),
        ("y", fp), ("y_bstride", c_int64), ("y_cstride", c_int64),
        ("rout", c_int32), ("out_len", c_int32), ("valid_len", c_int32),
        ("bias", fp),
        ("res1", fp), ("r1_bstride", c_int64), ("r1_cstride", c_int64), ("s1", c_float),
        ("film", fp), ("film_bstride", c_int64),
        ("res2", fp), ("r2_bstride", c_int64), ("r2_cstride", c_int64), ("s2", c_float),
        ("tile", c_int32), ("prec", c_int32), ("w_unscale", c_float), ("f0", c_int32),
        ("status", fp), ("ks_ws", fp), ("ks_ws_bytes", c_int64),
        ("sy", fp), ("sy_bstride", c_int64), ("sy_rows", c_int32), ("sy_shift", c_int32),
        ("sy_slope", c_float), ("sy_pad_", c_int32),
        ("xs", fp), ("xs_bstride", c_int64), ("xs_rows", c_int32), ("xs_shift", c_int32),
        ("fir", c_int32), ("fir_pad_", c_int32), ("fir_taps", fp),
    ]


class GruDesc(ctypes.Structure):
    _fields_ = [
        ("gi", fp), ("gi_bstride", c_int64), ("w_hh", fp), ("b_hh", fp),
        ("y", fp), ("y_bstride", c_int64), ("y_cstride", c_int64),
        ("res", fp), ("res_bstride", c_int64), ("res_cstride", c_int64),
        ("res_scale", c_float), ("hidden", c_int32), ("steps", c_int32), ("batch", c_int32),
        ("flags", c_int32), ("granules", fp), ("status", fp), ("t_begin", c_int32), ("t_end", c_int32),
        ("hstate", fp), ("ws_zeroed", c_int32), ("_pad", c_int32),
    ]


class EmbedDesc(ctypes.Structure):
    _fields_ = [
        ("sigma", fp), ("n", c_int32), ("kind", c_int32), ("dim", c_int32),
        ("te_weight", c_float), ("te_bias", c_float), ("rff_freq", fp), ("n_rff", c_int32),
        ("rows", c_int32), ("mlp_w", fp * 3), ("mlp_b", fp * 3), ("mlp_slope", c_float * 3),
        ("w", fp), ("bias", fp), ("out", fp), ("gbuf", fp),
    ]


class HeadDesc(ctypes.Structure):
    _fields_ = [
        ("h", fp), ("h_bstride", c_int64),
        ("channels", c_int32), ("length", c_int32), ("batch", c_int32), ("mode", c_int32),
        ("slope1", c_float), ("slope2", c_float), ("w", fp), ("bias", c_float),
        ("edm", c_int32), ("_pad", c_int32),
        ("w_skip", c_float), ("w_out", c_float), ("s2", c_float), ("c_score", c_float),
        ("c_noise", c_float), ("s_next", c_float),
        ("x", fp), ("z", fp), ("out", fp),
    ]


class SnakeDesc(ctypes.Structure):
    _fields_ = [
        ("h", fp), ("h_bstride", c_int64),
        ("channels", c_int32), ("length", c_int32), ("batch", c_int32), ("_pad0", c_int32),
        ("alpha", fp), ("k_up", fp), ("taps_up", c_int32), ("width_up", c_int32),
        ("k_down", fp), ("taps_down", c_int32), ("width_down", c_int32), ("out", fp),
    ]


class SyncArgs(ctypes.Structure):
    _fields_ = [("id", c_int32), ("_pad", c_int32)]


class MemsetArgs(ctypes.Structure):
    _fields_ = [("ptr", fp), ("bytes", c_int64)]


class NormArgs(ctypes.Structure):
    _fields_ = [("x", fp), ("y", fp), ("batch", c_int32), ("_pad", c_int32), ("n", c_int64),
                ("level", c_float), ("eps", c_float)]


class RmsArgs(ctypes.Structure):
    _fields_ = [("x", fp), ("out", fp), ("batch", c_int32), ("_pad", c_int32), ("n", c_int64),
                ("denom", c_float), ("eps", c_float)]


class PowerArgs(ctypes.Structure):
    _fields_ = [("x", fp), ("y", fp), ("batch", c_int32), ("nf", c_int32),
                ("frames", c_int32), ("_pad", c_int32)]


class PadArgs(ctypes.Structure):
    _fields_ = [("x", fp), ("x_bstride", c_int64), ("y", fp), ("batch", c_int32),
                ("n_in", c_int32), ("n_out", c_int32), ("left", c_int32)]


class ScaleArgs(ctypes.Structure):
    _fields_ = [("z", fp), ("y", fp), ("n", c_int64), ("scale", c_float), ("_pad", c_float),
                ("add", fp)]


class FinishArgs(ctypes.Structure):
    _fields_ = [("x", fp), ("x_bstride", c_int64), ("left", c_int32), ("batch", c_int32),
                ("len", c_int32), ("_pad", c_int32), ("y", fp), ("mix_rms", fp)]


class EnsembleArgs(ctypes.Structure):
    _fields_ = [("x", fp), ("y", fp), ("ensemble", c_int32), ("mode", c_int32), ("n", c_int64),
                ("batch", c_int32), ("_pad", c_int32), ("counts", c_void_p)]


class BlockDesc(ctypes.Structure):
    _fields_ = [
        ("h", fp), ("h_bstride", c_int64), ("h_cstride", c_int64),
        ("channels", c_int32), ("length", c_int32), ("batch", c_int32), ("prec", c_int32),
        ("w", fp * 3), ("bias", fp * 3), ("slope", c_float * 3), ("w_unscale", c_float * 3),
        ("sc", fp), ("sc_bstride", c_int64), ("sc_cstride", c_int64), ("s_sc", c_float), ("dbg", c_int32),
        ("film", fp), ("film_bstride", c_int64),
        ("cond_out", fp), ("co_bstride", c_int64), ("co_cstride", c_int64),
        ("y", fp), ("y_bstride", c_int64), ("y_cstride", c_int64), ("s_res", c_float), ("s2", c_float),
        ("res2", fp), ("r2_bstride", c_int64), ("r2_cstride", c_int64),
        ("status", fp),
        ("x", fp), ("x_bstride", c_int64), ("in_scale", fp), ("w_in", fp), ("b_in", fp),
        ("head", HeadDesc),
        ("w_down", fp), ("b_down", fp), ("slope_down", c_float), ("w_down_unscale", c_float),
        ("rate", c_int32), ("down_kt", c_int32), ("e", fp), ("e_bstride", c_int64), ("e_cstride", c_int64),
        ("f0", c_int32), ("f1", c_int32), ("h0", c_int32), ("h1", c_int32),
        ("shift", c_int32 * 4),
        ("sy", fp), ("sy_bstride", c_int64), ("sy_rows", c_int32), ("sy_shift", c_int32),
        ("sy_slope", c_float), ("sy_pad_", c_int32),
        ("xs", fp), ("xs_bstride", c_int64), ("xs_rows", c_int32), ("xs_pad_", c_int32),
    ]


OP_STRUCT = {
    OP_CONV: ConvDesc, OP_GRU: GruDesc, OP_EMBED: EmbedDesc, OP_HEAD: HeadDesc,
    OP_NORMALIZE: NormArgs, OP_INV_RMS: RmsArgs, OP_RMS: RmsArgs, OP_POWER: PowerArgs,
    OP_PAD: PadArgs, OP_SCALE: ScaleArgs, OP_FINISH: FinishArgs, OP_SNAKE: SnakeDesc,
    OP_MEMSET: MemsetArgs, OP_ENSEMBLE: EnsembleArgs, OP_BLOCK: BlockDesc,
    OP_LANE: SyncArgs, OP_SIGNAL: SyncArgs, OP_WAIT: SyncArgs,
}

# every symbol include/ouhip.h declares (checked by tests/test_abi.py)
EXPORTS = {
    "ou_abi_version": (c_int, []),
    "ou_last_error": (ctypes.c_char_p, []),
    "ou_conv_chunk": (c_int, [c_int, c_int]),
    "ou_conv_packed_size": (c_int64, [c_int, c_int, c_int, c_int]),
    "ou_conv_pack": (c_int, [POINTER(c_float), c_int, c_int, c_int, c_int, POINTER(c_float)]),
    "ou_conv_pack_split": (c_int, [POINTER(c_float), c_int, c_int, c_int, POINTER(c_float),
                                   POINTER(c_float)]),
    "ou_conv_pack_split_nat": (c_int, [POINTER(c_float), c_int, c_int, c_int, POINTER(c_float),
                                       POINTER(c_float)]),
    "ou_conv": (c_int, [POINTER(ConvDesc), c_void_p]),
    "ou_conv_pick_tile": (c_int, [POINTER(ConvDesc)]),
    "ou_conv_num_tiles": (c_int, []),
    "ou_conv_tile_ok": (c_int, [c_int, c_int]),
    "ou_conv_lds_info": (c_int, [c_int, c_int, POINTER(c_int), POINTER(c_int)]),
    "ou_gru_workspace_bytes": (c_int64, [c_int, c_int]),
    "ou_gru": (c_int, [POINTER(GruDesc), c_void_p]),
    "ou_embed": (c_int, [POINTER(EmbedDesc), c_void_p]),
    "ou_head": (c_int, [POINTER(HeadDesc), c_void_p]),
    "ou_normalize": (c_int, [fp, fp, c_int, c_int64, c_float, c_float, c_void_p]),
    "ou_inv_rms": (c_int, [fp, fp, c_int, c_int64, c_float, c_float, c_void_p]),
    "ou_rms": (c_int, [fp, fp, c_int, c_int64, c_void_p]),
    "ou_power": (c_int, [fp, fp, c_int, c_int, c_int, c_void_p]),
    "ou_pad": (c_int, [fp, c_int64, fp, c_int, c_int, c_int, c_int, c_void_p]),
    "ou_scale": (c_int, [fp, fp, c_int64, c_float, fp, c_void_p]),
    "ou_finish": (c_int, [fp, c_int64, c_int, fp, c_int, c_int, fp, c_void_p]),
    "ou_ensemble_reduce": (c_int, [fp, fp, c_int, c_int64, c_int, c_void_p]),
    "ou_signal_median": (c_int, [fp, fp, c_int, c_int, c_int64, c_void_p, c_void_p]),
    "ou_snake_aa": (c_int, [POINTER(SnakeDesc), c_void_p]),
    "ou_block_supported": (c_int, [c_int, c_int]),
    "ou_block_frames": (c_int, [c_int]),
    "ou_block_packed_halves": (c_int64, [c_int, c_int]),
    "ou_block_pack": (c_int, [POINTER(c_float), c_int, c_int, c_void_p, POINTER(c_float)]),
    "ou_block_packed_f32": (c_int64, [c_int, c_int]),
    "ou_block_pack_f32": (c_int, [POINTER(c_float), c_int, c_int, POINTER(c_float), POINTER(c_float)]),
    "ou_block_pack_rect": (c_int, [POINTER(c_float), c_int, c_int, c_int, c_void_p, POINTER(c_float)]),
    "ou_block_down_supported": (c_int, [c_int, c_int, c_int, c_int]),
    "ou_block": (c_int, [POINTER(BlockDesc), c_void_p]),
    "ou_resample": (c_int, [fp, c_int64, fp, c_int64, c_int, c_int, c_int, fp, c_int, c_int, c_int, c_int,
                            c_void_p]),
    "ou_flac_info": (c_int, [c_void_p, c_int64, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32),
                             POINTER(c_int64)]),
    "ou_flac_decode": (c_int64, [c_void_p, c_int64, c_void_p, c_int64]),
    "ou_flac_encode_bound": (c_int64, [c_int, c_int64, c_int]),
    "ou_flac_encode": (c_int64, [c_void_p, c_int, c_int64, c_int, c_int, c_void_p, c_int64]),
    "ou_program_create": (c_void_p, []),
    "ou_program_destroy": (None, [c_void_p]),
    "ou_program_add": (c_int, [c_void_p, c_int, c_void_p, c_size_t]),
    "ou_program_patch": (c_int, [c_void_p, c_int, c_int, c_void_p, c_size_t]),
    "ou_program_size": (c_int, [c_void_p]),
    "ou_program_run": (c_int, [c_void_p, c_void_p]),
    "ou_program_capture": (c_int, [c_void_p]),
    "ou_program_capture_segments": (c_int, [c_void_p]),
    "ou_program_validate": (c_int, [c_void_p]),
    "ou_program_launch": (c_int, [c_void_p, c_void_p]),
    "ou_program_op_kind": (c_int, [c_void_p, c_int]),
    "ou_program_profile": (c_int, [c_void_p, c_void_p, POINTER(c_float)]),
    "ou_program_trace": (c_int, [c_void_p, c_void_p, POINTER(c_float), POINTER(c_float)]),
}

_lib = None


class OuHipError(RuntimeError):
    pass


class OuRangeError(OuHipError):
    """A split-f16 operand left its range (|prelu(x)| 2^-s >= 2^15 for the
    layer's staging exponent s): the result of that replay is not valid.
    ``flags``: the (layer slot, range code) pairs that name the layers
    (Engine.widen_ranges widens their exponents; empty: rerun in f32)."""
    flags = ()


def load():
    """Load libouhip.so (raises if it is missing -- no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OuHipError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
            "g.build()'` or open_universe_amd/csrc/build.sh")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in EXPORTS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.ou_abi_version() != ABI_VERSION:
        raise OuHipError("libouhip ABI version mismatch")
    _lib = lib
    return lib


def check(rc, what=""):
    if rc != 0:
        msg = load().ou_last_error()
        raise OuHipError(f"{what}: ouhip error {rc}: {msg.decode() if msg else ''}")


def conv_chunk(kt, frame):
    return load().ou_conv_chunk(kt, frame)


def conv_pack(w_logical, cc):
    """w_logical: float32 numpy array [m][cin_eff][kt] -> packed numpy array."""
    import numpy as np

    w = np.ascontiguousarray(w_logical, dtype=np.float32)
    m, cin, kt = w.shape
    n = load().ou_conv_packed_size(m, cin, kt, cc)
    out = np.empty(n, dtype=np.float32)
    check(load().ou_conv_pack(w.ctypes.data_as(POINTER(c_float)), m, cin, kt, cc,
                              out.ctypes.data_as(POINTER(c_float))), "conv_pack")
    return out


def _split_scale(w):
    """Per-layer power-of-two scale of the split packings: max|w * 2^e| in
    [2^9, 2^10); returns (2^e, w_unscale = 2^(6 - e))."""
    import numpy as np

    if not np.isfinite(w).all():
        raise OuHipError("split packing: non-finite weight")
    mx = float(np.abs(w).max()) if w.size else 0.0
    e = 0
    if mx > 0.0:
        e = min(100, max(-100, 10 - int(np.frexp(np.float32(mx))[1])))
    return np.float32(2.0**e), float(2.0 ** (6 - e))


def _hi_lo(a):
    import numpy as np

    hi = a.astype(np.float16)
    lo = ((a - hi.astype(np.float32)) * np.float32(2048.0)).astype(np.float16)
    return hi, lo


def conv_pack_split_np(w_logical):
    """ou_conv_pack_split restated with numpy array ops (byte-identical,
    tests/test_weight_prep.py): the C loop converts to f16 in software on the
    host and dominates model load time."""
    import numpy as np

    w = np.ascontiguousarray(w_logical, dtype=np.float32)
    m, cin, kt = w.shape
    sc, unscale = _split_scale(w)
    mt = (m + 31) // 32
    cpad = (cin + 63) // 64 * 64
    a = np.zeros((mt * 32, cpad, kt), dtype=np.float32)
    a[:m, :cin] = w * sc
    # out[mt][g][part][k][lane = h*32 + r][j] = a[mt*32 + r][16 g + 2 j + h][k]
    a = a.reshape(mt, 32, cpad // 16, 8, 2, kt).transpose(0, 2, 5, 4, 1, 3)   # mt, g, k, h, r, j
    hi, lo = _hi_lo(np.ascontiguousarray(a))
    out = np.stack([hi, lo], axis=2)                                           # mt, g, part, k, h, r, j
    return np.ascontiguousarray(out).reshape(-1).view(np.float32), unscale


def conv_pack_split_nat_np(w_logical):
    """ou_conv_pack_split_nat restated with numpy (byte-identical): [mt][g]
    [hi|lo][k][lane = h*32 + r][j] of a[mt*32 + r][16 g + 8 h + j][k] -- the
    natural channel order of the split-image kernel (tile bit 15)."""
    import numpy as np

    w = np.ascontiguousarray(w_logical, dtype=np.float32)
    m, cin, kt = w.shape
    sc, unscale = _split_scale(w)
    mt = (m + 31) // 32
    cpad = (cin + 63) // 64 * 64
    a = np.zeros((mt * 32, cpad, kt), dtype=np.float32)
    a[:m, :cin] = w * sc
    a = a.reshape(mt, 32, cpad // 16, 2, 8, kt).transpose(0, 2, 5, 3, 1, 4)   # mt, g, k, h, r, j
    hi, lo = _hi_lo(np.ascontiguousarray(a))
    out = np.stack([hi, lo], axis=2)                                           # mt, g, part, k, h, r, j
    return np.ascontiguousarray(out).reshape(-1).view(np.float32), unscale


def block_pack_np(w_logical):
    """ou_block_pack restated with numpy (byte-identical): [mt][tap][ks][hi|lo]
    [lane = h*32 + r][i] of a[mt*32 + r][16 ks + 8 h + i][tap]."""
    import numpy as np

    w = np.ascontiguousarray(w_logical, dtype=np.float32)
    m, c, kt = w.shape
    assert m % 32 == 0 and c % 16 == 0, w.shape
    sc, unscale = _split_scale(w)
    a = (w * sc).reshape(m // 32, 32, c // 16, 2, 8, kt).transpose(0, 5, 2, 3, 1, 4)   # mt, k, ks, h, r, i
    hi, lo = _hi_lo(np.ascontiguousarray(a))
    out = np.stack([hi, lo], axis=3)                                                   # mt, k, ks, part, h, r, i
    return np.ascontiguousarray(out).reshape(-1).view(np.int16), unscale


def block_pack_f32_np(w_logical):
    """ou_block_pack_f32 restated with numpy (byte-identical): [mt][tap][s4]
    [lane = h*32 + r][j] of w[mt*32 + r][2 (4 s4 + j) + h][tap] (rows already
    padded to a multiple of 32); w_unscale = 2^6."""
    import numpy as np

    w = np.ascontiguousarray(w_logical, dtype=np.float32)
    m, c, kt = w.shape
    assert m % 32 == 0 and c % 16 == 0, w.shape
    a = w.reshape(m // 32, 32, c // 8, 4, 2, kt).transpose(0, 5, 2, 4, 1, 3)   # mt, k, s4, h, r, j
    return np.ascontiguousarray(a).reshape(-1), 64.0


def block_pack_f32(w_logical):
    """ou_block_pack_f32 through the C ABI (channels x channels x kt)."""
    import numpy as np

    w = np.ascontiguousarray(w_logical, dtype=np.float32)
    c, _, kt = w.shape
    out = np.empty(load().ou_block_packed_f32(c, kt), dtype=np.float32)
    un = c_float(0.0)
    check(load().ou_block_pack_f32(w.ctypes.data_as(POINTER(c_float)), c, kt, out.ctypes.data_as(POINTER(c_float)),
                                   ctypes.byref(un)), "block_pack_f32")
    return out, float(un.value)


def conv_pack_split(w_logical, natural=False):
    """Split-f16 packing (ConvDesc.prec = 1) through the C ABI: returns
    (packed, w_unscale); natural: ou_conv_pack_split_nat's channel order."""
    import numpy as np

    w = np.ascontiguousarray(w_logical, dtype=np.float32)
    m, cin, kt = w.shape
    n = load().ou_conv_packed_size(m, cin, kt, 0)
    out = np.empty(n, dtype=np.float32)
    un = c_float(0.0)
    fn = load().ou_conv_pack_split_nat if natural else load().ou_conv_pack_split
    check(fn(w.ctypes.data_as(POINTER(c_float)), m, cin, kt, out.ctypes.data_as(POINTER(c_float)),
             ctypes.byref(un)), "conv_pack_split")
    return out, float(un.value)


def block_pack(w_logical):
    """Fused-block packing of one m x C x kt conv (ou_block_pack_rect; m = C
    for the block's own convs): returns (packed f16 as an int16 numpy array,
    w_unscale)."""
    import numpy as np

    w = np.ascontiguousarray(w_logical, dtype=np.float32)
    m, c, kt = w.shape
    out = np.empty(2 * m * c * kt, dtype=np.int16)
    un = c_float(0.0)
    check(load().ou_block_pack_rect(w.ctypes.data_as(POINTER(c_float)), m, c, kt, out.ctypes.data,
                                    ctypes.byref(un)), "block_pack")
    return out, float(un.value)


# tile bit 16 (ou_conv.hip kMajBit): m-groups fastest in the workgroup order,
# so every input window is fetched from HBM once and re-read by its other
# m-groups from the XCD's L2.  Chosen for inputs too large to stay in the
# caches between m-groups (OUHIP_MMAJOR_MB, default 128 MB of input per
# launch; OUHIP_MMAJOR=0 never): the batched long-signal levels (C4).
MAJ_BIT = 1 << 16
_MMAJOR = os.environ.get("OUHIP_MMAJOR", "1") != "0"
_MMAJOR_BYTES = float(os.environ.get("OUHIP_MMAJOR_MB", "128")) * 2**20


FIR_BIT = 1 << 17   # FIR-applied rate-change kernels (bits 0-7 shape, bit 8 early epilogue loads)


def mmajor_order(desc):
    multi = desc.tile & ((3 << 8) | (1 << 10)) and not desc.tile & FIR_BIT
    if not _MMAJOR or multi:   # one-tile, register-streamed and FIR kernels only
        return False
    in_bytes = 4.0 * desc.batch * desc.cin * desc.frame * desc.n_frames
    return in_bytes > _MMAJOR_BYTES


# Optional per-layer tile autotuner for ou_conv (set by the engine on a GPU):
# called with a ConvDesc whose tile is -1, returns the tile id to record.
TUNER = None


ADD_HOOK = None   # engine.split_hook while a plan records: links an op to its producer's split image
                 # (ADD_HOOK.note(prog, index, op, desc) then sees every op added)
SS_BIT = 1 << 15  # ConvDesc.tile bit: the split-image kernel (conv_skernel), bits 0-7 = NR - 1


class Program:
    """A recorded launch list (ou_program) with optional hipGraph replay."""

    def __init__(self):
        self.lib = load()
        self.h = self.lib.ou_program_create()
        self.keep = []          # tensors whose memory the program references
        self.cur_lane = 0
        self.captured = False
        self.flops = []         # algorithmic FLOPs of the reference ops each op replaces
        self.bytes = []         # algorithmic HBM bytes of each op (0 where not counted)
        self.info = []          # per-op geometry (profiling / reports)
        self.lanes = []         # lane of each op
        self.label = ""         # phase label recorded with each op (engine sets it; reports only)
        self.labels = []
        self.descs = []         # each op's descriptor (patched in place by the split-image hook; hazards.py)

    def add(self, op, desc):
        assert isinstance(desc, OP_STRUCT[op])
        if op == OP_LANE:
            self.cur_lane = desc.id
        if op in (OP_CONV, OP_BLOCK) and ADD_HOOK is not None:
            ADD_HOOK(self, op, desc)   # may link it to the lane's previous op (split image)
        if op == OP_CONV and desc.tile < 0 and TUNER is not None:
            desc.tile = TUNER(desc)
        if op == OP_CONV and desc.tile >= 0 and mmajor_order(desc):
            desc.tile |= MAJ_BIT
        check(self.lib.ou_program_add(self.h, op, ctypes.byref(desc), ctypes.sizeof(desc)),
              f"program_add(op={op})")
        if ADD_HOOK is not None and hasattr(ADD_HOOK, "note"):
            ADD_HOOK.note(self, len(self.flops), op, desc)   # the split-image producers' bookkeeping
        self.descs.append(desc)
        self.flops.append(float(getattr(desc, "_flops", 0.0)))
        self.bytes.append(float(getattr(desc, "_bytes", 0.0)))
        self.lanes.append(self.cur_lane)
        self.labels.append(self.label)
        if op == OP_CONV:
            self.info.append({"m": desc.m, "cin": desc.cin, "frame": desc.frame, "kt": desc.kt,
                              "n": desc.n_frames, "b": desc.batch, "rout": desc.rout,
                              "tile": desc.tile, "fir": desc.fir})
        elif op == OP_GRU:
            self.info.append({"H": desc.hidden, "T": desc.steps, "b": desc.batch})
        elif op == OP_BLOCK:
            self.info.append({"C": desc.channels, "n": desc.length, "b": desc.batch, "prec": desc.prec,
                              "rate": desc.rate if desc.e else 0, "head": bool(desc.head.w), "in": bool(desc.x)})
        else:
            self.info.append({})

    # ---- lanes: concurrent branches of the recorded program (side streams
    # in eager replay, parallel branches of the captured hipGraph)
    def lane(self, i):
        self.add(OP_LANE, SyncArgs(id=i))

    def new_event(self):
        self.n_events = getattr(self, "n_events", 0) + 1
        return self.n_events - 1

    def signal(self, ev=None):
        ev = self.new_event() if ev is None else ev
        self.add(OP_SIGNAL, SyncArgs(id=ev))
        return ev

    def wait(self, ev):
        self.add(OP_WAIT, SyncArgs(id=ev))

    def patch(self, index, op, desc):
        """Re-send op ``index``'s descriptor after changing it (before capture)."""
        check(self.lib.ou_program_patch(self.h, index, op, ctypes.byref(desc), ctypes.sizeof(desc)),
              f"program_patch({index})")

    def __len__(self):
        return self.lib.ou_program_size(self.h)

    def run(self, stream):
        check(self.lib.ou_program_run(self.h, c_void_p(stream)), "program_run")

    def validate(self):
        """Host-only lane-structure check (no HIP call): raises on error."""
        check(self.lib.ou_program_validate(self.h), "program_validate")

    def capture(self, segments=None):
        """Capture as one hipGraph, or (segments, env OUHIP_GRAPH_MODE=seg)
        one hipGraph per run of kernels on a lane, replayed on real streams."""
        import os

        if segments is None:
            segments = os.environ.get("OUHIP_GRAPH_MODE", "whole") == "seg"
        fn = self.lib.ou_program_capture_segments if segments else self.lib.ou_program_capture
        check(fn(self.h), "program_capture")
        self.captured = True

    def launch(self, stream):
        check(self.lib.ou_program_launch(self.h, c_void_p(stream)), "program_launch")

    def op_kinds(self):
        return [self.lib.ou_program_op_kind(self.h, i) for i in range(len(self))]

    def profile(self, stream):
        """Eager replay with an event pair around each op -> per-op ms."""
        n = len(self)
        buf = (c_float * n)()
        check(self.lib.ou_program_profile(self.h, c_void_p(stream), buf), "program_profile")
        return list(buf)

    def trace(self, stream):
        """Eager replay with the lanes on their streams and events around
        each op -> per-op (start ms, end ms) from the replay's start (None
        for sync ops)."""
        n = len(self)
        a, b = (c_float * n)(), (c_float * n)()
        check(self.lib.ou_program_trace(self.h, c_void_p(stream), a, b), "program_trace")
        return [(x, y) if x >= 0 else None for x, y in zip(a, b)]

    def __del__(self):
        try:
            if self.h:
                self.lib.ou_program_destroy(self.h)
                self.h = None
        except Exception:
            pass


def run_now(op, desc, stream):
    """Launch one op immediately (used by layer-level tests)."""
    lib = load()
    fns = {OP_CONV: lib.ou_conv, OP_GRU: lib.ou_gru, OP_EMBED: lib.ou_embed,
           OP_HEAD: lib.ou_head, OP_SNAKE: lib.ou_snake_aa, OP_BLOCK: lib.ou_block}
    check(fns[op](ctypes.byref(desc), c_void_p(stream)), f"op {op}")
