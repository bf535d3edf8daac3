"""Race check of a recorded program's lanes (host only, no GPU).

A program's lanes run concurrently: side streams in an eager replay,
parallel branches of the captured hipGraph.  Two ops on different lanes are
ordered only through SIGNAL / WAIT events; everything else may overlap in
time.  ``find_hazards`` computes that happens-before order with vector
clocks over the recorded op list and reports every pair of ops that is NOT
ordered although one writes memory the other reads or writes -- the class of
bug that shows up only when a replay's timing changes (a first replay, a
busier box) and otherwise hides, because the later replays of a deterministic
program read the previous replay's identical values.

Each op's footprint is derived from its descriptor (include/ouhip.h) as
strided boxes: base + item * bstride + row * cstride + [t0, t1) bytes.  Two
boxes overlap iff some (item, row, byte) of one equals one of the other,
which is decided exactly per item offset (no layout assumptions).  Weights,
biases and other recorded constants are never written during a replay and
are left out.  Every plan schedule the package records is checked
(tests/test_hazards.py)."""
from dataclasses import dataclass

from . import _lib as L


@dataclass(frozen=True)
class Box:
    base: int       # byte address of item 0, row 0, byte 0
    bs: int         # bytes between items
    cs: int         # bytes between rows
    nb: int         # items
    nc: int         # rows per item
    t0: int         # byte range [t0, t1) inside a row
    t1: int

    @property
    def lo(self):
        return self.base + self.t0

    @property
    def hi(self):   # one past the last byte
        return self.base + (self.nb - 1) * self.bs + (self.nc - 1) * self.cs + self.t1


def _box(ptr, bs, cs, nb, nc, t0, t1):
    ptr = ptr or 0
    if not ptr or nb <= 0 or nc <= 0 or t1 <= t0:
        return None
    return Box(int(ptr), int(bs), int(cs), int(nb), int(nc), int(t0), int(t1))


def _span(ptr, nbytes):
    return _box(ptr, 0, 0, 1, 1, 0, nbytes)


def overlap(a: Box, b: Box) -> bool:
    """Exact: is there (ia, ca, ta) of a and (ib, cb, tb) of b with
    a.base + ia a.bs + ca a.cs + ta == b.base + ib b.bs + cb b.cs + tb?
    (Row by row of the box with fewer rows against the other's items.)"""
    if a.hi <= b.lo or b.hi <= a.lo:
        return False
    if a.nb * a.nc > b.nb * b.nc:
        a, b = b, a
    if a.nb * a.nc > 1 << 16:
        return True   # not worth the time: call it a hit
    n = a.t1 - a.t0
    for ia in range(a.nb):
        for ca in range(a.nc):
            s0 = a.base + ia * a.bs + ca * a.cs + a.t0
            if _span_hits(s0, s0 + n, b):
                return True
    return False


def _span_hits(s0, s1, b: Box) -> bool:
    """Does the byte range [s0, s1) meet box b?"""
    if s1 <= b.lo or b.hi <= s0:
        return False
    for ib in range(b.nb):
        base = b.base + ib * b.bs
        if b.nc == 1 or b.cs == 0:
            if s0 < base + b.t1 and base + b.t0 < s1:
                return True
            continue
        # rows c with [base + c cs + t0, base + c cs + t1) meeting [s0, s1)
        c_lo = max(0, -(-(s0 - base - b.t1 + 1) // b.cs))
        c_hi = min(b.nc - 1, (s1 - 1 - base - b.t0) // b.cs)
        if c_lo <= c_hi:
            return True
    return False


def _conv(d):
    R, W = [], []
    cout = d.m // abs(d.rout)
    R.append(_box(d.x, 4 * d.x_bstride, 4 * d.x_cstride, d.batch, d.cin, 0, 4 * d.in_len))
    R.append(_span(d.in_scale, 4 * d.batch))
    r = abs(d.rout)
    a = d.f0 * r
    b = min((d.f0 + d.n_frames) * r, d.out_len)
    for p, bs, cs in ((d.res1, d.r1_bstride, d.r1_cstride), (d.res2, d.r2_bstride, d.r2_cstride)):
        R.append(_box(p, 4 * bs, 4 * cs, d.batch, cout, 4 * a, 4 * b))
    R.append(_span(d.film, 4 * ((d.batch - 1) * d.film_bstride + 2 * cout)))
    W.append(_box(d.y, 4 * d.y_bstride, 4 * d.y_cstride, d.batch, cout, 4 * a, 4 * b))
    if d.xs:
        R.append(_box(d.xs, d.xs_bstride, 0, d.batch, 1, 0, (d.cin // 32) * d.xs_rows * 128))
    if d.sy:
        W.append(_box(d.sy, d.sy_bstride, 0, d.batch, 1, 0, (d.m // 32) * d.sy_rows * 128))
    if d.tile >= 0 and (d.tile >> 12) & 3 and not d.tile & (1 << 15):
        W.append(_span(d.ks_ws, d.ks_ws_bytes))   # K-slice partial sums
    return R, W


def _block(d):
    R, W = [], []
    C, T = d.channels, d.length
    f0, f1 = d.f0, d.f1 or T
    h0, h1 = d.h0, d.h1 or T
    if d.x:
        R.append(_box(d.x, 4 * d.x_bstride, 0, d.batch, 1, 0, 4 * T))
        R.append(_span(d.in_scale, 4 * d.batch))
    else:
        R.append(_box(d.h, 4 * d.h_bstride, 4 * d.h_cstride, d.batch, C, 4 * max(0, h0), 4 * min(T, h1)))
    lo, hi = max(0, f0 - 8), min(T, f1 + 8)   # conv1's halo (k5) and the stages behind it
    R.append(_box(d.sc, 4 * d.sc_bstride, 4 * d.sc_cstride, d.batch, C, 4 * lo, 4 * hi))
    R.append(_span(d.film, 4 * ((d.batch - 1) * d.film_bstride + 2 * C)))
    R.append(_box(d.res2, 4 * d.r2_bstride, 4 * d.r2_cstride, d.batch, C, 4 * f0, 4 * f1))
    if d.xs:
        R.append(_box(d.xs, d.xs_bstride, 0, d.batch, 1, 0, (C // 32) * d.xs_rows * 128))
    W.append(_box(d.cond_out, 4 * d.co_bstride, 4 * d.co_cstride, d.batch, C, 4 * f0, 4 * f1))
    if d.head.w:
        hd = d.head
        for p in (hd.x, hd.z):
            R.append(_box(p, 4 * T, 0, d.batch, 1, 4 * f0, 4 * f1))
        W.append(_box(hd.out, 4 * T, 0, d.batch, 1, 4 * f0, 4 * f1))
    else:
        W.append(_box(d.y, 4 * d.y_bstride, 4 * d.y_cstride, d.batch, C, 4 * f0, 4 * f1))
    if d.e:
        r = max(1, d.rate)
        W.append(_box(d.e, 4 * d.e_bstride, 4 * d.e_cstride, d.batch, 2 * C, 4 * (f0 // r), 4 * (-(-f1 // r))))
    if d.sy:
        W.append(_box(d.sy, d.sy_bstride, 0, d.batch, 1, 0, (C // 32) * d.sy_rows * 128))
    return R, W


def _gru(d, lib):
    H, T = d.hidden, d.steps
    R = [_box(d.gi, 4 * d.gi_bstride, 0, d.batch, 1, 0, 4 * 6 * H * T),
         _box(d.res, 4 * d.res_bstride, 4 * d.res_cstride, d.batch, 2 * H, 0, 4 * T)]
    W = [_box(d.y, 4 * d.y_bstride, 4 * d.y_cstride, d.batch, 2 * H, 0, 4 * T),
         _span(d.granules, lib.ou_gru_workspace_bytes(H, d.batch)),
         _span(d.hstate, 4 * d.batch * 2 * H)]
    return R, W


def footprint(op, d, lib=None):
    """(reads, writes): lists of Box for one recorded op."""
    lib = lib or L.load()
    if op == L.OP_CONV:
        R, W = _conv(d)
    elif op == L.OP_BLOCK:
        R, W = _block(d)
    elif op == L.OP_GRU:
        R, W = _gru(d, lib)
    elif op == L.OP_HEAD:
        R = [_box(d.h, 4 * d.h_bstride, 0, d.batch, 1, 0, 4 * d.channels * d.length),
             _box(d.x, 4 * d.length, 0, d.batch, 1, 0, 4 * d.length),
             _box(d.z, 4 * d.length, 0, d.batch, 1, 0, 4 * d.length)]
        W = [_box(d.out, 4 * d.length, 0, d.batch, 1, 0, 4 * d.length)]
    elif op == L.OP_EMBED:
        R = [_span(d.sigma, 4 * d.n)]
        W = [_span(d.out, 4 * d.n * d.rows), _span(d.gbuf, 4 * d.n * d.dim)]
    elif op == L.OP_MEMSET:
        R, W = [], [_span(d.ptr, d.bytes)]
    elif op == L.OP_NORMALIZE:
        R, W = [_span(d.x, 4 * d.batch * d.n)], [_span(d.y, 4 * d.batch * d.n)]
    elif op in (L.OP_RMS, L.OP_INV_RMS):
        R, W = [_span(d.x, 4 * d.batch * d.n)], [_span(d.out, 4 * d.batch)]
    elif op == L.OP_POWER:
        R = [_span(d.x, 4 * d.batch * 2 * d.nf * d.frames)]
        W = [_span(d.y, 4 * d.batch * d.nf * d.frames)]
    elif op == L.OP_PAD:
        R = [_box(d.x, 4 * d.x_bstride, 0, d.batch, 1, 0, 4 * d.n_in)]
        W = [_span(d.y, 4 * d.batch * d.n_out)]
    elif op == L.OP_SCALE:
        R, W = [_span(d.z, 4 * d.n), _span(d.add, 4 * d.n)], [_span(d.y, 4 * d.n)]
    elif op == L.OP_FINISH:
        R = [_box(d.x, 4 * d.x_bstride, 0, d.batch, 1, 0, 4 * (d.left + d.len)), _span(d.mix_rms, 4 * d.batch)]
        W = [_span(d.y, 4 * d.batch * d.len)]
    elif op == L.OP_ENSEMBLE:
        R = [_span(d.x, 4 * d.ensemble * d.n)]
        W = [_span(d.y, 4 * d.n), _span(d.counts, 4 * 32 * max(1, d.batch))]
    elif op == L.OP_SNAKE:
        R = [_box(d.h, 4 * d.h_bstride, 0, d.batch, 1, 0, 4 * d.channels * d.length)]
        W = [_span(d.out, 4 * d.batch * d.channels * d.length)]
    else:
        R, W = [], []
    return [b for b in R if b is not None], [b for b in W if b is not None]


def happens_before(prog):
    """Per op: (lane, its index on the lane, vector clock) -- op j is
    ordered after op i (on lane a, index k) iff clock_j[a] >= k."""
    clocks = {}     # lane -> vector clock (dict lane -> count)
    events = {}
    lane = 0
    out = []
    for op, d in zip(prog.op_kinds(), prog.descs):
        if op == L.OP_LANE:
            lane = d.id
            out.append(None)
            continue
        vc = clocks.setdefault(lane, {})
        if op == L.OP_SIGNAL:
            events[d.id] = dict(vc)
            out.append(None)
            continue
        if op == L.OP_WAIT:
            for k, v in events[d.id].items():
                if vc.get(k, 0) < v:
                    vc[k] = v
            out.append(None)
            continue
        vc[lane] = vc.get(lane, 0) + 1
        out.append((lane, vc[lane], dict(vc)))
    return out


def find_hazards(prog, limit=20):
    """Unordered pairs of ops on different lanes with a write-read or
    write-write overlap: [(i, j, kind, label_i, label_j)], at most ``limit``."""
    lib = L.load()
    hb = happens_before(prog)
    kinds = prog.op_kinds()
    fps = {}
    for i, (op, d) in enumerate(zip(kinds, prog.descs)):
        if hb[i] is not None:
            fps[i] = footprint(op, d, lib)
    found = []
    idx = sorted(fps)
    for jj, j in enumerate(idx):
        lane_j, _, vc_j = hb[j]
        Rj, Wj = fps[j]
        if not Rj and not Wj:
            continue
        for i in idx[:jj]:
            lane_i, k_i, _ = hb[i]
            if lane_i == lane_j or vc_j.get(lane_i, 0) >= k_i:
                continue   # same lane (stream order) or ordered by events
            Ri, Wi = fps[i]
            kind = None
            if any(overlap(a, b) for a in Wi for b in Wj):
                kind = "write-write"
            elif any(overlap(a, b) for a in Wi for b in Rj):
                kind = "write-read"
            elif any(overlap(a, b) for a in Ri for b in Wj):
                kind = "read-write"
            if kind:
                found.append((i, j, kind, prog.labels[i], prog.labels[j]))
                if len(found) >= limit:
                    return found
    return found


def live_ranges(*roots):
    """Byte ranges of the storages of every torch tensor reachable from
    ``roots`` (attributes, dicts, lists, tuples; Act views through .t)."""
    import torch

    seen, out, stack = set(), [], list(roots)
    while stack:
        o = stack.pop()
        if id(o) in seen or o is None or isinstance(o, (int, float, str, bytes, bool)):
            continue
        seen.add(id(o))
        if isinstance(o, torch.Tensor):
            st = o.untyped_storage()
            if st.nbytes():
                out.append((st.data_ptr(), st.data_ptr() + st.nbytes()))
            continue
        if isinstance(o, dict):
            stack.extend(o.values())
        elif isinstance(o, (list, tuple, set)):
            stack.extend(o)
        elif hasattr(o, "__dict__") and not isinstance(o, type):
            stack.extend(vars(o).values())
    out.sort()
    return out


def dangling(prog, *roots, limit=20):
    """Ops whose footprint reaches memory no tensor reachable from ``roots``
    owns: the program would read or write freed memory (the caching allocator
    hands it to the next tensor).  [(op index, label, Box)], at most ``limit``."""
    import bisect

    lib = L.load()
    live = live_ranges(prog, *roots)
    starts = [a for a, _ in live]
    bad = []
    for i, (op, d) in enumerate(zip(prog.op_kinds(), prog.descs)):
        if op in (L.OP_LANE, L.OP_SIGNAL, L.OP_WAIT):
            continue
        R, W = footprint(op, d, lib)
        for b in R + W:
            k = bisect.bisect_right(starts, b.lo) - 1
            if k < 0 or not any(live[j][0] <= b.lo and b.hi <= live[j][1] for j in range(max(0, k - 4), k + 1)):
                bad.append((i, prog.labels[i], b))
                break
        if len(bad) >= limit:
            break
    return bad
