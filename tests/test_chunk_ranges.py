"""Host logic of the chunked score pass (Engine.chunk_plan, _enc_ranges,
_dec_ranges, rec_score_chunked), recorded on CPU memory without a GPU: the
chunks' frame ranges cover every level, the middle decoder chunks read only
bottleneck frames both GRU directions have finished, the recorded lanes pass
the runtime's structure check (including its refusal of side-lane wait
cycles), and the chunked program counts the same algorithmic work as the
unchunked one.  Bit-exactness against the unchunked program is
tests/test_gpu_chunked.py."""
import pytest

from open_universe_amd import _lib as L
from open_universe_amd.configs import get_config
from open_universe_amd.engine import Engine, level_lengths
from open_universe_amd.networks.universe import UniverseGAN
from open_universe_amd.plan import EnhancePlan
from open_universe_amd.utils.synthetic import synth_state_dict


@pytest.fixture(scope="module")
def eng():
    cfg = get_config("pp16")
    m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
    sd = synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()])
    return Engine(cfg, sd, "cpu", _record_only=True)


def _covers(ranges, n):
    got = sorted(ranges)
    pos = 0
    for a, b in got:
        if a > pos:
            return False
        pos = max(pos, b)
    return pos >= n


@pytest.mark.parametrize("T", [37011, 64000, 128000, 960000])
def test_chunk_ranges_cover_and_respect_the_recurrence(eng, T):
    Tp = T + 160 - T % 160
    cp = eng.chunk_plan(1, Tp, force=True)
    assert cp is not None
    T4, (s1, s2), h, (m0, m1), D = cp["T4"], cp["s"], cp["h"], cp["mid"], cp["D"]
    Ts = level_lengths(Tp, eng.rates)
    assert 0 < s1 < h < s2 < T4 and T4 - s2 <= m0 < m1 <= s2
    # encoder: owned bottleneck frames partition [0, T4); every level's block
    # output (the decoder's skip) and rate-change output is produced somewhere
    owned = [(0, s1), (s1, h), (h, T4 - s1), (T4 - s1, T4)]
    assert sum(b - a for a, b in owned) == T4
    enc = [eng._enc_ranges(Tp, O) for O in owned]
    n_lvl, nr = len(eng.s_enc), len(eng.rates)
    for i in range(n_lvl):
        Ti = Ts[min(i, nr)]
        assert _covers([r[i]["out"] for r in enc], Ti), i
        for r in enc:
            a, b = r[i]["h"]
            assert 0 <= a < b <= Ti
        if eng.s_enc[i].kind == "down":
            assert _covers([r[i]["e"] for r in enc], Ts[i + 1]), i
            # the level above reads only what this level's chunks produce
            for r in enc:
                ea, eb = r[i]["e"]
                ha, hb = r[i + 1]["h"]
                assert ea <= ha and hb <= eb, (i, r[i]["e"], r[i + 1]["h"])
    # decoder: owned output samples partition [0, T0); the middle chunks
    # (run after GRU segment 2, steps [0, s2) done) read bottleneck frames
    # that both directions have finished: [T4 - s2, s2)
    mid = [(m0 * D, h * D), (h * D, min(Ts[0], m1 * D))]
    outer = [(0, m0 * D), (min(Ts[0], m1 * D), Ts[0])]
    assert sum(b - a for a, b in mid + outer) == Ts[0]
    for P in mid:
        a, b = eng._dec_ranges(Tp, P)[0]["h"]
        assert T4 - s2 <= a and b <= s2
    for P in mid + outer:
        rr = eng._dec_ranges(Tp, P)
        for l, r in enumerate(rr):
            Ti = Ts[min(n_lvl - 1 - l, nr)]
            assert 0 <= r["h"][0] < r["h"][1] <= Ti
            assert r["out"][0] <= P[0] or l < n_lvl - 1


def test_chunked_program_structure_and_accounting(eng):
    T = 64000
    p1 = EnhancePlan(eng, 1, T, 8, 1.3, chunk=True)
    p0 = EnhancePlan(eng, 1, T, 8, 1.3, chunk=False)
    assert p1.chunks is not None and p0.chunks is None
    p1.prog.validate()
    p0.prog.validate()
    # halo recomputation is not algorithmic work: both count the same
    assert sum(p1.prog.flops) == pytest.approx(sum(p0.prog.flops), rel=1e-9)
    assert sum(p1.prog.bytes) == pytest.approx(sum(p0.prog.bytes), rel=1e-9)
    kinds = p1.prog.op_kinds()
    assert kinds.count(L.OP_GRU) == 2 + 3 * 8   # conditioner layers + 3 segments per step
    # the chunk lanes are in use
    lanes = {p1.prog.lib.ou_program_op_kind(p1.prog.h, i) for i in range(len(p1.prog))}
    assert L.OP_LANE in lanes


def test_validate_refuses_side_lane_cycles():
    """Side lanes waiting on each other crash the HIP runtime's stream
    capture: the runtime refuses such a program up front."""
    p = L.Program()
    e0 = p.signal()
    p.lane(1)
    p.wait(e0)
    a = p.signal()
    p.lane(2)
    p.wait(e0)
    p.wait(a)
    b = p.signal()
    p.lane(1)
    p.wait(b)   # 1 -> 2 -> 1
    c = p.signal()
    p.lane(0)
    p.wait(c)
    p.wait(b)
    with pytest.raises(L.OuHipError, match="waits on itself"):
        p.validate()
    q = L.Program()
    e0 = q.signal()
    q.lane(1)
    q.wait(e0)
    a = q.signal()
    q.lane(0)
    q.wait(a)
    q.validate()
