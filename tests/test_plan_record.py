"""Record (never launch) the full enhance program on CPU memory: exercises the
host-side layer walk, buffer shapes and descriptor validation without a GPU."""
import pytest
import torch

from conftest import golden_state_dict, load_golden
from open_universe_amd import _lib as L
from open_universe_amd.configs import get_config
from open_universe_amd.engine import Engine
from open_universe_amd.plan import CondPlan, EnhancePlan, ScorePlan


@pytest.mark.parametrize("tag,name,nch", [("pp16_c4", "pp16", 4), ("orig16_c4", "orig16", 4),
                                          ("pp24_c4", "pp24", 4)])
@pytest.mark.parametrize("opts", [{}, {"keep_rms": True}, {"use_aux_signal": True},
                                  {"warm_start": 3}])
def test_record_enhance_program(tag, name, nch, opts):
    if name == "orig16" and opts.get("use_aux_signal") or name == "orig16" and "warm_start" in opts:
        pytest.skip("UNIVERSE has no signal-decoupling layer")
    d = load_golden(tag)
    sd = golden_state_dict(d)
    eng = Engine(get_config(name, nch), sd, "cpu", _record_only=True)
    plan = EnhancePlan(eng, 2, 3000, 8, 1.3, **opts)
    n = len(plan.prog)
    assert n > 50
    # every conv descriptor satisfies the kernel's preconditions
    sp = ScorePlan(eng, 1, 800)
    cp = CondPlan(eng, 1, 800)
    assert len(sp.prog) > 30 and len(cp.prog) > 30


def test_arena_carves_aligned_views_and_reports_overflow():
    from open_universe_amd import engine as E

    ar = E.Arena("cpu", 4096)
    a = ar.take((3, 5), torch.float32)
    b = ar.take((7,), torch.int64)
    assert a.shape == (3, 5) and b.shape == (7,)
    base = ar.buf.data_ptr()   # device allocations are 256-B aligned; offsets keep that
    assert (a.data_ptr() - base) % 256 == 0 and (b.data_ptr() - base) % 256 == 0
    assert b.data_ptr() >= a.data_ptr() + 60
    with pytest.raises(E.ArenaFull):
        ar.take((1024,), torch.float32)
    ar.off = 0   # the next plan of the slot starts over at offset 0
    assert ar.take((3, 5), torch.float32).data_ptr() == a.data_ptr()


def test_enhance_plan_records_onto_an_arena():
    """All EnhancePlan buffers come from the arena when one is given; a too
    small arena raises ArenaFull (the model then retries with a bigger one)."""
    from open_universe_amd import engine as E

    d = load_golden("pp16_c4")
    eng = Engine(get_config("pp16", 4), golden_state_dict(d), "cpu", _record_only=True)
    with pytest.raises(E.ArenaFull):
        EnhancePlan(eng, 1, 3000, 8, 1.3, arena=E.Arena("cpu", 1 << 16))
    assert E._ARENA is None
    ar = E.Arena("cpu", 64 << 20)
    plan = EnhancePlan(eng, 1, 3000, 8, 1.3, arena=ar)
    lo, hi = ar.buf.data_ptr(), ar.buf.data_ptr() + ar.nbytes
    for t in (plan.MIX, plan.NZ, plan.OUT, plan.X.t, plan.sb["E0"].t, plan.cb["SPEC"].t):
        assert lo <= t.data_ptr() < hi


@pytest.mark.parametrize("env", [{}, {"OUHIP_MEL_LANE": "2"}, {"OUHIP_MEL_LANE": "0"},
                                 {"OUHIP_SCORE_AFTER_CENC": "1"},
                                 {"OUHIP_MEL_LANE": "2", "OUHIP_SCORE_AFTER_CENC": "1"}])
def test_lane_schedule_variants_validate(monkeypatch, env):
    """Every lane schedule of the first step (mel branch in line, on the st
    lane or a lane of its own; the score pass started after the
    conditioner's encoder) records a program whose lane structure
    ou_program_validate accepts (host-only: joins, signal-before-wait, no
    side-lane wait cycles), with the same ops as the default schedule."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    d = load_golden("pp16_c4")
    eng = Engine(get_config("pp16", 4), golden_state_dict(d), "cpu", _record_only=True)
    plan = EnhancePlan(eng, 1, 3000, 8, 1.3)
    plan.prog.validate()
    kinds = [k for k in plan.prog.op_kinds() if k not in (L.OP_LANE, L.OP_SIGNAL, L.OP_WAIT)]
    for k in env:
        monkeypatch.delenv(k)
    ref = EnhancePlan(eng, 1, 3000, 8, 1.3)
    assert kinds == [k for k in ref.prog.op_kinds() if k not in (L.OP_LANE, L.OP_SIGNAL, L.OP_WAIT)]
