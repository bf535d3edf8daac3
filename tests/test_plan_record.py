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


@pytest.mark.parametrize("rates", [None, [4]])
@pytest.mark.parametrize("env", [{}, {"OUHIP_OVERLAP": "0"}])
def test_lane_schedules_validate(monkeypatch, env, rates):
    """The first step's lane schedules (conditioner beside the first score
    pass, mel branch on a lane of its own, st_convs on the score lane; or
    everything in line) record a program whose lane structure
    ou_program_validate accepts (host-only: joins, signal-before-wait, no
    side-lane wait cycles), with the same ops either way.  With one rate
    factor there are no st_convs: the mel branch then stays in line (the
    last st_conv is what joins its lane)."""
    from open_universe_amd.networks.universe import UniverseGAN
    from open_universe_amd.utils.synthetic import synth_state_dict

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cfg = get_config("pp16", 4)
    if rates is None:
        sd = golden_state_dict(load_golden("pp16_c4"))
    else:
        cfg["score_model"]["rate_factors"] = cfg["condition_model"]["rate_factors"] = rates
        m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
        sd = synth_state_dict([(k, v.shape) for k, v in m.state_dict().items() if not k.startswith("loss_")])
    eng = Engine(cfg, sd, "cpu", _record_only=True)
    plan = EnhancePlan(eng, 1, 3000, 8, 1.3)
    plan.prog.validate()
    kinds = [k for k in plan.prog.op_kinds() if k not in (L.OP_LANE, L.OP_SIGNAL, L.OP_WAIT)]
    for k in env:
        monkeypatch.delenv(k)
    ref = EnhancePlan(eng, 1, 3000, 8, 1.3)
    ref.prog.validate()
    # the same ops (in line, the conditioner's ops come in another order)
    assert sorted(kinds) == sorted(k for k in ref.prog.op_kinds() if k not in (L.OP_LANE, L.OP_SIGNAL, L.OP_WAIT))


def test_split_images_link_the_deep_level_convs():
    """Full-width PP16 (256 / 512-channel levels): every conv whose input a
    conv or fused block wrote last reads that producer's split image
    (ou_conv_desc.xs; on any lane: the program orders the consumer after its
    producer), the producer's descriptor is patched to store it (sy), and one
    image per activation buffer serves all diffusion steps."""
    from open_universe_amd.hazards import happens_before

    d = load_golden("pp16")
    eng = Engine(get_config("pp16"), golden_state_dict(d), "cpu", _record_only=True)
    plan = EnhancePlan(eng, 1, 16000, 8, 1.3)
    links = plan.prog.split_links
    steps = len(links) // 8
    assert steps >= 12, len(links)            # per score step: the 256 / 512-channel chains
    assert len(plan.prog.split_bufs) <= 40    # images shared across the steps
    hb = happens_before(plan.prog)
    for prod, cons in links:
        lane, k, _ = hb[prod]
        assert prod < cons and hb[cons][2].get(lane, 0) >= k   # the consumer runs after its producer


def test_split_images_off_records_plain_convs(monkeypatch):
    monkeypatch.setenv("OUHIP_SPLIT_IMAGES", "0")
    d = load_golden("pp16")
    eng = Engine(get_config("pp16"), golden_state_dict(d), "cpu", _record_only=True)
    plan = EnhancePlan(eng, 1, 16000, 8, 1.3)
    assert not getattr(plan.prog, "split_links", [])
