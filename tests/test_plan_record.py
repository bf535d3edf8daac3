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
