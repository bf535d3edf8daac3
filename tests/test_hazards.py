"""Race and lifetime checks of recorded programs (open_universe_amd/hazards.py),
on the CPU: every pair of ops on different lanes that touch the same bytes
(one writing) must be ordered by the lanes' events, and every byte a
descriptor points at must belong to a tensor the plan keeps alive."""
import gc

import pytest
import torch

from conftest import golden_state_dict, load_golden
from open_universe_amd import _lib as L
from open_universe_amd import hazards as H
from open_universe_amd.configs import get_config
from open_universe_amd.engine import Engine
from open_universe_amd.plan import CondPlan, EnhancePlan, ScorePlan


def test_box_overlap_is_exact():
    # rows 0..3 of 100-byte rows, bytes [0, 40) and [40, 80): interleaved, disjoint
    a = H.Box(1000, 0, 100, 1, 4, 0, 40)
    b = H.Box(1000, 0, 100, 1, 4, 40, 80)
    assert not H.overlap(a, b) and not H.overlap(b, a)
    assert H.overlap(a, H.Box(1000, 0, 100, 1, 4, 39, 41))
    # two batch items of 1000 bytes, the second item's first row
    c = H.Box(1000, 1000, 100, 2, 4, 0, 40)
    assert H.overlap(c, H.Box(2000, 0, 0, 1, 1, 0, 4))
    assert not H.overlap(c, H.Box(1400, 0, 0, 1, 1, 0, 600))   # between item 0's rows and item 1
    assert H.overlap(c, H.Box(1400, 0, 0, 1, 1, 0, 601))


def _memset(p, t):
    p.add(L.OP_MEMSET, L.MemsetArgs(ptr=t.data_ptr(), bytes=t.numel() * 4))


def _scale(p, src, dst):
    p.add(L.OP_SCALE, L.ScaleArgs(z=src.data_ptr(), y=dst.data_ptr(), n=src.numel(), scale=1.0, add=0))


@pytest.mark.parametrize("ordered", [False, True])
def test_unordered_lanes_are_reported(ordered):
    a, b = torch.zeros(256), torch.zeros(256)
    p = L.Program()
    ev0 = p.signal()
    p.lane(1)
    p.wait(ev0)
    _memset(p, a)              # lane 1 writes a
    ev1 = p.signal()
    p.lane(0)
    if ordered:
        p.wait(ev1)
    _scale(p, a, b)            # lane 0 reads a
    if not ordered:
        p.wait(ev1)
    hz = H.find_hazards(p)
    assert (hz == []) == ordered, hz
    if not ordered:
        assert hz[0][2] == "write-read"


def test_dangling_pointer_is_reported():
    keep = torch.zeros(64)
    p = L.Program()
    tmp = torch.zeros(64)
    _scale(p, keep, tmp)
    assert H.dangling(p, keep, tmp) == []
    del tmp
    gc.collect()
    assert [i for i, _, _ in H.dangling(p, keep)] == [0]


@pytest.fixture(scope="module")
def engines():
    out = {}
    for tag, name, nch in (("pp16_c4", "pp16", 4), ("orig16_c4", "orig16", 4), ("pp24_c4", "pp24", 4),
                           ("pp16", "pp16", None)):
        d = load_golden(tag)
        out[tag] = Engine(get_config(name, nch), golden_state_dict(d), "cpu", _record_only=True)
    return out


def _check(plan):
    gc.collect()
    assert H.find_hazards(plan.prog) == []
    assert H.dangling(plan.prog, plan) == []


@pytest.mark.parametrize("tag", ["pp16_c4", "orig16_c4", "pp24_c4", "pp16"])
@pytest.mark.parametrize("B", [1, 2, 3])
def test_enhance_plans_are_race_free(engines, tag, B):
    T = 16000 if tag == "pp16" else 4000
    _check(EnhancePlan(engines[tag], B, T, 8, 1.3))


@pytest.mark.parametrize("opts", [{"keep_rms": True}, {"use_aux_signal": True}, {"warm_start": 3},
                                  {"ensemble": 2, "ensemble_mode": 1}, {"st_lane": False}])
def test_enhance_plan_options_are_race_free(engines, opts):
    B = 2 * opts.get("ensemble", 1)
    _check(EnhancePlan(engines["pp16"], B, 16000, 8, 1.3, **opts))


@pytest.mark.parametrize("env", [{"OUHIP_OVERLAP": "0"}, {"OUHIP_SPLIT_IMAGES": "0"}, {"OUHIP_FIR": "1"},
                                 {"OUHIP_FIR": "0"}])
def test_enhance_plan_schedules_are_race_free(engines, env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    _check(EnhancePlan(engines["pp16_c4"], 2, 4000, 8, 1.3))


def test_network_plans_are_race_free(engines):
    _check(ScorePlan(engines["pp16"], 2, 1600))
    _check(CondPlan(engines["pp16"], 2, 1600))
