"""Small-batch enhance as two score sub-batches on two lanes
(engine.score_sub_batches, plan.EnhancePlan): one half's bottleneck GRU runs
beside the other half's convolutions.  Each item's arithmetic is the whole
batch's -- the sub-batches run the whole batch's tiles (ConvTuner keys on the
plan's batch) -- so the result must equal the unsplit plan BIT FOR BIT on the
same noise (which is itself pinned to the oracle in test_gpu_parity*.py)."""
import pytest
import torch

from open_universe_amd.configs import get_config
from open_universe_amd.networks.universe import UniverseGAN
from open_universe_amd.plan import EnhancePlan
from open_universe_amd.utils.synthetic import synth_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", params=[1, 2], ids=["split16", "f16"])
def model(request):
    cfg = get_config("pp16")
    m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()]), strict=False)
    m = m.to(DEV).eval()
    m._conv_prec = request.param
    return m


@pytest.mark.parametrize("B,T", [(4, 64000), (3, 37011), (2, 128000)])
def test_sub_batched_enhance_bit_exact(model, B, T, monkeypatch):
    eng = model._get_engine()
    monkeypatch.setenv("OUHIP_SUB_BATCH", "1")
    p1 = EnhancePlan(eng, B, T, 8, 1.3)
    monkeypatch.setenv("OUHIP_SUB_BATCH", "0")
    p0 = EnhancePlan(eng, B, T, 8, 1.3)
    assert p1.subs is not None and p0.subs is None
    g = torch.Generator().manual_seed(T)
    mix = (0.1 * torch.randn(B, 1, T, generator=g)).to(DEV)
    a = p0(mix, torch.Generator(device=DEV).manual_seed(7)).clone()
    b = p1(mix, torch.Generator(device=DEV).manual_seed(7)).clone()   # first replay: eager lanes
    assert torch.isfinite(b).all()
    assert torch.equal(a, b), (a - b).abs().max().item()
    c = p1(mix, torch.Generator(device=DEV).manual_seed(7)).clone()   # captured hipGraph
    assert p1.prog.captured
    assert torch.equal(b, c)


def test_sub_batched_model_enhance(model, monkeypatch):
    """Universe.enhance at B = 4 with OUHIP_SUB_BATCH=1 records the sub-batched plan."""
    monkeypatch.setenv("OUHIP_SUB_BATCH", "1")
    model._plans.clear()
    mix = 0.1 * torch.randn(4, 32000, generator=torch.Generator().manual_seed(3)).to(DEV)
    y = model.enhance(mix, rng=torch.Generator(device=DEV).manual_seed(1))
    assert y.shape == mix.shape and torch.isfinite(y).all()
    plan = next(reversed(model._plans.values()))
    assert plan.subs == [(0, 2), (2, 4)]
