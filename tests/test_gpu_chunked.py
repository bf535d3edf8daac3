"""The chunked score pass (Engine.chunk_plan / rec_score_chunked) against the
unchunked one: the convs run in frame chunks on two side lanes around the
bottleneck GRU's step segments, recomputing halo frames with the tiles of the
whole ops, so the whole enhance() must agree BIT FOR BIT with the unchunked
program on the same noise (the unchunked program is itself pinned to the
oracle / reference in test_gpu_parity*.py).  Lengths cover the C2 clip, a
ragged one, a long-form one and the split points' edges; both operand
precisions the chunked pass runs (split-f16, f16)."""
import pytest
import torch

from open_universe_amd.configs import get_config
from open_universe_amd.networks.universe import UniverseGAN
from open_universe_amd.plan import EnhancePlan
from open_universe_amd.utils.synthetic import synth_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _model(prec):
    cfg = get_config("pp16")
    m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()]), strict=False)
    m = m.to(DEV).eval()
    m._conv_prec = prec
    return m


@pytest.fixture(scope="module", params=[1, 2], ids=["split16", "f16"])
def model(request):
    return _model(request.param)


def _pair(eng, B, T, split=None, monkeypatch=None, **kw):
    """A chunked plan and the unchunked one it must equal bit for bit.  The
    chunked pass records no split-image links (its chunks keep the whole ops'
    tiles), so the unchunked plan is recorded without them too."""
    import os

    if split is not None:
        monkeypatch.setenv("OUHIP_CHUNK_SPLIT", split)
    p1 = EnhancePlan(eng, B, T, 8, 1.3, chunk=True, **kw)
    saved = os.environ.get("OUHIP_SPLIT_IMAGES")
    os.environ["OUHIP_SPLIT_IMAGES"] = "0"
    try:
        p0 = EnhancePlan(eng, B, T, 8, 1.3, chunk=False, **kw)
    finally:
        if saved is None:
            del os.environ["OUHIP_SPLIT_IMAGES"]
        else:
            os.environ["OUHIP_SPLIT_IMAGES"] = saved
    return p0, p1


@pytest.mark.parametrize("B,T", [(1, 128000), (1, 37011), (2, 50000), (1, 960000)])
def test_chunked_enhance_bit_exact(model, B, T):
    eng = model._get_engine()
    p0, p1 = _pair(eng, B, T)
    assert p1.chunks is not None and p0.chunks is None
    g = torch.Generator().manual_seed(T)
    mix = (0.1 * torch.randn(B, 1, T, generator=g)).to(DEV)
    a = p0(mix, torch.Generator(device=DEV).manual_seed(7)).clone()
    b = p1(mix, torch.Generator(device=DEV).manual_seed(7)).clone()   # first replay: eager lanes
    assert torch.isfinite(b).all()
    assert torch.equal(a, b), (a - b).abs().max().item()
    # the second replay captures the hipGraph (lanes = parallel branches)
    c = p1(mix, torch.Generator(device=DEV).manual_seed(7)).clone()
    assert p1.prog.captured
    assert torch.equal(b, c)


@pytest.mark.parametrize("split", ["0.05,0.6", "0.45,0.95", "0.3,0.55"])
def test_chunked_split_points(split, monkeypatch):
    """Extreme segment splits (tiny first segment, a middle that barely
    covers, a late middle) stay bit-exact."""
    m = _model(1)
    eng = m._get_engine()
    T = 64000
    p0, p1 = _pair(eng, 1, T, split, monkeypatch)
    assert p1.chunks is not None
    mix = (0.1 * torch.randn(1, 1, T, generator=torch.Generator().manual_seed(1))).to(DEV)
    a = p0(mix, torch.Generator(device=DEV).manual_seed(3)).clone()
    b = p1(mix, torch.Generator(device=DEV).manual_seed(3)).clone()
    c = p1(mix, torch.Generator(device=DEV).manual_seed(3)).clone()
    assert torch.equal(a, b) and torch.equal(a, c)


def test_chunked_keep_rms_and_model_enhance(model, monkeypatch):
    """enhance() itself takes the chunked pass at batch 1 with OUHIP_CHUNK=1
    (keep_rms too)."""
    monkeypatch.setenv("OUHIP_CHUNK", "1")
    T = 48000
    mix = (0.1 * torch.randn(T, generator=torch.Generator().manual_seed(2))).to(DEV)
    with torch.no_grad():
        out = model.enhance(mix, rng=torch.Generator(device=DEV).manual_seed(4), keep_rms=True)
    plan = next(p for k, p in model._plans.items() if k[1] == T)
    assert plan.chunks is not None
    monkeypatch.setenv("OUHIP_SPLIT_IMAGES", "0")   # as the chunked plan: no split-image links
    p0 = EnhancePlan(model._get_engine(), 1, T, 8, 1.3, keep_rms=True, chunk=False)
    ref = p0(mix[None, None], torch.Generator(device=DEV).manual_seed(4)).clone()
    assert torch.equal(out, ref[0])


def test_short_clips_are_not_chunked(model, monkeypatch):
    eng = model._get_engine()
    assert eng.chunk_plan(1, 128160) is None   # off by default
    monkeypatch.setenv("OUHIP_CHUNK", "1")
    assert eng.chunk_plan(1, 128160) is not None
    assert eng.chunk_plan(1, 160 * 60) is None   # T4 = 60: too few GRU steps to split
    assert eng.chunk_plan(8, 128160) is None     # wide batches fill the chip without it


@pytest.mark.parametrize("chunk", [False, True], ids=["lanes", "chunked"])
def test_segment_capture_equals_whole_graph(chunk, monkeypatch):
    """ou_program_capture_segments (one hipGraph per run of kernels on a
    lane, lanes on real streams) replays the same program bit for bit."""
    m = _model(1)
    eng = m._get_engine()
    T = 64000
    mix = (0.1 * torch.randn(1, 1, T, generator=torch.Generator().manual_seed(5))).to(DEV)
    p = EnhancePlan(eng, 1, T, 8, 1.3, chunk=chunk)
    a = p(mix, torch.Generator(device=DEV).manual_seed(9), use_graph=False).clone()
    p.prog.capture(segments=True)
    b = p(mix, torch.Generator(device=DEV).manual_seed(9)).clone()
    c = p(mix, torch.Generator(device=DEV).manual_seed(9)).clone()
    assert torch.equal(a, b) and torch.equal(a, c)
