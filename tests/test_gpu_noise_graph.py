"""The sampler's noise draws replayed as one captured graph (plan.NoiseDraws)
give the values and the generator state of the eager torch.randn calls, call
after call, for a device generator and the default one."""
import pytest
import torch

from open_universe_amd import plan as P

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("use_default", [False, True])
def test_noise_graph_equals_eager_draws(use_default):
    shape = (2, 1, 3001)
    nz = torch.empty((7,) + shape, device=DEV)
    nd = P.NoiseDraws(nz, shape)
    if use_default:
        torch.cuda.manual_seed(1234)
        rng, ref_rng = None, torch.Generator(device=DEV)
        ref_rng.set_state(torch.cuda.default_generators[0].get_state())
    else:
        rng, ref_rng = torch.Generator(device=DEV).manual_seed(99), torch.Generator(device=DEV).manual_seed(99)
    ref = torch.empty_like(nz)
    for call in range(3):
        nd.draw(rng)
        for k in range(nz.shape[0]):
            torch.randn(shape, generator=ref_rng, out=ref[k])
        assert torch.equal(nz, ref), call
    gen = torch.cuda.default_generators[0] if use_default else rng
    assert torch.equal(gen.get_state(), ref_rng.get_state())
    # the graph path was taken from the second call on (not the eager fallback)
    assert all(g is not None and g is not False for _, g in nd.graphs.values())
    # a later eager draw continues the same sequence
    a = torch.randn(shape, generator=rng, device=DEV) if rng is not None else torch.randn(shape, device=DEV)
    b = torch.randn(shape, generator=ref_rng, device=DEV)
    assert torch.equal(a, b)
