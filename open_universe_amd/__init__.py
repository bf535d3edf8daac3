"""open_universe_amd -- MI355X-native (gfx950) implementation of open-universe's
``inference_utils.load_model()`` -> ``model.enhance()`` hot path.

    from open_universe_amd import inference_utils
    model = inference_utils.load_model("weights.ckpt", device="cuda:0")
    enhanced = model.enhance(noisy_16k)

The compute runs in hand-written HIP kernels (libouhip.so, C ABI in
include/ouhip.h); PyTorch provides device memory, streams and the RNG.
"""
from . import inference_utils  # noqa: F401

__version__ = "0.1.0"
