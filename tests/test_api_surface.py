"""Drop-in surface (CPU): parameter tree / EMA order match the reference, the
checkpoint loader reads the reference's layout, the CLI argument builder works."""
import argparse
import os
import typing

import numpy as np
import pytest
import torch
import yaml

from conftest import load_golden
from open_universe_amd.configs import get_config
from open_universe_amd.inference_utils import add_enhance_arguments, load_model
from open_universe_amd.networks.universe import Universe, UniverseGAN
from open_universe_amd.utils.synthetic import synth_state_dict


def _build(name, nch=None):
    cfg = get_config(name, nch)
    cls = UniverseGAN if cfg["_target_"].endswith("UniverseGAN") else Universe
    return cls(**{k: v for k, v in cfg.items() if k != "_target_"})


@pytest.mark.parametrize("tag,name,nch", [("pp16", "pp16", None), ("pp16_c4", "pp16", 4),
                                          ("orig16_c4", "orig16", 4), ("pp24_c4", "pp24", 4),
                                          ("pp24_manifest", "pp24", None),
                                          ("orig16_manifest", "orig16", None)])
def test_state_dict_and_ema_order_match_reference(tag, name, nch):
    d = load_golden(tag)
    ref_names = [n for n in d["manifest_names"] if not n.startswith("loss_")]
    ref_shapes = [s for n, s in zip(d["manifest_names"], d["manifest_shapes"]) if not n.startswith("loss_")]
    m = _build(name, nch)
    sd = m.state_dict()
    assert list(sd.keys()) == list(ref_names)
    for n, s in zip(ref_names, ref_shapes):
        assert ",".join(map(str, sd[n].shape)) == s, n
    pid = {id(p): n for n, p in m.named_parameters()}
    assert [pid[id(p)] for p in m.model_parameters()] == list(d["param_order"])


def test_enhance_signature_is_the_reference_one():
    hints = typing.get_type_hints(UniverseGAN.enhance)
    assert hints == {
        "n_steps": typing.Optional[int], "epsilon": typing.Optional[float],
        "target": typing.Optional[torch.Tensor], "fake_score_snr": typing.Optional[float],
        "rng": typing.Optional[torch.Generator], "use_aux_signal": typing.Optional[bool],
        "keep_rms": typing.Optional[bool], "ensemble": typing.Optional[int],
        "ensemble_stat": typing.Optional[str], "warm_start": typing.Optional[int],
        "return": torch.Tensor}


def _write_ckpt(tmp, with_ema):
    m = _build("pp16", 4)
    spec = [(k, v.shape) for k, v in m.state_dict().items()]
    sd = synth_state_dict(spec, seed=3)
    full = m.state_dict()
    full.update(sd)
    full["loss_mpd.discriminators.0.convs.0.weight"] = torch.zeros(3)  # training-only key
    data = {"state_dict": full}
    ema_vals = None
    if with_ema:
        params = list(m.model_parameters())
        ema_vals = [torch.randn(p.shape) for p in params]
        data["ema"] = {"decay": 0.999, "num_updates": 10, "shadow_params": ema_vals,
                       "collected_params": None}
    run = os.path.join(tmp, "exp", "checkpoints")
    os.makedirs(run)
    os.makedirs(os.path.join(tmp, "exp", ".hydra"))
    torch.save(data, os.path.join(run, "last.ckpt"))
    cfg = get_config("pp16", 4)
    cfg["condition_model"]["n_channels"] = "${model.score_model.n_channels}"
    cfg["condition_model"]["rate_factors"] = "${model.score_model.rate_factors}"
    cfg["training"] = {"audio_len": "${datamodule.datasets.vb-train-16k.audio_len}", "ema_decay": 0.999}
    with open(os.path.join(tmp, "exp", ".hydra", "config.yaml"), "w") as f:
        yaml.safe_dump({"model": cfg}, f)
    return os.path.join(run, "last.ckpt"), m, sd, ema_vals


@pytest.mark.parametrize("with_ema", [False, True])
def test_load_model_reads_reference_checkpoint_layout(tmp_path, with_ema):
    path, m, sd, ema = _write_ckpt(str(tmp_path), with_ema)
    model, cfg = load_model(path, device=None, return_config=True)
    assert isinstance(model, UniverseGAN)
    assert model.fs == 16000 and model.diff_kwargs.get("n_steps") == 8
    assert cfg["model"]["condition_model"]["n_channels"] == 4
    got = model.state_dict()
    if with_ema:
        for p, e in zip(model.model_parameters(), ema):
            torch.testing.assert_close(p.detach(), e)
    else:
        for k, v in sd.items():
            torch.testing.assert_close(got[k], v.to(got[k].dtype))


def test_add_enhance_arguments(tmp_path):
    path, *_ = _write_ckpt(str(tmp_path), False)
    model = load_model(path)
    parser = argparse.ArgumentParser()
    add_enhance_arguments(model, parser)
    args = parser.parse_args(["--n_steps", "4", "--epsilon", "1.1"])
    assert args.n_steps == 4 and args.epsilon == 1.1 and args.keep_rms is None
    args = parser.parse_args([])
    assert args.n_steps == 8 and args.epsilon == 1.3


_LIGHTNING_SAVER = r'''
import sys, types, typing, torch
# stand-ins shaped like omegaconf's pickled objects (the real package is absent)
dc = types.ModuleType("omegaconf.dictconfig"); nodes = types.ModuleType("omegaconf.nodes")
base = types.ModuleType("omegaconf.base")
sys.modules["omegaconf"] = types.ModuleType("omegaconf")
class ContainerMetadata:
    def __init__(self): self.ref_type = typing.Any; self.object_type = dict; self.key_type = typing.Any
class DictConfig:
    def __init__(self, content): self._metadata = ContainerMetadata(); self._parent = None; self._content = content
    def __getstate__(self): return {"_metadata": self._metadata, "_parent": self._parent, "_content": self._content}
class AnyNode:
    def __init__(self, v): self._val = v; self._metadata = ContainerMetadata()
for cls, mod in ((DictConfig, dc), (AnyNode, nodes), (ContainerMetadata, base)):
    cls.__module__ = mod.__name__; setattr(mod, cls.__name__, cls); sys.modules[mod.__name__] = mod
data = torch.load(sys.argv[1], weights_only=True)
data["hyper_parameters"] = {"fs": 16000, "score_model": DictConfig({"n_channels": AnyNode(4)})}
data["optimizer_states"] = [{"state": {}, "param_groups": [{"lr": 1e-4}]}]
data["callbacks"] = {"ModelCheckpoint": {"best_model_path": "x.ckpt"}}
data["epoch"], data["global_step"], data["pytorch-lightning_version"] = 3, 1000, "2.1.0"
torch.save(data, sys.argv[1])
'''


def test_load_model_lightning_checkpoint_with_pickled_hparams(tmp_path):
    """A checkpoint as the reference's Lightning trainer writes it:
    hyper_parameters hold pickled omegaconf objects, which the weights-only
    loader reads as inert stand-ins; state_dict and ema still load."""
    import subprocess
    import sys

    path, m, sd, ema = _write_ckpt(str(tmp_path), True)
    subprocess.run([sys.executable, "-c", _LIGHTNING_SAVER, path], check=True, timeout=120)
    with pytest.raises(Exception):
        torch.load(path, weights_only=True)   # plain weights-only refuses it
    model = load_model(path)
    for p, e in zip(model.model_parameters(), ema):
        torch.testing.assert_close(p.detach(), e)


@pytest.mark.parametrize("shape", [(3000,), (2, 3000), (1, 1, 3200)])
@pytest.mark.parametrize("kw", [{}, {"n_steps": 3}, {"warm_start": 2}, {"ensemble": 2},
                                {"use_aux_signal": True}, {"n_steps": 4, "target": True}])
def test_noise_shapes_match_the_oracle_draws(shape, kw):
    """Universe.noise_shapes (what bin/enhance.py discards for other ranks'
    files) lists exactly the randn draws of one enhance, in order: checked
    against the oracle's restatement of universe.py:231-375 (reduced width)."""
    from oracle import ou_oracle

    m = _build("pp16", 4)
    sd = synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()], 0)
    m.load_state_dict(sd, strict=False)
    orc = ou_oracle.Oracle({k: v for k, v in m.state_dict().items()}, get_config("pp16", 4))
    drawn = []

    def noise_fn(s):
        drawn.append(tuple(s))
        return torch.zeros(s)

    mix = torch.randn(shape, generator=torch.Generator().manual_seed(0)) * 0.1
    okw = dict(kw)
    if okw.get("target"):
        okw["target"] = mix.reshape(-1, 1, shape[-1]).clone()
    with torch.no_grad():
        orc.enhance(mix, noise_fn=noise_fn, **okw)
    assert m.noise_shapes(mix.shape, **kw) == drawn
