"""Drop-in ``load_model`` (mirrors inference_utils/model_loader.py:33-140).

Reads the reference's checkpoint layout unchanged:
  * ``config.yaml`` next to the checkpoint, in ``../.hydra/`` or
    ``../../../.hydra/`` (model_loader.py:33-51); hydra ``_target_`` strings of
    ``open_universe.networks.universe{,_orig}.*`` resolve to this package's
    classes, ``${a.b.c}`` interpolations are resolved without omegaconf;
  * ``torch.load(..., weights_only=True)["state_dict"]`` (Lightning's
    pickled ``hyper_parameters`` etc. load as inert stand-ins, see
    ``load_checkpoint``); discriminator / MDN loss keys
    (``loss_*``) are training-only and skipped;
  * the torch_ema block ``ckpt["ema"]["shadow_params"]``, a positional list in
    ``model.model_parameters()`` order, which ``Universe.eval()`` copies over
    the live parameters in the reference (universe.py:841-865): applied here at
    load time, so inference always runs on the EMA weights.
"""
import re
from pathlib import Path

import torch
import yaml

from ..networks.universe import ConditionerNetwork, ScoreNetwork, Universe, UniverseGAN

_TARGETS = {
    "UniverseGAN": UniverseGAN,
    "Universe": Universe,
    "ScoreNetwork": ScoreNetwork,
    "ConditionerNetwork": ConditionerNetwork,
}
_KNOWN_PREFIXES = ("open_universe.networks.universe", "open_universe.networks.universe_orig",
                   "open_universe_amd.networks.universe")


def ckpt_to_config_path(ckpt_path):
    ckpt_path = Path(ckpt_path)
    candidates = [ckpt_path.parent / "config.yaml"]
    parents = ckpt_path.parents
    if len(parents) > 1:
        candidates.append(parents[1] / ".hydra/config.yaml")
    if len(parents) > 3:
        candidates.append(parents[3] / ".hydra/config.yaml")
    for c in candidates:
        if c.exists():
            return c
    raise ValueError(f"Could not find the configuration file for model {ckpt_path}.")


_INTERP = re.compile(r"\$\{([^}]+)\}")


def _lookup(root, path):
    node = root
    for part in path.split("."):
        node = node[part]
    return node


def resolve_interpolations(cfg, root=None):
    """Resolve OmegaConf-style absolute ``${a.b.c}`` references."""
    root = cfg if root is None else root
    if isinstance(cfg, dict):
        return {k: resolve_interpolations(v, root) for k, v in cfg.items()}
    if isinstance(cfg, list):
        return [resolve_interpolations(v, root) for v in cfg]
    if isinstance(cfg, str):
        m = _INTERP.fullmatch(cfg.strip())
        if m:
            try:
                return resolve_interpolations(_lookup(root, m.group(1)), root)
            except (KeyError, TypeError):
                return None  # e.g. ${datamodule...} (training-only keys)
    return cfg


def open_update_config(path):
    with open(path, "r") as f:
        config = yaml.safe_load(f)
    return resolve_interpolations(config)


def instantiate(cfg):
    target = cfg["_target_"]
    mod, _, name = target.rpartition(".")
    if mod not in _KNOWN_PREFIXES or name not in _TARGETS:
        raise ValueError(f"unsupported model target {target}")
    return _TARGETS[name](**{k: v for k, v in cfg.items() if k != "_target_"})


class _Inert:
    """Stand-in for one of the hyper-parameter classes listed below
    (omegaconf ``DictConfig`` / node / metadata objects and the typing and
    builtins globals their metadata names).  Constructing it and setting its
    state run no code from the file; the loader never reads these objects."""

    def __init__(self, *args, **kwargs):
        pass

    def __setstate__(self, state):
        self.__dict__["_state"] = state


# The non-tensor globals a checkpoint of the reference's Lightning trainer
# names (save_hyperparameters(), universe.py:66, pickles omegaconf containers
# into ``hyper_parameters``): each is allow-listed for the weights-only
# unpickler as an inert ``_Inert`` stand-in, never as the real class.
_HPARAM_GLOBALS = (
    ["omegaconf.dictconfig.DictConfig", "omegaconf.listconfig.ListConfig",
     "omegaconf.base.ContainerMetadata", "omegaconf.base.Metadata", "omegaconf.base.Node",
     "omegaconf.base.Container", "omegaconf.basecontainer.BaseContainer"]
    + [f"omegaconf.nodes.{n}" for n in ("AnyNode", "ValueNode", "StringNode", "IntegerNode", "FloatNode",
                                         "BooleanNode", "BytesNode", "PathNode", "EnumNode")]
    + ["typing.Any"]
    + [f"builtins.{n}" for n in ("dict", "list", "int", "float", "str", "bool")]
    + ["pytorch_lightning.utilities.parsing.AttributeDict", "lightning_fabric.utilities.data.AttributeDict"]
)


def load_checkpoint(path):
    """``torch.load(path, weights_only=True)`` that also accepts a checkpoint
    the reference's Lightning trainer wrote: the fixed list of
    hyper-parameter globals above loads as inert stand-ins.  Anything else the
    weights-only unpickler refuses still raises.  Only ``state_dict`` and
    ``ema`` are read from the result."""
    stubs = []
    for name in _HPARAM_GLOBALS:
        stub = type(name.rsplit(".", 1)[-1], (_Inert,), {})
        stubs.append((stub, name))
        if name.startswith("builtins."):   # the unpickler may name builtins bare
            stubs.append((stub, name[len("builtins."):]))
    with torch.serialization.safe_globals(stubs):
        return torch.load(path, map_location="cpu", weights_only=True)


def load_model(ckpt_path, device=None, strict=True, return_config=False, hf_token=None):
    """Load a model from a checkpoint file (or a Hugging Face id when the hub is
    reachable) -- model_loader.py:65-140."""
    if not Path(ckpt_path).exists():
        try:
            from huggingface_hub import hf_hub_download

            colon = ckpt_path.find(":")
            repo_id, revision = (ckpt_path[:colon], ckpt_path[colon + 1:]) if colon >= 0 else (ckpt_path, None)
            ckpt_path = hf_hub_download(repo_id=repo_id, filename="weights.ckpt", revision=revision,
                                        token=hf_token)
            config_path = hf_hub_download(repo_id=repo_id, filename="config.yaml", revision=revision,
                                          token=hf_token)
        except Exception as e:
            print(f"{ckpt_path} is not a local file and download from HF hub failed.")
            raise e
    else:
        ckpt_path = Path(ckpt_path)
        config_path = ckpt_to_config_path(ckpt_path)

    config = open_update_config(config_path)
    model = instantiate(config["model"])
    data = load_checkpoint(ckpt_path)
    state = {k: v for k, v in data["state_dict"].items() if not k.startswith("loss_")}
    if "ema" in data and data["ema"] is not None:
        model.load_state_dict(state, strict=False)
        shadow = data["ema"]["shadow_params"]
        params = list(model.model_parameters())
        if len(shadow) != len(params):
            raise RuntimeError(f"EMA has {len(shadow)} tensors, model has {len(params)} parameters")
        with torch.no_grad():
            for p, s in zip(params, shadow):
                if p.shape != s.shape:
                    raise RuntimeError(f"EMA shape mismatch {tuple(s.shape)} vs {tuple(p.shape)}")
                p.copy_(s)
    else:
        model.load_state_dict(state, strict=strict)
    model = model.to(device) if device is not None else model
    model.eval()
    if return_config:
        return model, config
    return model
