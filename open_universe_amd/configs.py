"""Model configurations for the three target architectures.

These are the ``model:`` sections of the reference's hydra ``config.yaml`` files,
restricted to the keys the enhancement path reads.  A real checkpoint's
``config.yaml`` is parsed by :mod:`open_universe_amd.inference_utils.model_loader`
into the same structure.

* ``PP16``   -- UNIVERSE++ 16 kHz  (reference ``config/model/default.yaml:1-45``,
  ``config/model/default_orig.yaml``)
* ``ORIG16`` -- UNIVERSE 16 kHz    (reference ``config/model/_old/universe_original.yaml:1-42``)
* ``PP24``   -- UNIVERSE++ 24 kHz  (reference ``config/model/_old/universepp_24k.yaml:1-45``)
"""
import copy

_PP_SCORE = {
    "_target_": "open_universe.networks.universe.ScoreNetwork",
    "fb_kernel_size": 3,
    "rate_factors": [2, 4, 4, 5],
    "n_channels": 32,
    "n_rff": 32,
    "noise_cond_dim": 512,
    "encoder_gru_conv_sandwich": False,
    "extra_conv_block": True,
    "decoder_act_type": "prelu",
    "use_weight_norm": True,
    "use_antialiasing": True,
    "time_embedding": "simple",
}

_PP_COND = {
    "_target_": "open_universe.networks.universe.ConditionerNetwork",
    "fb_kernel_size": 3,
    "rate_factors": [2, 4, 4, 5],
    "n_channels": 32,
    "n_mels": 80,
    "n_mel_oversample": 4,
    "encoder_gru_residual": True,
    "extra_conv_block": True,
    "decoder_act_type": "prelu",
    "use_weight_norm": True,
    "use_antialiasing": False,
}

PP16 = {
    "_target_": "open_universe.networks.universe.UniverseGAN",
    "fs": 16000,
    "normalization_norm": 2,
    "normalization_kwargs": {"ref": "both", "level_db": -26.0},
    "edm": {"noise": 0.25},
    "score_model": _PP_SCORE,
    "condition_model": _PP_COND,
    "diffusion": {
        "schedule": "geometric",
        "sigma_min": 0.0005,
        "sigma_max": 5.0,
        "n_steps": 8,
        "epsilon": 1.3,
    },
    "losses": {"use_signal_decoupling": True, "signal_decoupling_act": "snake"},
}

ORIG16 = {
    "_target_": "open_universe.networks.universe.Universe",
    "fs": 16000,
    "normalization_norm": 2,
    "normalization_kwargs": {"ref": "both", "level_db": -26.0},
    "score_model": dict(
        _PP_SCORE,
        use_weight_norm=False,
        use_antialiasing=False,
        seq_model="gru",
        time_embedding=None,
    ),
    "condition_model": dict(_PP_COND, use_weight_norm=False, seq_model="gru"),
    "diffusion": {
        "schedule": "geometric",
        "sigma_min": 5e-4,
        "sigma_max": 5.0,
        "n_steps": 8,
        "epsilon": 1.3,
    },
    "losses": {},
}

PP24 = copy.deepcopy(PP16)
PP24["fs"] = 24000
PP24["score_model"].update(rate_factors=[2, 3, 5, 8], n_channels=48)
PP24["condition_model"].update(rate_factors=[2, 3, 5, 8], n_channels=48, n_mels=128)

CONFIGS = {"pp16": PP16, "orig16": ORIG16, "pp24": PP24}


def get_config(name, n_channels=None):
    """Return a deep copy of a named config, optionally at reduced width."""
    cfg = copy.deepcopy(CONFIGS[name])
    if n_channels is not None:
        cfg["score_model"]["n_channels"] = n_channels
        cfg["condition_model"]["n_channels"] = n_channels
    return cfg
