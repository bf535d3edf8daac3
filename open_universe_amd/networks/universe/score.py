"""UNIVERSE score network (mirrors networks/universe/score.py).

Parameter layout is the reference's; ``ScoreNetwork.forward`` runs the whole
network on the MI355X through the HIP engine (one recorded program per input
shape).
"""
import copy

import torch
from torch import nn

from ... import _lib as L
from .blocks import ConvBlock, GRUParams, PReLU, PReLU_Conv, conv_params, linear_params
from .sigma_block import SigmaBlock, SimpleTimeEmbedding


class ScoreEncoder(nn.Module):
    """score.py:27-128."""

    def __init__(self, ds_factors, input_channels, noise_cond_dim, with_gru_conv_sandwich=False,
                 with_extra_conv_block=False, act_type="prelu", use_weight_norm=False,
                 seq_model="gru", use_antialiasing=False):
        super().__init__()
        c = input_channels
        self.extra_conv_block = with_extra_conv_block
        self.ds_modules = nn.ModuleList([
            ConvBlock(c * 2**i, r, "down", act_type=act_type, use_weight_norm=use_weight_norm,
                      antialiasing=use_antialiasing)
            for i, r in enumerate(ds_factors)])
        self.cond_proj = nn.ModuleList([
            linear_params(noise_cond_dim, c * 2 ** (i + 1), weight_norm=use_weight_norm)
            for i in range(len(ds_factors))])
        oc = input_channels * 2 ** len(ds_factors)
        if self.extra_conv_block:
            self.ds_modules.append(ConvBlock(oc, act_type=act_type, use_weight_norm=use_weight_norm))
            self.cond_proj.append(linear_params(noise_cond_dim, 2 * oc, weight_norm=use_weight_norm))
        if seq_model != "gru":
            raise ValueError("only seq_model='gru' is on the enhancement path")
        if with_gru_conv_sandwich:
            raise NotImplementedError("encoder_gru_conv_sandwich is not used by any target config")
        self.seq_model = seq_model
        self.gru = GRUParams(oc, oc // 2, 1)
        self.gru_conv_sandwich = False


class ScoreDecoder(nn.Module):
    """score.py:131-211."""

    def __init__(self, up_factors, input_channels, noise_cond_dim, with_extra_conv_block=False,
                 act_type="prelu", use_weight_norm=False, use_antialiasing=False):
        super().__init__()
        self.extra_conv_block = with_extra_conv_block
        n_channels = [input_channels * 2 ** (len(up_factors) - i - 1) for i in range(len(up_factors))]
        self.up_modules = nn.ModuleList()
        self.noise_cond_proj = nn.ModuleList()
        self.signal_cond_proj = nn.ModuleList()
        if self.extra_conv_block:
            oc = input_channels * 2 ** len(up_factors)
            self.up_modules.append(ConvBlock(oc, act_type=act_type, use_weight_norm=use_weight_norm))
            self.noise_cond_proj.append(linear_params(noise_cond_dim, 2 * oc, weight_norm=use_weight_norm))
            self.signal_cond_proj.append(conv_params(oc, oc, 1, weight_norm=use_weight_norm))
        for c, r in zip(n_channels, up_factors):
            self.up_modules.append(ConvBlock(c, r, "up", act_type=act_type, use_weight_norm=use_weight_norm,
                                             antialiasing=use_antialiasing))
            self.noise_cond_proj.append(linear_params(noise_cond_dim, 2 * c, weight_norm=use_weight_norm))
            self.signal_cond_proj.append(conv_params(c, c, 1, weight_norm=use_weight_norm))


class ScoreNetwork(nn.Module):
    """score.py:214-298."""

    def __init__(self, fb_kernel_size=3, rate_factors=(2, 4, 4, 5), n_channels=32, n_rff=32,
                 noise_cond_dim=512, encoder_gru_conv_sandwich=False, extra_conv_block=False,
                 encoder_act_type="prelu", decoder_act_type="prelu", precoding=None,
                 input_channels=1, output_channels=1, use_weight_norm=False, seq_model="gru",
                 use_antialiasing=False, time_embedding=None, **unused):
        super().__init__()
        if precoding:
            raise NotImplementedError("precoding is not used by any target config")
        if not extra_conv_block:
            raise NotImplementedError("the HIP engine targets extra_conv_block=True configs")
        self.config = dict(fb_kernel_size=fb_kernel_size, rate_factors=list(rate_factors),
                           n_channels=n_channels, n_rff=n_rff, noise_cond_dim=noise_cond_dim,
                           extra_conv_block=extra_conv_block, use_weight_norm=use_weight_norm,
                           use_antialiasing=use_antialiasing, time_embedding=time_embedding)
        if time_embedding == "simple":
            self.sigma_block = SimpleTimeEmbedding(n_dim=noise_cond_dim)
        else:
            self.sigma_block = SigmaBlock(n_rff, noise_cond_dim)
        self.input_channels = input_channels
        self.output_channels = output_channels
        self.input_conv = conv_params(input_channels, n_channels, fb_kernel_size)
        self.encoder = ScoreEncoder(rate_factors, n_channels, noise_cond_dim,
                                    encoder_gru_conv_sandwich, extra_conv_block, encoder_act_type,
                                    use_weight_norm, seq_model, use_antialiasing)
        self.decoder = ScoreDecoder(list(rate_factors)[::-1], n_channels, noise_cond_dim,
                                    extra_conv_block, decoder_act_type, use_weight_norm,
                                    use_antialiasing)
        self.prelu = PReLU()
        self.output_conv = PReLU_Conv(n_channels, output_channels, fb_kernel_size, padding="same",
                                      use_weight_norm=use_weight_norm)
        self.precoding = None
        self._engine = None
        self._plans = {}
        self._conv_prec = None   # None: OUHIP_CONV_PREC; 0 after a split-f16 range error

    def _get_engine(self):
        from ...engine import Engine

        dev = self.input_conv.weight.device
        if self._engine is None or self._engine.device != dev:
            cfg = {"score_model": self.config, "condition_model": None, "diffusion": None}
            sd = {"score_model." + k: v for k, v in self.state_dict().items()}
            self._engine = Engine(cfg, sd, dev, parts=("score",), conv_prec=self._conv_prec)
            self._plans = {}
        return self._engine

    def _apply(self, fn, *args, **kwargs):
        self._engine, self._plans = None, {}
        return super()._apply(fn, *args, **kwargs)

    def forward(self, x, sigma, cond):
        """score.py:278-298 on the HIP engine.  x (B, 1, T), sigma (B,), cond =
        the conditioner's 5 per-level tensors."""
        from ...plan import ScorePlan

        eng = self._get_engine()
        B, _, T = x.shape
        key = (B, T)
        if key not in self._plans:
            self._plans[key] = ScorePlan(eng, B, T)
        try:
            return self._plans[key](x, sigma, cond).clone()
        except L.OuRangeError:   # activations left the split-f16 range: f32 operands from now on
            self._conv_prec, self._engine, self._plans = 0, None, {}
            return self.forward(x, sigma, cond)
