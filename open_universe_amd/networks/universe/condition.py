"""UNIVERSE conditioner network (mirrors networks/universe/condition.py).

``ConditionerNetwork.forward`` runs on the MI355X through the HIP engine: the
mel front end is a framed GEMM (STFT) + |.|^2 + filterbank GEMM + global
normalisation folded into the next convolution's input scale.
"""
import math

import torch
from torch import nn

from ... import _lib as L
from ... import dsp
from .blocks import ConvBlock, GRUParams, PReLU_Conv, conv_params


class _Spectrogram(nn.Module):
    def __init__(self, n_fft):
        super().__init__()
        self.register_buffer("window", torch.from_numpy(dsp.hann_periodic(n_fft)))


class _MelScale(nn.Module):
    def __init__(self, n_mels, sample_rate, n_stft):
        super().__init__()
        fb = dsp.melscale_fbanks(n_stft, 0.0, float(sample_rate // 2), n_mels, sample_rate)
        self.register_buffer("fb", torch.from_numpy(fb))


class MelSpectrogram(nn.Module):
    """Buffer container with torchaudio.transforms.MelSpectrogram's names."""

    def __init__(self, sample_rate, n_mels, n_fft, hop_length):
        super().__init__()
        self.spectrogram = _Spectrogram(n_fft)
        self.mel_scale = _MelScale(n_mels, sample_rate, n_fft // 2 + 1)


def make_st_convs(ds_factors, input_channels, num_layers=None, use_weight_norm=False):
    """condition.py:33-65 (use_antialiasing is always False for the encoder)."""
    if num_layers is None:
        num_layers = len(ds_factors) - 1
    st_convs = nn.ModuleList()
    rates = [ds_factors[-1]]
    for r in ds_factors[-2::-1]:
        rates.append(rates[-1] * r)
    rates = rates[::-1]
    for i in range(len(ds_factors)):
        if i >= num_layers:
            st_convs.append(None)
        else:
            st_convs.append(PReLU_Conv(input_channels * 2**i, input_channels * 2 ** len(ds_factors),
                                       rates[i], stride=rates[i], use_weight_norm=use_weight_norm))
    return st_convs


class MelAdapter(nn.Module):
    """condition.py:68-114 (sample_rate hard-coded to 24000 as in the reference)."""

    def __init__(self, n_mels, output_channels, ds_factor, oversample=2, use_weight_norm=False):
        super().__init__()
        self.ds_factor = ds_factor
        n_fft = oversample * ds_factor
        self.mel_spec = MelSpectrogram(24000, n_mels, n_fft, ds_factor)
        self.conv = conv_params(n_mels, output_channels, 3, weight_norm=use_weight_norm)
        self.conv_block = ConvBlock(output_channels, use_weight_norm=use_weight_norm)
        pad_tot = n_fft - ds_factor
        self.pad_left, self.pad_right = pad_tot // 2, pad_tot - pad_tot // 2


class ConditionerEncoder(nn.Module):
    """condition.py:117-220."""

    def __init__(self, ds_factors, input_channels, with_gru_residual=False,
                 with_extra_conv_block=False, act_type="prelu", use_weight_norm=False,
                 seq_model="gru", use_antialiasing=False):
        super().__init__()
        self.with_gru_residual = with_gru_residual
        self.extra_conv_block = with_extra_conv_block
        c = input_channels
        self.ds_modules = nn.ModuleList([
            ConvBlock(c * 2**i, r, "down", act_type=act_type, use_weight_norm=use_weight_norm,
                      antialiasing=use_antialiasing) for i, r in enumerate(ds_factors)])
        self.st_convs = make_st_convs(ds_factors, input_channels, len(ds_factors) - 1, use_weight_norm)
        if self.extra_conv_block:
            self.ds_modules.append(ConvBlock(c * 2 ** len(ds_factors), act_type=act_type,
                                             use_weight_norm=use_weight_norm))
            self.st_convs.append(None)
        oc = input_channels * 2 ** len(ds_factors)
        if seq_model != "gru":
            raise ValueError("Values for 'seq_model' can be gru|attention")
        self.seq_model = seq_model
        self.gru = GRUParams(oc, oc // 2, 2)
        self.conv_block1 = ConvBlock(oc, act_type=act_type, use_weight_norm=use_weight_norm)
        self.conv_block2 = ConvBlock(oc, act_type=act_type, use_weight_norm=use_weight_norm)


class ConditionerDecoder(nn.Module):
    """condition.py:223-270."""

    def __init__(self, up_factors, input_channels, with_extra_conv_block=False, act_type="prelu",
                 use_weight_norm=False, use_antialiasing=False):
        super().__init__()
        self.extra_conv_block = with_extra_conv_block
        n_channels = [input_channels * 2 ** (len(up_factors) - i - 1) for i in range(len(up_factors))]
        self.input_conv_block = ConvBlock(n_channels[0] * 2, act_type=act_type,
                                          use_weight_norm=use_weight_norm)
        up_modules = [ConvBlock(c, r, "up", act_type=act_type, use_weight_norm=use_weight_norm,
                                antialiasing=use_antialiasing) for c, r in zip(n_channels, up_factors)]
        if self.extra_conv_block:
            up_modules = [ConvBlock(2 * n_channels[0], act_type=act_type,
                                    use_weight_norm=use_weight_norm)] + up_modules
        self.up_modules = nn.ModuleList(up_modules)


class ConditionerNetwork(nn.Module):
    """condition.py:273-377."""

    def __init__(self, fb_kernel_size=3, rate_factors=(2, 4, 4, 5), n_channels=32, n_mels=80,
                 n_mel_oversample=4, encoder_gru_residual=False, extra_conv_block=False,
                 encoder_act_type="prelu", decoder_act_type="prelu", precoding=None,
                 input_channels=1, output_channels=None, use_weight_norm=False, seq_model="gru",
                 use_antialiasing=False, **unused):
        super().__init__()
        if precoding or output_channels is not None or input_channels != 1:
            raise NotImplementedError("precoding / output_channels / multichannel input are not "
                                      "used by any target config")
        if not extra_conv_block:
            raise NotImplementedError("the HIP engine targets extra_conv_block=True configs")
        self.config = dict(fb_kernel_size=fb_kernel_size, rate_factors=list(rate_factors),
                           n_channels=n_channels, n_mels=n_mels, n_mel_oversample=n_mel_oversample,
                           encoder_gru_residual=encoder_gru_residual,
                           extra_conv_block=extra_conv_block, use_weight_norm=use_weight_norm,
                           use_antialiasing=use_antialiasing)
        self.input_conv = conv_params(input_channels, n_channels, fb_kernel_size,
                                      weight_norm=use_weight_norm)
        self.output_conv = None
        total_ds = math.prod(rate_factors)
        total_channels = 2 ** len(rate_factors) * n_channels
        self.input_mel = MelAdapter(n_mels, total_channels, total_ds * input_channels,
                                    n_mel_oversample, use_weight_norm=use_weight_norm)
        self.encoder = ConditionerEncoder(rate_factors, n_channels, encoder_gru_residual,
                                          extra_conv_block, encoder_act_type, use_weight_norm,
                                          seq_model, False)
        self.decoder = ConditionerDecoder(list(rate_factors)[::-1], n_channels, extra_conv_block,
                                          decoder_act_type, use_weight_norm, use_antialiasing)
        self.precoding = None
        self._engine = None
        self._plans = {}
        self._conv_prec = None   # None: OUHIP_CONV_PREC; 0 after a split-f16 range error

    def _get_engine(self):
        from ...engine import Engine

        dev = next(self.parameters()).device
        if self._engine is None or self._engine.device != dev:
            cfg = {"score_model": None, "condition_model": self.config, "diffusion": None}
            sd = {"condition_model." + k: v for k, v in self.state_dict().items()}
            self._engine = Engine(cfg, sd, dev, parts=("cond",), conv_prec=self._conv_prec)
            self._plans = {}
        return self._engine

    def _apply(self, fn, *args, **kwargs):
        self._engine, self._plans = None, {}
        return super()._apply(fn, *args, **kwargs)

    def forward(self, x, x_wav=None, train=False):
        """condition.py:346-377 on the HIP engine (x_wav must be x or None:
        no target config uses a transform)."""
        from ...plan import CondPlan

        if x_wav is not None and x_wav is not x and not torch.equal(x_wav, x):
            raise NotImplementedError("x_wav differing from x needs a precoding transform")
        eng = self._get_engine()
        B, _, T = x.shape
        key = (B, T)
        if key not in self._plans:
            self._plans[key] = CondPlan(eng, B, T, need_aux=True)
        try:
            conds, y, h = self._plans[key](x)
        except L.OuRangeError:   # activations left the split-f16 range: f32 operands from now on
            self._conv_prec, self._engine, self._plans = 0, None, {}
            return self.forward(x, x_wav, train)
        conds = [c.clone() for c in conds]
        if train:
            return conds, y.clone(), h.clone()
        return conds
