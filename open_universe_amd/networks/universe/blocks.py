"""Parameter containers mirroring networks/universe/blocks.py.

These modules register exactly the parameters and buffers of the reference
modules, under the same names and in the same order, so that a reference
state dict (and the positional EMA list of torch_ema, ordered like
``model_parameters()``) loads unchanged.  They hold weights only: the compute
is done by the HIP engine (open_universe_amd/engine.py), which reads them once
and packs them for the MI355X kernels.

Reference: networks/universe/blocks.py:34-416 (PReLU_Conv :137-231,
ConvBlock :234-416, BinomialAntiAlias :123-134, cond_weight_norm :40-46).
"""
import math

import torch
from torch import nn

from ... import dsp


class ParamConv(nn.Module):
    """Parameters of a Conv1d / ConvTranspose1d / Linear, optionally
    weight-normalised.  torch.nn.utils.weight_norm deletes ``weight`` and then
    registers ``weight_g`` and ``weight_v``, so the order becomes
    (bias, weight_g, weight_v); plain modules keep (weight, bias)."""

    def __init__(self, weight_shape, bias=True, weight_norm=False, out_dim=0):
        super().__init__()
        weight_shape = tuple(int(s) for s in weight_shape)
        n_out = weight_shape[out_dim]
        b = nn.Parameter(torch.zeros(n_out)) if bias else None
        if weight_norm:
            self.register_parameter("bias", b)
            g_shape = (weight_shape[0],) + (1,) * (len(weight_shape) - 1)
            self.weight_g = nn.Parameter(torch.ones(g_shape))
            self.weight_v = nn.Parameter(torch.empty(weight_shape).normal_(0.0, 0.01))
        else:
            self.weight = nn.Parameter(torch.empty(weight_shape).normal_(0.0, 0.01))
            self.register_parameter("bias", b)


def conv_params(cin, cout, k, bias=True, weight_norm=False, transpose=False):
    if transpose:
        return ParamConv((cin, cout, k), bias, weight_norm, out_dim=1)
    return ParamConv((cout, cin, k), bias, weight_norm)


def linear_params(din, dout, bias=True, weight_norm=False):
    return ParamConv((dout, din), bias, weight_norm)


class PReLU(nn.Module):
    """torch.nn.PReLU() with one scalar slope."""

    def __init__(self, init=0.25):
        super().__init__()
        self.weight = nn.Parameter(torch.full((1,), init))


class BinomialAntiAlias(nn.Module):
    """blocks.py:123-134 (buffer ``weights``)."""

    def __init__(self, kernel_size):
        super().__init__()
        self.register_buffer("weights", torch.from_numpy(dsp.binomial_taps(kernel_size)))


class Snake(nn.Module):
    """bigvgan/snake.py:11-64 (alpha_logscale -> alpha initialised to 0)."""

    def __init__(self, in_features):
        super().__init__()
        self.alpha = nn.Parameter(torch.zeros(in_features))


class _Resample(nn.Module):
    """torchaudio.transforms.Resample buffer container (``kernel``)."""

    def __init__(self, orig, new):
        super().__init__()
        k, _ = dsp.sinc_resample_kernel(orig, new)
        self.register_buffer("kernel", torch.from_numpy(k)[:, None, :])


class Activation1d(nn.Module):
    """bigvgan/alias_free_act.py:8-30."""

    def __init__(self, activation):
        super().__init__()
        self.act = activation
        self.upsample = _Resample(1, 2)
        self.downsample = _Resample(2, 1)


class AliasFreeSnake(nn.Module):
    """bigvgan/snake.py:131-157."""

    def __init__(self, in_features):
        super().__init__()
        self.act = Activation1d(Snake(in_features))


class PReLU_Conv(nn.Module):
    """blocks.py:137-231."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 bias=True, use_transpose=False, act_type="prelu", use_weight_norm=False,
                 use_antialiasing=False):
        super().__init__()
        self.stride = stride
        self.kernel_size = kernel_size
        self.padding = padding
        self.use_transpose = use_transpose
        self.antialiasing = use_antialiasing
        self.bias = None
        if self.antialiasing:
            self.bias = nn.Parameter(torch.zeros(out_channels)) if bias else None
            self.low_pass_filter = BinomialAntiAlias(2 * kernel_size + 1)
            bias = False
        if act_type == "snake":
            self.prelu = AliasFreeSnake(in_channels)
        elif act_type == "prelu":
            self.prelu = PReLU()
        elif act_type == "none":
            self.prelu = None
        else:
            raise ValueError("'act_type' should be one of [prelu | snake]")
        self.conv = conv_params(in_channels, out_channels, kernel_size, bias, use_weight_norm,
                                use_transpose)


class ConvBlock(nn.Module):
    """blocks.py:234-351 (parameters only; forward is the HIP engine)."""

    def __init__(self, n_channels, rate_change=None, rate_change_dir="none", act_type="prelu",
                 antialiasing=False, use_weight_norm=False, signal_cond_type=None):
        super().__init__()
        if rate_change_dir not in ["up", "down", "none"]:
            raise ValueError("The rate_change_dir value should be one of 'up' or 'down'")
        if rate_change_dir in ["up", "down"] and rate_change is None:
            raise ValueError("The rate_change should be specified when using for down/upsampling")
        self.rate = rate_change
        self.rate_change_dir = rate_change_dir
        if rate_change_dir == "down":
            self.in_channels, self.out_channels = n_channels, 2 * n_channels
            self.rate_change_conv = PReLU_Conv(n_channels, 2 * n_channels, rate_change, rate_change,
                                               use_weight_norm=use_weight_norm,
                                               use_antialiasing=antialiasing)
        elif rate_change_dir == "up":
            self.in_channels, self.out_channels = 2 * n_channels, n_channels
            self.rate_change_conv = PReLU_Conv(2 * n_channels, n_channels, rate_change, rate_change,
                                               use_transpose=True, use_weight_norm=use_weight_norm,
                                               use_antialiasing=antialiasing)
        else:
            self.in_channels = self.out_channels = n_channels
            self.rate_change_conv = None
        self.conv1 = PReLU_Conv(n_channels, n_channels, 5, padding="same", act_type=act_type,
                                use_weight_norm=use_weight_norm)
        self.conv2 = PReLU_Conv(n_channels, n_channels, 3, padding="same", act_type=act_type,
                                use_weight_norm=use_weight_norm)
        self.conv3 = PReLU_Conv(n_channels, n_channels, 3, padding="same", act_type=act_type,
                                use_weight_norm=use_weight_norm)
        if signal_cond_type not in (None, "none"):
            raise NotImplementedError("signal_cond_type is only used by research variants")
        self.signal_cond_proj = None


class GRUParams(nn.Module):
    """torch.nn.GRU(bidirectional=True) parameters: per layer, per direction
    weight_ih, weight_hh, bias_ih, bias_hh (gate order r, z, n)."""

    def __init__(self, input_size, hidden_size, num_layers=1):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        k = 1.0 / math.sqrt(hidden_size)
        for layer in range(num_layers):
            din = input_size if layer == 0 else 2 * hidden_size
            for sfx in ("", "_reverse"):
                s = f"_l{layer}{sfx}"
                self.register_parameter("weight_ih" + s, nn.Parameter(torch.empty(3 * hidden_size, din).uniform_(-k, k)))
                self.register_parameter("weight_hh" + s, nn.Parameter(torch.empty(3 * hidden_size, hidden_size).uniform_(-k, k)))
                self.register_parameter("bias_ih" + s, nn.Parameter(torch.empty(3 * hidden_size).uniform_(-k, k)))
                self.register_parameter("bias_hh" + s, nn.Parameter(torch.empty(3 * hidden_size).uniform_(-k, k)))


def film(x, y):
    """blocks.py:57-63 (host-side helper kept for API parity)."""
    if y.shape[1] != 2 * x.shape[1]:
        raise ValueError("g should have 2 times more channels than y")
    y = y.view(y.shape + (1,) * (x.ndim - y.ndim))
    return y[:, : x.shape[1], ...] * x + y[:, x.shape[1]:, ...]
