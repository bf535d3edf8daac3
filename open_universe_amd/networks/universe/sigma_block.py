"""Noise-level embeddings (parameters mirror networks/universe/sigma_block.py).

The embedding itself is computed on the device by ``ou_embed`` together with
every FiLM projection of the score network (engine.Engine.rec_embed).
"""
import torch
from torch import nn

from .blocks import PReLU, linear_params


class Linear_PReLU(nn.Module):
    """sigma_block.py:24-33."""

    def __init__(self, in_features, out_features):
        super().__init__()
        self.prelu = PReLU()
        self.lin = linear_params(in_features, out_features)


class SigmaBlock(nn.Module):
    """Random-Fourier-feature MLP of UNIVERSE (sigma_block.py:36-57)."""

    def __init__(self, n_rff=32, n_dim=256, scale=16):
        super().__init__()
        self.register_buffer("freq", scale * torch.zeros(n_rff).normal_())
        self.layer1 = Linear_PReLU(2 * n_rff, 4 * n_rff)
        self.layer2 = Linear_PReLU(4 * n_rff, 8 * n_rff)
        self.layer3 = Linear_PReLU(8 * n_rff, n_dim)


class SimpleTimeEmbedding(nn.Module):
    """UNIVERSE++ sinusoidal embedding with learnt frequency (sigma_block.py:60-78)."""

    def __init__(self, n_dim=256):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros((1, 1)))
        self.bias = nn.Parameter(torch.zeros((1, 1)))
        self.n_dim = n_dim
