"""nn.Modules with the reference's constructor signatures and state_dict key names.

Mirrors models/utils/{tgcn,layernorm,batchnorm}.py and StgcnLayer (models/stgcn/stgcn.py:104-193).
Parameters live in the same submodules as in the reference (``gcn.conv``, ``tcn.0``, ``tcn.2``,
``tcn.3``, ``residual.0``, ``residual.1``) so reference checkpoints load unchanged; the forward
passes go through the HIP kernels (layer_fn.py), never through the submodules' own forward.

``compute_dtype`` (module attribute, default fp32) selects the kernel arithmetic: fp32 for the
parity path, bf16 (fp32 accumulate) for the perf path.  Activations are returned as logical
(N, C, T, V) tensors in channels-last memory.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import layer_fn as F_
from . import native as K
from .syncbn import active_sync

_DTYPES = {"fp32": torch.float32, "bf16": torch.bfloat16, torch.float32: torch.float32,
           torch.bfloat16: torch.bfloat16}


def resolve_dtype(d):
    return _DTYPES[d]


class LayerNorm(nn.Module):
    """Custom LayerNorm over (C,V) per (n,t), unbiased variance (models/utils/layernorm.py:4-28)."""

    def __init__(self, normalized_shape, eps=1e-05, elementwise_affine=True, bias=True, device=None, dtype=None):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(normalized_shape, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.zeros(normalized_shape, device=device, dtype=dtype))
        self.eps = eps
        self.compute_dtype = torch.float32

    def forward(self, x):
        return F_.LayerNormFunction.apply(x, self.weight, self.bias, self.compute_dtype)


class BatchNorm1d(nn.Module):
    """Input BatchNorm1d(V*C) on (N, V*C, T) (models/utils/batchnorm.py:3-23); key ``norm.*``."""

    def __init__(self, features, track_running_stats=False):
        super().__init__()
        self.norm = nn.BatchNorm1d(features, track_running_stats=track_running_stats)
        self.compute_dtype = torch.float32

    def forward(self, x):
        return F_.InputBatchNormFunction.apply(x, self.norm.weight, self.norm.bias, self.compute_dtype,
                                               active_sync(self))


def make_norm(normalization, channels, num_joints):
    """Norm factory of stgcn.py:152 / rtstgcn.py:320."""
    if normalization == "LayerNorm":
        return LayerNorm([channels, 1, num_joints])
    return nn.BatchNorm2d(channels, track_running_stats=False)


class ConvTemporalGraphical(nn.Module):
    """Graph convolution (models/utils/tgcn.py:4-79): ``conv`` = Conv2d(Cin, Cout*P, (t_kernel,1))."""

    def __init__(self, in_channels, out_channels, kernel_size, partitions, t_kernel_size=1, t_stride=1,
                 t_padding=0, t_dilation=1, bias=True):
        super().__init__()
        if (t_kernel_size, t_stride, t_padding, t_dilation) != (1, 1, 0, 1) or not bias:
            raise NotImplementedError("stgcn_amd: ConvTemporalGraphical supports the reference's only use "
                                      "(t_kernel_size=1, stride 1, no padding/dilation, bias=True)")
        self.out_channels = out_channels
        self.partitions = partitions
        self.kernel_size = kernel_size
        self.conv = nn.Conv2d(in_channels, out_channels * partitions, kernel_size=(t_kernel_size, 1))
        self.compute_dtype = torch.float32

    def forward(self, x, A):
        return F_.GcnFunction.apply(x, A, self.conv.weight, self.conv.bias, self.compute_dtype)


class StgcnLayer(nn.Module):
    """Spatial temporal graph convolution layer (models/stgcn/stgcn.py:104-193).

    forward(x (N,C_in,T,V), A (P,V,V) | (N,P,V,V)) -> (N, C_out, T_out, V).
    """

    def __init__(self, in_channels, out_channels, kernel_size, partitions, num_joints, stride=1, dropout=0,
                 residual=True, normalization="LayerNorm"):
        super().__init__()
        assert len(kernel_size) == 2
        assert kernel_size[0] % 2 == 1
        padding = ((kernel_size[0] - 1) // 2, 0)
        self.kernel_size = kernel_size
        self.stride = stride
        self.dropout = dropout
        self.normalization = normalization
        self.is_residual = residual
        self.is_residual_conv = residual and not ((in_channels == out_channels) and (stride == 1))
        self.gcn = ConvTemporalGraphical(in_channels, out_channels, kernel_size[1], partitions)
        self.tcn = nn.Sequential(
            make_norm(normalization, out_channels, num_joints),
            nn.ReLU(inplace=True),
            nn.Conv2d(out_channels, out_channels, (kernel_size[0], 1), stride=(stride, 1), padding=padding),
            make_norm(normalization, out_channels, num_joints),
            nn.Dropout(dropout, inplace=True))
        if self.is_residual_conv:
            self.residual = nn.Sequential(
                nn.Conv2d(in_channels, out_channels, kernel_size=1, stride=(stride, 1)),
                make_norm(normalization, out_channels, num_joints))
        else:
            self.residual = nn.Identity()
        self.compute_dtype = torch.float32
        self._gsup = None
        self._graph_bound = False
        self._fused_cache = {}  # packed weights of the fused inference forward (layer_fn._packs)

    def _drop_packs(self):
        """Forget the packed weights of the fused inference forward.  The cache is keyed by each weight's
        storage and in-place version counter, which optimizer steps and ordinary in-place ops bump; writes
        through ``param.data`` do not, so call ``train()`` / ``eval()`` (or load a state_dict) after such a
        write — both drop the cache."""
        self._fused_cache.clear()

    def train(self, mode: bool = True):
        self._drop_packs()
        return super().train(mode)

    def _load_from_state_dict(self, *args, **kwargs):
        self._drop_packs()
        return super()._load_from_state_dict(*args, **kwargs)

    def bind_graph(self, A, masked=True):
        """Cache the support lists of the static adjacency A (P, V, V) for the joint-gathered graph
        conv.  Every A later passed to forward must have its nonzeros inside this support.  A Model
        binds its graph buffer (``masked``: it passes A * edge_importance, so the gradient of A off the
        support is multiplied by zero and never needed); a bare layer binds the first A it sees and
        keeps the reference's dense dA."""
        s = self._gsup
        if A.dim() == 3 and (s is None or s.V != A.shape[-1] or s.mask.device != A.device):
            self._gsup = K.GraphSupport(A)
        self._graph_bound = self._graph_bound or masked

    def graph_support(self, A):
        if A.dim() != 3:
            return None  # per-sample A (AAGCN): the A-first path
        self.bind_graph(A, masked=False)
        return self._gsup

    def forward(self, x, A, packs=None):
        """``packs``: this layer's layer_fn.LayerPacks from the owning model's one-launch weight preparation
        (stgcn.Model._prepared), or None (the layer packs per call)."""
        if self.dropout and self.training:
            raise NotImplementedError("stgcn_amd: dropout > 0 in training is not implemented (every reference "
                                      "config uses dropout 0)")
        if not self.is_residual and x.shape[1] != self.tcn[2].out_channels:
            # the reference fails here too (stgcn.py:184 keeps C_in channels for the zero residual)
            raise RuntimeError("StgcnLayer(residual=False) requires in_channels == out_channels")
        n1, conv, n2 = self.tcn[0], self.tcn[2], self.tcn[3]
        if self.is_residual_conv:
            rc, rn = self.residual[0], self.residual[1]
            wr, br, nrw, nrb = rc.weight, rc.bias, rn.weight, rn.bias
        else:
            wr = br = nrw = nrb = None
        # inference (no autograd graph will be built): the layer may run the fused forward kernel, which
        # keeps nothing for a backward
        infer = not torch.is_grad_enabled() or not (
            x.requires_grad or A.requires_grad or any(p.requires_grad for p in self.parameters()))
        cfg = (self.kernel_size[0], self.stride, self.is_residual, self.normalization, self.compute_dtype,
               self.graph_support(A), not self._graph_bound, infer, self._fused_cache, None if infer else packs,
               active_sync(self))
        return F_.StgcnLayerFunction.apply(x, A, self.gcn.conv.weight, self.gcn.conv.bias, n1.weight, n1.bias,
                                           conv.weight, conv.bias, n2.weight, n2.bias, wr, br, nrw, nrb, cfg)


def set_compute_dtype(module: nn.Module, dtype):
    """Select fp32 (parity) or bf16 (perf) kernels for every submodule."""
    dt = resolve_dtype(dtype)
    for m in module.modules():
        if hasattr(m, "compute_dtype"):
            m.compute_dtype = dt
    return module
