"""Optional SyncBatchNorm for the HIP BatchNorm layers (the data-parallel default keeps
per-replica batch statistics, mirroring the reference's nn.DataParallel (processor.py:32-33); SyncBN is the
opt-in alternative).  Semantics are torch.nn.SyncBatchNorm's in training mode over one process group:

* forward — every rank merges the BatchNorm partials its GEMM epilogue (or stats pass) wrote into ONE
  (count, mean, M2) entry per channel (``stgcn_bn_merge``, fp64 merge on the GPU), the [ranks][C] entries are
  all-gathered, and ``stgcn_bn_finalize`` merges that list exactly as a single process merges its row blocks:
  the global batch mean and biased variance (stgcn.py:152,160,171 with track_running_stats=False;
  batchnorm.py:13-23 for the input norm).  Ranks may hold different row counts.
* backward — the reduce pass's per-channel (sum dz, sum dz*xhat) are all-reduced together with each rank's
  row count and scaled by M_local / M_global, because the apply kernels divide by their own M: the data
  gradient then uses the global means, as torch's batch_norm_backward_elemt does with the all-reduced sums.
  The parameter gradients stay this rank's own sums (DDP averages them, as with torch.nn.SyncBatchNorm).
* eval — no exchange (torch.nn.SyncBatchNorm syncs only while training).

Messages are 4*C floats per norm and direction (latency-bound small collectives over RCCL); the partial
lists themselves never leave the GPU.  Enable with ``convert_sync_batchnorm(model)`` after
``torch.distributed.init_process_group``; state_dict keys are unchanged.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from . import native as K


class BnSync:
    """The exchange of one process group; shared by every BatchNorm of a model (it holds no per-norm state)."""

    def __init__(self, group=None):
        self.group = group

    def world(self) -> int:
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("stgcn_amd SyncBatchNorm: torch.distributed is not initialised")
        return dist.get_world_size(self.group)

    def finalize(self, part, nb, ld_part, C, gamma, beta, eps=1e-5):
        """bn_finalize over the partials of EVERY rank: (mean_rstd [C][2], scale [C], shift [C])."""
        W = self.world()
        if W == 1:
            return K.bn_finalize(part, nb, ld_part, C, gamma, beta, eps)
        merged = K.bn_merge(part, nb, ld_part, C)
        gathered = torch.empty((W, C, 4), dtype=torch.float32, device=part.device)
        dist.all_gather(list(gathered.unbind(0)), merged, group=self.group)
        return K.bn_finalize(gathered, W, C, C, gamma, beta, eps)

    def all_reduce_sums(self, sums, M, count_lane=False):
        """In place: this rank's per-channel backward sums [C][k] over M rows -> the sums of every rank scaled
        by M / M_global (what the apply kernels, which divide by M, need).  ``count_lane``: sums is [C][4] with
        lane 3 free (the fused backward's float4 rows), which then carries the row count."""
        W = self.world()
        if W == 1:
            return sums
        if count_lane:
            sums[:, 3].fill_(float(M))
            dist.all_reduce(sums, group=self.group)
            sums[:, :3].mul_(float(M) / sums[:, 3:4])
            return sums
        flat = sums.view(-1)
        buf = torch.empty(flat.numel() + 1, dtype=torch.float32, device=sums.device)
        buf[:-1].copy_(flat)
        buf[-1:].fill_(float(M))
        dist.all_reduce(buf, group=self.group)
        flat.copy_(buf[:-1] * (float(M) / buf[-1:]))
        return sums


def _sync_targets(model: nn.Module):
    from .modules import BatchNorm1d, StgcnLayer
    from .rtstgcn import OfflineLayer
    for m in model.modules():
        if isinstance(m, StgcnLayer) and m.normalization != "LayerNorm":
            yield m
        elif isinstance(m, BatchNorm1d):
            yield m
        elif isinstance(m, OfflineLayer) and m.normalization != "LayerNorm":
            yield m


def convert_sync_batchnorm(model: nn.Module, process_group=None) -> nn.Module:
    """Make every BatchNorm of the model's HIP layers (StgcnLayer norm1 / norm2 / residual norm, the input
    BatchNorm1d and its window-staged form, OfflineLayer) synchronise its batch statistics over
    ``process_group`` in training — the counterpart of torch.nn.SyncBatchNorm.convert_sync_batchnorm, in place
    (parameters and state_dict keys untouched).  Returns the model."""
    sync = BnSync(process_group)
    for m in _sync_targets(model):
        m.sync_bn = sync
    return model


def revert_sync_batchnorm(model: nn.Module) -> nn.Module:
    """Back to per-replica statistics (the reference's DataParallel semantics, the default)."""
    for m in _sync_targets(model):
        m.sync_bn = None
    return model


def active_sync(module):
    """The BnSync a module's forward should use now: set and in training mode, else None."""
    s = getattr(module, "sync_bn", None)
    return s if s is not None and module.training else None
