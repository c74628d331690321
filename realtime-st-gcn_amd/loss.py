"""Segmentation loss and statistics on the GPU (utils/loss.py:8-41, utils/statistics.py:4-16).

``Loss(rank, class_dist, output_type)(i, predictions, ground_truth) -> (ce, mse)`` and
``Statistics()(i, predictions, ground_truth) -> (top1_predicted, top5_predicted, top1_cor, top5_cor, tot)``
keep the reference's call signatures; ``predictions`` is the (1, C, L) series of
``segment_generator.mask_segment`` and ``ground_truth`` (1, L') int64.  Both run one HIP kernel
(loss.hip: log-softmax, weighted CE, clamped temporal MSE, top-1/top-5, and the gradient of both
loss terms in the same pass); the backward is one more launch.  ``shard=`` (parallel.SegmentShard)
makes a data-parallel rank's share of a trial's loss exact: per-rank values sum to the single-process
loss and per-rank gradients equal the single-process ones (parallel.sharded_loss adds DDP's world
scaling and empty shards).
"""
from __future__ import annotations

import torch

from . import _lib as L
from . import native as K

_MODES = {"logits": 0, "logsoftmax": 1, "softmax": 2}


def _rows(predictions: torch.Tensor) -> torch.Tensor:
    """(1, C, L) -> fp32 [L][C] rows (a view when the series is already class-contiguous)."""
    if predictions.dim() != 3 or predictions.shape[0] != 1:
        raise RuntimeError(f"stgcn_amd: loss expects (1, C, L) predictions, got {tuple(predictions.shape)}")
    p = predictions[0].t()
    if p.dtype != torch.float32:
        p = p.float()
    if p.stride(1) != 1:
        p = p.contiguous()
    return p


def seg_loss(p_rows, labels, weight, first=0, mode=0, prev=None, den=None, pairs=None, grads=True, top5=False):
    """Raw launch: p_rows fp32 [L][C] (row stride >= C), labels int64 [L - first] (frames first..L-1).  Returns (out[8], dce, dmse, top5)."""
    L.require_device(p_rows)
    Lw, C = p_rows.shape
    dev = p_rows.device
    labels = labels.reshape(-1)
    if labels.numel() != Lw - int(first):
        raise RuntimeError(f"stgcn_amd: {labels.numel()} labels for {Lw} predictions (first={int(first)})")
    labels = labels.to(device=dev, dtype=torch.long).contiguous()
    weight = weight.to(device=dev, dtype=torch.float32).contiguous()
    out = torch.empty(8, dtype=torch.float32, device=dev)
    dce = torch.empty((Lw, C), dtype=torch.float32, device=dev) if grads else None
    dmse = torch.empty((Lw, C), dtype=torch.float32, device=dev) if grads else None
    t5 = torch.empty((Lw, 5), dtype=torch.int32, device=dev) if top5 else None
    work = torch.empty(max(1, L.lib().stgcn_seg_loss_workspace(Lw) // 4), dtype=torch.float32, device=dev)
    prev_ = den_ = None
    if prev is not None:
        prev_ = prev.reshape(-1).to(device=dev, dtype=torch.float32).contiguous()
    if den is not None:
        den_ = torch.as_tensor(den, dtype=torch.float32).to(dev).reshape(1).contiguous()
    L.check(L.lib().stgcn_seg_loss(p_rows.data_ptr(), p_rows.stride(0), labels.data_ptr(), weight.data_ptr(),
                                   L.ptr(prev_), Lw, C, int(first), int(mode), L.ptr(den_),
                                   float(pairs or 0.0), L.ptr(dce), L.ptr(dmse), L.ptr(t5), work.data_ptr(),
                                   out.data_ptr(), L.stream()), "seg_loss")
    return out, dce, dmse, t5


@K.on_tensor_device
class SegLossFunction(torch.autograd.Function):
    """(ce, mse) of loss.py:25-41 with the gradients computed in the forward launch."""

    @staticmethod
    def forward(ctx, predictions, labels, weight, first, mode, prev, den, pairs):
        p = _rows(predictions)
        out, dce, dmse, _ = seg_loss(p, labels, weight, first, mode, prev, den, pairs,
                                     grads=predictions.requires_grad)
        ctx.save_for_backward(dce, dmse)
        ctx.shape = predictions.shape
        return out[0], out[1]

    @staticmethod
    def backward(ctx, gce, gmse):
        dce, dmse = ctx.saved_tensors
        Lw, C = dce.shape
        dp = torch.empty((Lw, C), dtype=torch.float32, device=dce.device)
        g1 = None if gce is None else gce.float().contiguous()
        g2 = None if gmse is None else gmse.float().contiguous()
        L.check(L.lib().stgcn_seg_loss_bwd(dce.data_ptr(), dmse.data_ptr(), L.ptr(g1), L.ptr(g2), Lw * C,
                                           dp.data_ptr(), L.stream()), "seg_loss_bwd")
        return dp.t().unsqueeze(0), None, None, None, None, None, None, None


class Loss:
    """utils/loss.py:8-41.  ``class_dist`` (C,) class frequencies; CE weights = 1 - class_dist/sum."""

    def __init__(self, rank, class_dist, output_type="logits"):
        if output_type not in _MODES:
            raise ValueError(f"unknown output_type {output_type!r}")
        cd = torch.as_tensor(class_dist, dtype=torch.float32)
        self.weight = (1 - cd / torch.sum(cd)).to(rank)
        self.mode = _MODES[output_type]

    def __call__(self, i, predictions, ground_truth, shard=None):
        first = 0 if i == 0 else 1
        prev = den = pairs = None
        if shard is not None:
            prev, den, pairs = shard.prev, shard.den, shard.pairs
            first = first if shard.rank_first else 0
        return SegLossFunction.apply(predictions, ground_truth, self.weight, first, self.mode, prev, den, pairs)


class Statistics:
    """utils/statistics.py:4-16: top-1 / top-5 hits of the series (frame 0 dropped for i > 0)."""

    def __call__(self, i, predictions, ground_truth):
        first = 0 if i == 0 else 1
        p = _rows(predictions.detach())
        C = p.shape[1]
        out, _, _, t5 = seg_loss(p, ground_truth, torch.ones(C, device=p.device), first, 0, grads=False, top5=True)
        t5 = t5[first:].long().t().unsqueeze(0)                  # (1, 5, L')
        top1_predicted = t5[:, 0, :]
        h = out[2:4].tolist()
        return top1_predicted, t5, int(h[0]), int(h[1]), ground_truth.numel()
