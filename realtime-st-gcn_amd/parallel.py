"""Data-parallel plumbing: shard long trials across ranks, wrap the model for RCCL gradient all-reduce.

The reference's multi-GPU path is single-process nn.DataParallel (processor.py:32-33): it scatters the
batch dimension — sliding windows (WindowSegment, utils/segment_generator.py:109-154) or overlapping
time chunks (BufferSegment, segment_generator.py:18-106) of ONE trial — over the GPUs and reduces the
gradients onto cuda:0.  Here every GPU is its own process (torch.distributed, backend "nccl" = RCCL
over xGMI); each rank takes a contiguous slice of the windows/chunks (no data-path collective), and
DistributedDataParallel all-reduces the fp32 gradients in buckets overlapped with backward.
BatchNorm statistics stay per replica, exactly like the reference's DataParallel replicas.
"""
from __future__ import annotations

import torch


def rank_slice(n_units: int, world: int, rank: int):
    """Contiguous [start, end) of ``n_units`` owned by ``rank`` (sizes differ by at most one)."""
    base, extra = divmod(n_units, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def window_starts(L: int, W: int):
    """WindowSegment: the trial is left-padded by W-1 zero frames (segment_generator.py:116-122) and
    every output frame t is predicted from the window [t, t+W) of the padded trial (:143)."""
    return torch.arange(L)


def windows_for_rank(trial: torch.Tensor, W: int, world: int, rank: int) -> torch.Tensor:
    """trial (1, C, L, V) on the device -> this rank's windows (n, C, W, V) (segment_generator.py:132-145)."""
    _, C, L, V = trial.shape
    s, e = rank_slice(L, world, rank)
    padded = torch.nn.functional.pad(trial, (0, 0, W - 1, 0))
    win = padded[:, :, s:e + W - 1].unfold(2, W, 1)           # (1, C, n, V, W)
    return win.permute(0, 2, 1, 4, 3).reshape(e - s, C, W, V)


def chunk_bounds(L: int, chunk: int, overlap: int):
    """BufferSegment: chunks of ``chunk`` frames overlapping by ``overlap`` = Kt-1 frames so that the
    causal state of the RT model is replayed (segment_generator.py:25-77).  Returns [(start, end)]."""
    if chunk <= overlap:
        raise ValueError("chunk must exceed the overlap")
    out, s = [], 0
    while True:
        e = min(L, s + chunk)
        out.append((s, e))
        if e == L:
            return out
        s = e - overlap


def chunks_for_rank(L: int, chunk: int, overlap: int, world: int, rank: int):
    b = chunk_bounds(L, chunk, overlap)
    s, e = rank_slice(len(b), world, rank)
    return b[s:e]


def ddp(model: torch.nn.Module, device: torch.device, bucket_cap_mb: int = 16):
    """DistributedDataParallel over the initialised process group (RCCL on the GPU box, gloo in tests)."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    ids = [device.index] if device.type == "cuda" else None
    return DDP(model, device_ids=ids, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True)
