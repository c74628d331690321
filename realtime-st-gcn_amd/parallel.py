"""Data-parallel plumbing: shard long trials across ranks, make the loss of a sharded trial exact, wrap
the model for RCCL gradient all-reduce, accumulate gradients over micro-steps.

The reference's multi-GPU path is single-process nn.DataParallel (processor.py:32-33): it scatters the
batch dimension — sliding windows (WindowSegment, utils/segment_generator.py:109-154) or overlapping
time chunks (BufferSegment, segment_generator.py:18-106) of ONE trial — over the GPUs, gathers the
predictions onto cuda:0 for the loss, and reduces the gradients there.  Here every GPU is its own
process (torch.distributed, backend "nccl" = RCCL over xGMI); each rank takes a contiguous slice of the
windows/chunks, computes its share of the trial's loss (``SegmentShard``: the one cross-shard term is
the temporal MSE pair at the shard boundary, which needs the previous rank's last prediction row — an
all-gather of C floats per rank), and DistributedDataParallel all-reduces the fp32 gradients in buckets
overlapped with backward.  BatchNorm statistics stay per replica, exactly like the reference's
DataParallel replicas.  Gradient accumulation over trials (processor.py:531-564: ``loss /= batch_size``,
optimizer step every ``batch_size`` trials) skips the all-reduce on all but the last micro-step
(``accumulate``).
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass
from typing import Optional

import torch


def rank_slice(n_units: int, world: int, rank: int):
    """Contiguous [start, end) of ``n_units`` owned by ``rank`` (sizes differ by at most one)."""
    base, extra = divmod(n_units, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def windows_for_rank(trial: torch.Tensor, W: int, world: int, rank: int) -> torch.Tensor:
    """trial (1, C, L, V) -> this rank's windows (n, C, W, V) (segment_generator.py:116-122,132-145): the
    trial is left-padded by W-1 zero frames and output frame t is predicted from padded frames [t, t+W)."""
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


@dataclass
class SegmentShard:
    """What one rank needs to compute its exact share of a trial's loss (loss.Loss(..., shard=)).

    prev: (C,) predictions of the frame right before this shard (the detached left operand of the
          boundary MSE pair, loss.py:36-39), None for the shard that starts the series;
    den:  the trial's CE weight sum  sum_w wt[y_w]  (device scalar) — every rank holds the trial's labels;
    pairs: the trial's number of MSE pairs (L - 1);
    rank_first: this shard holds frame 0 (only it applies the subsegment's ``i > 0`` frame drop)."""
    prev: Optional[torch.Tensor]
    den: torch.Tensor
    pairs: int
    rank_first: bool

    @staticmethod
    def local(pred_full, labels_full, weight, start, end, L, rank):
        """Shard [start, end) of a series whose predictions are all in this process (tests, single GPU)."""
        prev = pred_full[0, :, start - 1].detach() if start > 0 else None
        den = weight[labels_full.reshape(-1).to(weight.device)].sum()
        return SegmentShard(prev, den, L - 1, start == 0)


def exchange_shard(pred_local, labels_full, weight, start, L, group=None):
    """Build this rank's SegmentShard in a process group: all-gather every rank's last prediction row
    (C floats each) so rank r gets the row right before its first frame.
    pred_local: (1, C, n) this rank's predictions (n may be 0); labels_full: the whole series' labels."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    C = pred_local.shape[1]
    last = pred_local[0, :, -1].detach().float() if pred_local.shape[2] > 0 else \
        torch.zeros((C,), device=pred_local.device)
    rows = [torch.empty_like(last) for _ in range(world)]
    dist.all_gather(rows, last.contiguous(), group=group)
    # rank_slice gives shards that differ by at most one unit, so only trailing shards can be empty and
    # the shard before a non-empty rank r > 0 is rank r - 1
    prev = rows[rank - 1] if start > 0 else None
    den = weight[labels_full.reshape(-1).to(weight.device)].sum()
    return SegmentShard(prev, den, L - 1, start == 0)


def sharded_loss(crit, i, pred_local, labels_local, shard: SegmentShard, world: int):
    """This rank's share of a sharded trial's loss, ready for DDP: ``crit`` (loss.Loss) on the local
    predictions (1, C, n) and their labels with the shard's cross-rank terms, each term multiplied by
    ``world`` because DistributedDataParallel averages the gradients over ranks (the shares sum to the
    trial's loss, so the averaged gradient is the single-process one).  A rank whose shard is empty
    (n = 0, possible when a trial has fewer units than ranks) contributes zeros connected to its
    predictions, so its backward still takes part in the all-reduce."""
    if pred_local.shape[2] == 0:
        z = pred_local.sum() * 0.0
        return z, z
    ce, mse = crit(i, pred_local, labels_local, shard=shard)
    return ce * world, mse * world


def ddp(model: torch.nn.Module, device: torch.device, bucket_cap_mb: int = 4):
    """DistributedDataParallel over the initialised process group (RCCL on the GPU box, gloo in tests).  4 MB
    buckets: the config-2 gradient (12.2 MB fp32) goes out in ~4 all-reduces, the first as soon as the last
    (256-channel, ~3 MB each) layers' backward is done, so the ring transfers overlap the rest of the backward
    (16 MB buckets held the whole gradient until the backward ended)."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    ids = [device.index] if device.type == "cuda" else None
    return DDP(model, device_ids=ids, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True)


@contextlib.contextmanager
def accumulate(model, last: bool):
    """Micro-step context for gradient accumulation (processor.py:531-564): under DDP the bucketed
    all-reduce runs only on the ``last`` micro-step of an optimizer step (DDP.no_sync on the others);
    a plain module accumulates locally either way."""
    if not last and hasattr(model, "no_sync"):
        with model.no_sync():
            yield
    else:
        yield


@dataclass
class SegmentUnit:
    """One WindowSegment subsegment of one trial: the unit of work the data-parallel path distributes.

    trial: index of the trial; i / count: the subsegment's index and the trial's subsegment count (the
    reference's ``i`` and ``num_subsegments``, processor.py:377-392); n0 / nw: windows [n0, n0 + nw) of the
    padded capture; y0 / y1: its label frames."""
    trial: int
    i: int
    count: int
    n0: int
    nw: int
    y0: int
    y1: int


def segment_units(lengths, W: int, segment: int):
    """Every subsegment of every trial (lengths = frames per trial), in trial order.  The subsegments of a
    trial are independent units — each has its own loss term ce/count + mse/count (processor.py:377-392,
    utils/loss.py:25-41, with the one-frame overlap that carries the MSE pair across the boundary) and the
    reference accumulates their gradients — so they shard across ranks with no data-path collective: the
    ranks' gradient sum (DDP's all-reduce) is the reference's accumulated gradient."""
    from .segment import window_segments
    out = []
    for k, L in enumerate(lengths):
        segs = window_segments(L, L + W - 1, L, W, segment)
        for i, (sx, ex, sy, ey) in enumerate(segs):
            out.append(SegmentUnit(k, i, len(segs), sx, ex - sx - (W - 1), sy, ey))
    return out


def units_for_rank(units, world: int, rank: int):
    """Round-robin deal of the units (sizes of consecutive units are alike, so every rank gets the same
    work within one unit)."""
    return units[rank::world]


class GraphedStep:
    """A fixed-shape training step replayed as HIP graphs (processor.py:531-564 inner loop with the batch in
    static buffers): one graph launch for the ~250 kernels of the forward, loss and backward on one stream.

    Flat mode (``bucket_mb=None``, any backend):

        graph 1: ``fwd_loss()`` (forward + loss), backward — the gradients are the backward's own outputs
                 (captured with ``grad = None``, so static graph-pool tensors, written afresh by every replay) —
                 [N > 1: copy the fp32 gradients into one flat buffer]
        N > 1:   all-reduce of the flat buffer over ``group`` (eager, one collective; not captured)
        graph 2: [N > 1: the averaged flat gradient back into .grad] + ``opt.step()``

    Bucket mode (``bucket_mb`` set; an initialised process group of a capturable backend — RCCL): ONE graph
    holds the whole step
    with the gradient exchange overlapped with the backward, as DistributedDataParallel does eagerly.  The
    gradients of the trained parameters are views into per-bucket flat buffers (``bucket_mb`` MB of fp32
    each, filled in reverse parameter order — the order the backward finishes them, as DDP assumes); a
    post-accumulate-grad hook counts each bucket's parameters while the step is captured and, when the last
    one is accumulated, issues that bucket's all-reduce asynchronously (RCCL's stream, captured as a fork of
    the graph), so it runs under the rest of the backward; the graph joins every bucket's collective, divides
    by N and runs ``opt.step()``.  Replays run the recorded collectives; the hooks fire only during capture.

    ``fwd_loss`` must only read tensors whose storage stays put between replays (copy new batches into the
    tensors it closes over).  The optimizer must be capturable: the package's ``optim.Adam`` (device-side step
    counters; what bench.py uses) or torch.optim.Adam(capturable=True).  One eager step runs first (on a side
    stream, as graph capture requires) so that every gradient and optimizer state tensor exists and keeps its
    address.  A parameter that got no gradient in it keeps ``grad = None`` and is left out of the captured zeroing,
    the all-reduce and the update (the optimizers skip ``None`` gradients, as an eager step would: its Adam
    moments and, with weight decay, its value stay put).  Replays do not bump the parameters' version counters (host-side bookkeeping is not captured):
    call ``train()`` / ``eval()`` before an inference forward that should see replayed updates."""

    def __init__(self, fwd_loss, params, opt, world: int = 1, group=None, bucket_mb=None, capture: bool = True):
        """``capture=False`` (bucket mode only): the same bucketed step run eagerly on every call — the hooks issue
        the bucket all-reduces as the backward finishes them — for process groups that cannot be captured
        (gloo) and for debugging the exchange outside a graph."""
        self.fwd_loss, self.params, self.opt = fwd_loss, list(params), opt
        self.world, self.group = world, group
        self.capture = capture
        if not capture and bucket_mb is None:
            raise ValueError("GraphedStep(capture=False) needs bucket_mb (the flat mode is graph-only)")
        self.flat = None
        self.buckets = None
        dev = self.params[0].device
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            self.opt.zero_grad(set_to_none=False)
            self.fwd_loss().backward()
            # the parameters this step trains: the ones that received a gradient in the eager step
            self.used = [p for p in self.params if p.grad is not None]
            self.numels = [p.numel() for p in self.used]
            if bucket_mb is not None:  # (world 1 too: the collectives then are identities, still recorded)
                self._make_buckets(bucket_mb)
                for flat, _ in self.buckets:
                    self._allreduce(flat)
                self._apply()
                self.g1, self.g2 = None, None
                if capture:
                    self.g1 = torch.cuda.CUDAGraph()
                    # thread-local capture: the process group's watchdog thread keeps querying its events meanwhile
                    with torch.cuda.graph(self.g1, stream=s, capture_error_mode="thread_local"):
                        self.loss = self._bucketed_step()
            else:
                if world > 1:
                    self.flat = torch.zeros(sum(self.numels), device=dev)
                    torch.cat([p.grad.reshape(-1) for p in self.used], out=self.flat)
                    self._allreduce(self.flat)
                self._apply()
                self.g1, self.g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                # the gradients are created by the captured backward itself (AccumulateGrad takes the produced
                # tensor, from the graph's private pool, static across replays): no per-parameter zero fill and
                # accumulate-add kernels (~2 x 96 small launches per replay)
                for p in self.used:
                    p.grad = None
                with torch.cuda.graph(self.g1, stream=s):
                    self.loss = self._fwd_bwd()
                if any(p.grad is None for p in self.used):
                    raise RuntimeError("GraphedStep: a parameter lost its gradient in the captured step")
                with torch.cuda.graph(self.g2, stream=s):
                    self._apply()
        torch.cuda.current_stream(dev).wait_stream(s)

    def _make_buckets(self, bucket_mb):
        """Per-bucket flat fp32 buffers, the trained parameters' .grad re-pointed into them (current values kept),
        and the readiness hooks."""
        cap = max(1, int(bucket_mb * (1 << 20)) // 4)
        groups, cur, n = [], [], 0
        for p in reversed(self.used):
            if p.grad.dtype != torch.float32:
                raise ValueError("GraphedStep(bucket_mb=...): fp32 gradients only")
            if cur and n + p.numel() > cap:
                groups.append(cur)
                cur, n = [], 0
            cur.append(p)
            n += p.numel()
        if cur:
            groups.append(cur)
        self.buckets = []
        self._hooks = []
        for b, ps in enumerate(groups):
            flat = torch.empty(sum(p.numel() for p in ps), dtype=torch.float32, device=ps[0].device)
            o = 0
            for p in ps:
                v = flat[o:o + p.numel()].view(p.shape)
                v.copy_(p.grad)
                p.grad = v
                o += p.numel()
                self._hooks.append(p.register_post_accumulate_grad_hook(lambda _p, b=b: self._ready(b)))
            self.buckets.append((flat, len(ps)))
        self._capturing = False

    def remove_hooks(self):
        """Detach the bucket mode's readiness hooks from the parameters (they hold this step object); the step
        must not be called afterwards."""
        for h in getattr(self, "_hooks", ()):
            h.remove()
        self._hooks = []

    def _ready(self, b):
        if not self._capturing:  # set during the captured (or, capture=False, the eager) bucketed step
            return
        self._count[b] += 1
        if self._count[b] == self.buckets[b][1]:
            import torch.distributed as dist
            self._works.append(dist.all_reduce(self.buckets[b][0], group=self.group, async_op=True))
            self._launched[b] = True

    def _bucketed_step(self):
        for flat, _ in self.buckets:
            flat.zero_()
        self._count = [0] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._works = []
        self._capturing = True
        try:
            loss = self.fwd_loss()
            loss.backward()
        finally:
            self._capturing = False
        import torch.distributed as dist
        for b, (flat, _) in enumerate(self.buckets):
            if not self._launched[b]:  # a parameter of the bucket got no gradient in this step: exchange anyway
                self._works.append(dist.all_reduce(flat, group=self.group, async_op=True))
        for w in self._works:
            w.wait()  # the capturing stream joins the collective's stream
        for flat, _ in self.buckets:
            flat.div_(self.world)
        self.opt.step()
        return loss.detach()

    def _fwd_bwd(self):
        loss = self.fwd_loss()
        loss.backward()
        if self.flat is not None:
            torch.cat([p.grad.reshape(-1) for p in self.used], out=self.flat)
        return loss.detach()

    def _allreduce(self, t):
        import torch.distributed as dist
        dist.all_reduce(t, group=self.group)

    def _apply(self):
        if self.buckets is not None:
            for flat, _ in self.buckets:
                flat.div_(self.world)
        elif self.flat is not None:
            for p, g in zip(self.used, torch.split(self.flat, self.numels)):
                p.grad.copy_(g.view_as(p.grad)).div_(self.world)
        self.opt.step()

    def __call__(self):
        if self.g1 is None:  # capture=False: the bucketed step eagerly
            self.loss = self._bucketed_step()
            return self.loss
        self.g1.replay()
        if self.g2 is not None:
            if self.flat is not None:
                self._allreduce(self.flat)
            self.g2.replay()
        return self.loss
