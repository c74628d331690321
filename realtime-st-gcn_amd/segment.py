"""Trial segmentation (utils/segment_generator.py): how a (1, C, L, V) capture becomes model batches.

``WindowSegment`` (segment_generator.py:109-154, st-gcn / aa-gcn): output frame t is predicted from the
``receptive_field`` W frames ending at t (the capture is left-padded by W-1 zero frames,
processor.py:372-374); ``segment`` windows form one batch.  The reference materialises every batch with
``unfold(...).contiguous()`` — (n, C, W, V), a W-fold copy of the capture — and then runs norm_in and
fcn_in over the copies.  Here ``get_segment`` yields a ``WindowBatch`` (the padded capture + window range,
no copy); ``stgcn.Model.forward`` recognises it and builds the first activation straight from the capture
(window.hip via ``layer_fn.WindowStageFunction``).  ``WindowBatch.materialize()`` gives the reference's
tensor for any other consumer.

``BufferSegment`` (segment_generator.py:18-106, rt-st-gcn): time chunks overlapping by G-1 frames
(``kernel`` G), batched over data-parallel replicas and folded back; a copy of C·S·V per chunk (no
window inflation), done with the same tensor ops as the reference.

Reference behaviours kept on purpose (tests pin them against fixtures made from the reference itself):
``WindowSegment`` counts ``(L + L % segment) // segment`` segments (none when L + L % segment < segment)
and prepends one extra window to every segment after the first (the frame its temporal MSE pairs with,
see loss.Loss); the last segment runs to the end of the capture.  Divergence: ``BufferSegment.get_segment``
without ``segment`` is a generator that returns before yielding anything in the reference (a ``return
value`` inside a generator, segment_generator.py:73-77); here it yields that one batch.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F


@dataclass
class WindowBatch:
    """Windows [n0, n0 + nw) of W frames over a padded capture (1, C, Lp, V): window n = frames [n, n+W)."""
    capture: torch.Tensor
    n0: int
    nw: int
    W: int

    @property
    def shape(self):
        _, C, _, V = self.capture.shape
        return torch.Size((self.nw, C, self.W, V))

    def size(self, dim=None):
        return self.shape if dim is None else self.shape[dim]

    @property
    def device(self):
        return self.capture.device

    def materialize(self) -> torch.Tensor:
        """The reference's batch tensor (segment_generator.py:143): (nw, C, W, V), contiguous."""
        _, C, _, V = self.capture.shape
        frames = self.capture[:, :, self.n0:self.n0 + self.nw + self.W - 1]
        return frames.unfold(2, self.W, 1).permute(0, 2, 1, 4, 3).contiguous().view(self.nw, C, self.W, V)


def window_segments(S, Lp, L_labels, W, seg):
    """[(startX, endX, startY, endY)] of WindowSegment.get_segment (segment_generator.py:133-139) for a trial
    of S frames: capture frames [startX, endX) of the padded capture (Lp = S + W - 1 frames) give windows
    startX .. endX - W, predicting label frames [startY, endY).  (S + S % seg) // seg segments; every one
    after the first starts one window early (the frame its temporal MSE pairs with); the last runs to the
    end of the capture."""
    n = (S + S % seg) // seg
    return [(seg * i - (1 if i > 0 else 0), seg * (i + 1) + (W - 1) if i < n - 1 else Lp,
             seg * i, seg * (i + 1) if i < n - 1 else L_labels) for i in range(n)]


class Segment:
    """segment_generator.py:5-15."""

    def __init__(self, rank, world_size, **kwargs):
        self.num_stages = kwargs["stages"]
        self.num_classes = kwargs["num_classes"]
        self.V = kwargs["graph"]["num_node"]
        self.C = kwargs["in_feat"]
        self.rank = rank
        self.world_size = world_size

    def alloc_output(self, L, dtype):
        return torch.zeros(self.num_stages, self.num_classes, L, dtype=dtype, device=self.rank)


class WindowSegment(Segment):
    """segment_generator.py:109-154.  ``staged=False`` yields the materialised tensors instead."""

    def __init__(self, staged=True, **kwargs):
        super().__init__(**kwargs)
        self.W = kwargs["receptive_field"]
        self.subsegment_size = kwargs["segment"]
        self.staged = staged

    def pad_sequence(self, L):
        self.S = L
        return self.W - 1, 0

    def pad_sequence_rt(self, L):
        self.L = L
        return self.W - 1, 0

    def segments(self, Lp, L_labels):
        """[(startX, endX, startY, endY)] of segment_generator.py:133-139 (capture frames / label frames)."""
        return window_segments(self.S, Lp, L_labels, self.W, self.subsegment_size)

    def get_segment(self, captures, labels):
        segs = self.segments(captures.size(2), labels.size(1))
        for sx, ex, sy, ey in segs:
            batch = WindowBatch(captures, sx, ex - sx - (self.W - 1), self.W)
            yield (batch if self.staged else batch.materialize()), labels[:, sy:ey], len(segs)

    def get_segment_rt(self, captures):
        for i in range(self.L):
            yield captures[:, :, i:i + self.W]

    def mask_segment(self, L, P_start, P_end, predictions):
        return predictions.permute(2, 1, 0)  # (N', C', 1) -> (1, C', N')


class BufferSegment(Segment):
    """segment_generator.py:18-106: chunks of ``segment`` frames overlapping by G-1 (G = ``kernel``), or, with
    ``segment`` None, ``world_size`` equal chunks."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.G = kwargs["kernel"]
        self.subsegment_size = kwargs.get("segment")

    def pad_sequence(self, L):
        self.L = L
        G, ws = self.G, self.world_size
        if self.subsegment_size:
            S = self.subsegment_size
            t1 = (L - S) % (S - G)
            t2 = (((L - G - t1) // (S - G)) + 1) % ws
            self.P_end = (0 if t1 == 0 else (S - G - t1)) + (0 if t2 == 0 else (S - G) * (ws - t2))
            return 0, self.P_end
        t = (L - (ws - 1) * (G - 1)) % ws
        P_end = 0 if t == 0 else ws - t
        self.S = ((L + P_end - (ws - 1) * (G - 1)) // ws) + (0 if ws == 1 else G - 1)
        return 0, P_end

    def pad_sequence_rt(self, L):
        self.L = L
        return 0, 0

    def get_segment(self, captures, labels):
        G, ws = self.G, self.world_size
        if self.subsegment_size:
            S = self.subsegment_size
            n = ((self.L + self.P_end - S) // (S - G)) + 1
            data = captures.unfold(2, S, S - G).permute(0, 2, 1, 4, 3).contiguous().view(n, self.C, S, self.V)
            for i in range(0, n, ws):
                start = 0 if i == 0 else S + (S - G) * (i - 1)
                end = S + (S - G) * (i + ws) if i + ws < n - 1 else self.L
                yield data[i:i + ws], labels[:, start:end], n
        else:
            data = captures.unfold(2, self.S, self.S - G).permute(0, 2, 1, 4, 3).contiguous()
            yield data.view(ws, self.C, self.S, self.V), labels, 1

    def get_segment_rt(self, captures):
        for i in range(self.L):
            yield captures[:, :, i:i + 1]

    def mask_segment(self, i, num_segments, L, P_start, P_end, predictions):
        G = self.G
        if self.subsegment_size:
            if i == 0:
                return predictions
            if i < num_segments - 1:
                return predictions[:, :, G - 1:]
            return predictions[:, :, G - 1:-P_end]
        predictions[1:, :, :G] = 0
        p = predictions[None].permute(0, 2, 3, 1).contiguous().view(1, self.num_classes * self.S, self.world_size)
        p = F.fold(p, output_size=(1, L + P_end), kernel_size=(1, self.S), stride=(1, self.S - G))[:, :, 0]
        return p[:, :, :L]
