"""Golden fixtures for trial segmentation (tests/golden/segment.npz) from the REFERENCE's own
utils/segment_generator.py (WindowSegment, BufferSegment), run on the CPU here in the build container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_segment.py

Per case: the seeded capture (1, 3, L, V) and labels (1, L), padded as processor.py:372-374 does, then every
(x, y, num_segments) the reference's get_segment yields, and for BufferSegment the mask_segment output of
seeded predictions per yielded batch.  Small shapes (V=5).  Data only.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REF = os.environ.get("STGCN_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
from utils.segment_generator import BufferSegment, WindowSegment  # noqa: E402  (reference)

V, C, K = 5, 3, 4
WINDOW = [(40, 5, 12), (61, 9, 16), (30, 5, 10), (25, 5, 30), (10, 5, 30), (53, 50, 20)]
BUFFER = [(40, 9, 20, 1), (61, 9, 20, 2), (100, 9, 30, 4), (57, 5, 12, 3), (40, 9, None, 2)]


def kw(**extra):
    return dict(rank="cpu", stages=1, num_classes=K, graph={"num_node": V}, in_feat=C, **extra)


def main():
    g = torch.Generator().manual_seed(17)
    d = {}
    for ci, (L, W, seg) in enumerate(WINDOW):
        cap = torch.randn(1, C, L, V, generator=g)
        lab = torch.randint(0, K, (1, L), generator=g)
        sg = WindowSegment(world_size=1, **kw(receptive_field=W, segment=seg))
        ps, pe = sg.pad_sequence(L)
        padded = F.pad(cap, (0, 0, ps, pe))
        out = list(sg.get_segment(padded, lab))
        d["w%d_cap" % ci], d["w%d_lab" % ci] = cap.numpy(), lab.numpy()
        d["w%d_cfg" % ci] = np.array([L, W, seg, ps, pe, len(out)])
        for si, (x, y, n) in enumerate(out):
            d["w%d_x%d" % (ci, si)], d["w%d_y%d" % (ci, si)] = x.numpy(), y.numpy()
            d["w%d_n%d" % (ci, si)] = np.array(n)
    for ci, (L, G, seg, ws) in enumerate(BUFFER):
        cap = torch.randn(1, C, L, V, generator=g)
        lab = torch.randint(0, K, (1, L), generator=g)
        sg = BufferSegment(world_size=ws, **kw(kernel=G, segment=seg))
        ps, pe = sg.pad_sequence(L)
        padded = F.pad(cap, (0, 0, ps, pe))
        out = list(sg.get_segment(padded, lab))
        d["b%d_cap" % ci], d["b%d_lab" % ci] = cap.numpy(), lab.numpy()
        d["b%d_cfg" % ci] = np.array([L, G, -1 if seg is None else seg, ws, ps, pe, len(out)])
        for si, (x, y, n) in enumerate(out):
            d["b%d_x%d" % (ci, si)], d["b%d_y%d" % (ci, si)] = x.numpy(), y.numpy()
            d["b%d_n%d" % (ci, si)] = np.array(n)
            pred = torch.randn(x.shape[0], K, x.shape[2], generator=g)
            d["b%d_p%d" % (ci, si)] = pred.numpy()
            d["b%d_m%d" % (ci, si)] = sg.mask_segment(si, n, L, ps, pe, pred.clone()).numpy()
    np.savez_compressed(os.path.join(OUT, "segment.npz"), **d)
    print("segment.npz:", {k: v.tolist() for k, v in d.items() if k.endswith("_cfg")})


if __name__ == "__main__":
    main()
