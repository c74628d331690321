"""Trial segmentation (realtime-st-gcn_amd/segment.py) against the reference's own WindowSegment and
BufferSegment (utils/segment_generator.py), pinned by tests/golden/segment.npz (made by
tests/golden/make_golden_segment.py from the reference): every yielded batch, label slice and segment count,
and BufferSegment's mask_segment.  The one divergence is pinned explicitly: BufferSegment without
``segment`` yields nothing in the reference (segment_generator.py:73-77) and the intended batch here.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "segment.npz"), allow_pickle=False)
V, C, K = 5, 3, 4


def kw(**extra):
    return dict(rank="cpu", stages=1, num_classes=K, graph={"num_node": V}, in_feat=C, **extra)


def _cases(prefix):
    return sorted({k.split("_")[0] for k in G.files if k.startswith(prefix) and k.endswith("_cfg")})


@pytest.mark.parametrize("case", _cases("w"))
@pytest.mark.parametrize("staged", [True, False])
def test_window_segment_matches_reference(pkg, case, staged):
    L, W, seg, ps, pe, n = (int(v) for v in G[case + "_cfg"])
    cap, lab = torch.from_numpy(G[case + "_cap"]), torch.from_numpy(G[case + "_lab"])
    sg = pkg.segment.WindowSegment(staged=staged, world_size=1, **kw(receptive_field=W, segment=seg))
    assert sg.pad_sequence(L) == (ps, pe)
    out = list(sg.get_segment(F.pad(cap, (0, 0, ps, pe)), lab))
    assert len(out) == n
    for si, (x, y, num) in enumerate(out):
        ref = torch.from_numpy(G["%s_x%d" % (case, si)])
        if staged:
            assert isinstance(x, pkg.segment.WindowBatch) and x.shape == ref.shape
            x = x.materialize()
        assert torch.equal(x, ref)
        assert torch.equal(y, torch.from_numpy(G["%s_y%d" % (case, si)]))
        assert num == int(G["%s_n%d" % (case, si)])
        pred = torch.randn(x.shape[0], K, 1)
        assert torch.equal(sg.mask_segment(L, ps, pe, pred), pred.permute(2, 1, 0))


@pytest.mark.parametrize("case", _cases("b"))
def test_buffer_segment_matches_reference(pkg, case):
    L, Gk, seg, ws, ps, pe, n = (int(v) for v in G[case + "_cfg"])
    cap, lab = torch.from_numpy(G[case + "_cap"]), torch.from_numpy(G[case + "_lab"])
    sg = pkg.segment.BufferSegment(world_size=ws, **kw(kernel=Gk, segment=None if seg < 0 else seg))
    assert sg.pad_sequence(L) == (ps, pe)
    out = list(sg.get_segment(F.pad(cap, (0, 0, ps, pe)), lab))
    if seg < 0:  # divergence: the reference yields nothing here; the intended single batch is yielded
        assert n == 0 and len(out) == 1
        x, y, num = out[0]
        assert x.shape == (ws, C, sg.S, V) and torch.equal(y, lab) and num == 1
        padded = F.pad(cap, (0, 0, ps, pe))
        for r in range(ws):
            s0 = r * (sg.S - Gk)
            assert torch.equal(x[r], padded[0, :, s0:s0 + sg.S])
        return
    assert len(out) == n
    for si, (x, y, num) in enumerate(out):
        assert torch.equal(x, torch.from_numpy(G["%s_x%d" % (case, si)]))
        assert torch.equal(y, torch.from_numpy(G["%s_y%d" % (case, si)]))
        assert num == int(G["%s_n%d" % (case, si)])
        pred = torch.from_numpy(G["%s_p%d" % (case, si)])
        got = sg.mask_segment(si, num, L, ps, pe, pred.clone())
        assert torch.equal(got, torch.from_numpy(G["%s_m%d" % (case, si)]))


def test_window_batch_shape(pkg):
    cap = torch.zeros(1, 3, 70, 25)
    b = pkg.segment.WindowBatch(cap, 4, 17, 50)
    assert b.shape == (17, 3, 50, 25) and b.size(2) == 50 and b.materialize().shape == (17, 3, 50, 25)
