"""Segment metrics kernel (metrics.hip) through the reference-shaped classes (metrics.F1Score, EditScore,
ConfusionMatrix) against the reference's outputs (tests/golden/metrics.npz) bit-exactly, and against the
oracle (oracle/segment_metrics.py, utils/metrics/*.py) on long random trials.  Integer work exact; float
results bit-identical (same float32 operation order)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import segment_metrics as SM

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def M(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg.metrics


def test_metrics_golden(M):
    d = np.load(os.path.join(GOLDEN, "metrics.npz"), allow_pickle=False)
    C, ov, nt = int(d["num_classes"]), d["overlap"].tolist(), int(d["ntrials"])
    f1, ed, cm = M.F1Score(DEV, C, ov), M.EditScore(DEV, C), M.ConfusionMatrix(DEV, C)
    for mtr in (f1, ed, cm):
        mtr.init_metric(nt)
    for i in range(nt):
        lab = torch.from_numpy(d["labels%d" % i])[None].to(DEV)
        pred = torch.from_numpy(d["pred%d" % i])[None].to(DEV)
        for mtr in (f1, ed, cm):
            mtr(lab, pred)
    np.testing.assert_array_equal(f1.value().cpu().numpy(), d["f1"])
    np.testing.assert_array_equal(ed.value().cpu().numpy()[:, 0], d["edit"])
    np.testing.assert_array_equal(cm.value().cpu().numpy(), d["confusion"])
    f1.reduce()
    np.testing.assert_allclose(f1.value().cpu().numpy(), np.nan_to_num(d["f1"]).mean(axis=0), rtol=1e-6)


@pytest.mark.parametrize("L,mean_len,seed", [(6000, 50.0, 1), (20000, 300.0, 2), (513, 3.0, 3), (1, 1.0, 4)])
def test_metrics_vs_oracle(M, L, mean_len, seed):
    rng = np.random.default_rng(seed)
    C = 52
    lab = np.repeat(rng.integers(0, C, L), rng.geometric(1 / mean_len, L))[:L].astype(np.int64)
    pred = lab.copy()
    flip = rng.random(L) < 0.02
    pred[flip] = rng.integers(0, C, int(flip.sum()))
    ov = [0.1, 0.25, 0.5, 0.75]
    cm = torch.zeros(C, C, dtype=torch.int64, device=DEV)
    out, status = M.segment_metrics(torch.from_numpy(lab).to(DEV), torch.from_numpy(pred).to(DEV), ov, C, confusion=cm)
    out = out.cpu().numpy()
    assert int(status.item()) == 0
    np.testing.assert_array_equal(out[:-1], SM.f1(lab, pred, ov))
    if L <= 6000:  # the pure-Python DP oracle is O(m n)
        assert out[-1] == SM.edit(lab, pred)
    np.testing.assert_array_equal(cm.cpu().numpy(), SM.confusion(lab, pred, C))
