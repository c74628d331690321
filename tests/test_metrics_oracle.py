"""The segment-metrics oracle (oracle/segment_metrics.py) against the reference's own outputs
(tests/golden/metrics.npz, tests/golden/make_golden_metrics.py): F1@{0.1,0.25,0.5} incl. NaN trials, edit
score, accumulated confusion matrix — bit-exact."""
import os

import numpy as np

from conftest import GOLDEN
from oracle import segment_metrics as SM


def _golden():
    return np.load(os.path.join(GOLDEN, "metrics.npz"), allow_pickle=False)


def test_metrics_oracle_golden():
    d = _golden()
    C, ov = int(d["num_classes"]), d["overlap"]
    cm = np.zeros((C, C), dtype=np.int64)
    for i in range(int(d["ntrials"])):
        lab, pred = d["labels%d" % i], d["pred%d" % i]
        np.testing.assert_array_equal(SM.f1(lab, pred, ov), d["f1"][i])  # NaN == NaN here
        assert SM.edit(lab, pred) == d["edit"][i]
        SM.confusion(lab, pred, C, cm)
    np.testing.assert_array_equal(cm, d["confusion"])
