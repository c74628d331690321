"""Golden fixtures for the segment metrics (tests/golden/metrics.npz) from the REFERENCE's own classes
(utils/metrics/f1.py, edit.py, confusion.py), run on the CPU here in the build container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_metrics.py

Synthetic trials: piecewise-constant ground truth (segments of random class and length) and predictions
derived from it (boundary jitter, relabelled segments, spurious short segments), int64, plus edge cases
(one segment, every frame its own segment, no overlap at all).  Stored per trial: labels, predictions,
F1@{0.1,0.25,0.5} (NaN kept), edit score; and the confusion matrix accumulated over all trials.  Data only.
"""
import os
import sys

import numpy as np
import torch

REF = os.environ.get("STGCN_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
from utils.metrics import ConfusionMatrix, EditScore, F1Score  # noqa: E402  (reference)

C = 52
OVERLAP = [0.1, 0.25, 0.5]


def piecewise(rng, L, mean_len):
    out = np.empty(L, dtype=np.int64)
    t = 0
    while t < L:
        n = max(1, int(rng.exponential(mean_len)))
        out[t:t + n] = rng.integers(0, C)
        t += n
    return out


def noisy(rng, lab):
    p = lab.copy()
    L = len(p)
    edges = np.nonzero(np.diff(lab))[0] + 1
    for e in edges:  # jitter boundaries
        d = int(rng.integers(-5, 6))
        if d > 0:
            p[e:min(L, e + d)] = lab[e - 1]
        elif d < 0:
            p[max(0, e + d):e] = lab[e]
    for _ in range(max(1, L // 150)):  # spurious short segments
        s = int(rng.integers(0, L))
        p[s:s + int(rng.integers(1, 8))] = rng.integers(0, C)
    for e in edges[rng.random(len(edges)) < 0.2]:  # relabelled segments
        p[e:e + int(rng.integers(5, 40))] = rng.integers(0, C)
    return p


def main():
    rng = np.random.default_rng(21)
    trials = []
    for L, m in ((300, 40.0), (1000, 60.0), (2500, 120.0), (777, 15.0), (64, 8.0)):
        lab = piecewise(rng, L, m)
        trials.append((lab, noisy(rng, lab)))
    trials.append((np.full(50, 3, np.int64), np.full(50, 3, np.int64)))                 # one segment, exact
    trials.append((np.arange(40, dtype=np.int64) % C, np.arange(40, dtype=np.int64) % C))  # every frame a segment
    trials.append((np.full(30, 1, np.int64), np.full(30, 2, np.int64)))                 # no correct segment
    f1 = F1Score("cpu", C, OVERLAP)
    ed = EditScore("cpu", C)
    cm = ConfusionMatrix("cpu", C)
    for mtr in (f1, ed, cm):
        mtr.init_metric(len(trials))
    d = {"overlap": np.array(OVERLAP, np.float32), "num_classes": np.array(C)}
    for i, (lab, pred) in enumerate(trials):
        lt, pt = torch.from_numpy(lab)[None], torch.from_numpy(pred)[None]
        f1(lt, pt)
        ed(lt, pt)
        cm(lt, pt)
        d["labels%d" % i], d["pred%d" % i] = lab, pred
    d["f1"] = f1.value().numpy().astype(np.float32)          # [trials][K], NaN kept
    d["edit"] = ed.value().numpy()[:, 0].astype(np.float32)  # [trials]
    d["confusion"] = cm.value().numpy()                       # [C pred][C label] int64
    d["ntrials"] = np.array(len(trials))
    np.savez_compressed(os.path.join(OUT, "metrics.npz"), **d)
    print("metrics.npz:", len(trials), "trials; f1", d["f1"].tolist(), "edit", d["edit"].tolist())


if __name__ == "__main__":
    main()
