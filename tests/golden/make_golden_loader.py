"""Golden fixtures for the trial loader format (tests/golden/loader.npz) from the REFERENCE's own
data_prep/prep.py (prep_pkummd) and data_prep/dataset.py (SkeletonDatasetFromDirectory), run on the CPU here
in the build container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_loader.py

Inputs are synthetic PKU-MMD-shaped raw files, regenerated bit-identically by the tests from what is stored:
per trial the (L, 150) feature matrix (written as text with FMT) and the action rows (class, start, end,
confidence), plus the cross-view train list.  Stored outputs: the .npy arrays prep_pkummd wrote and the
label vectors it wrote (length 3 — prep.py:28 sizes them by features.shape[0] AFTER the (3,L,25,2)
transpose), the split it chose, and — over a directory of full-length label files — every dataset item
(data, labels) and __get_distribution__.  Data only.
"""
import os
import sys
import tempfile

import numpy as np

REF = os.environ.get("STGCN_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
from data_prep.dataset import SkeletonDatasetFromDirectory  # noqa: E402  (reference)
from data_prep.prep import prep_pkummd  # noqa: E402  (reference)

FMT = "%.6f"
NAMES = ["0002-L", "0002-M", "0003-R", "0005-L", "0007-M"]
LENS = [48, 30, 64, 20, 40]
TRAIN = ["0002-L", "0003-R", "0007-M"]
NCLASS = 51  # actions.txt lines; + background


def synth(rng, L):
    """At least two action rows per trial: prep.py:27 np.loadtxt turns a one-row file into a 1-D array
    that its row loop cannot index (the restatement reads ndmin=2 and accepts it)."""
    feat = (rng.standard_normal((L, 150)) * 0.5).astype(np.float32)
    rows = []
    while len(rows) < 2:
        rows, t = [], int(rng.integers(0, 10))
        while t < L - 5:
            n = int(rng.integers(5, 40))
            rows.append((int(rng.integers(1, NCLASS + 1)), t, min(L, t + n), int(rng.integers(0, 2))))
            t += n + int(rng.integers(0, 15))
    return feat, np.array(rows, np.int32)


def write_raw(root, names, feats, rows, train):
    for sub in ("features", "labels", "train/features", "train/labels", "val/features", "val/labels"):
        os.makedirs(os.path.join(root, sub), exist_ok=True)
    for n, f, r in zip(names, feats, rows):
        np.savetxt(os.path.join(root, "features", n + ".txt"), f, fmt=FMT)
        np.savetxt(os.path.join(root, "labels", n + ".txt"), r, fmt="%d", delimiter=",")
    with open(os.path.join(root, "cross-view.txt"), "w") as fo:
        fo.write("Training videos:\n" + ", ".join(train) + ", \nValidataion videos:\n")


def main():
    rng = np.random.default_rng(31)
    feats, rows = zip(*(synth(rng, L) for L in LENS))
    d = {"names": np.array(NAMES), "train": np.array(TRAIN), "fmt": np.array(FMT), "nclass": np.array(NCLASS)}
    for i in range(len(NAMES)):
        d["feat%d" % i], d["rows%d" % i] = feats[i], rows[i]
    with tempfile.TemporaryDirectory() as tmp:
        write_raw(tmp, NAMES, feats, rows, TRAIN)
        prep_pkummd(tmp)
        for i, n in enumerate(NAMES):
            split = "train" if os.path.exists(os.path.join(tmp, "train", "features", n + ".npy")) else "val"
            d["split%d" % i] = np.array(split)
            d["npy%d" % i] = np.load(os.path.join(tmp, split, "features", n + ".npy"), allow_pickle=False)
            d["csv%d" % i] = np.loadtxt(os.path.join(tmp, split, "labels", n + ".csv"), delimiter=",")
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "f"))
        os.makedirs(os.path.join(tmp, "l"))
        for i, n in enumerate(NAMES):  # full-length per-frame labels (the format the loader reads)
            lab = np.zeros(LENS[i], np.int32)
            for r in rows[i]:
                lab[r[1]:r[2]] = r[0]
            d["frames%d" % i] = lab
            np.save(os.path.join(tmp, "f", n + ".npy"), d["npy%d" % i])
            np.savetxt(os.path.join(tmp, "l", n + ".csv"), lab, delimiter=",")
        with open(os.path.join(tmp, "actions.txt"), "w") as fo:
            fo.write("\n".join("action%d" % k for k in range(NCLASS)))
        ds = SkeletonDatasetFromDirectory(os.path.join(tmp, "f"), os.path.join(tmp, "l"),
                                          os.path.join(tmp, "actions.txt"))
        d["len"] = np.array(len(ds))
        for i in range(len(ds)):
            x, y = ds[i]
            d["item_x%d" % i], d["item_y%d" % i] = x.numpy(), y.numpy()
        d["distribution"] = ds.__get_distribution__("cpu").numpy()
    np.savez_compressed(os.path.join(OUT, "loader.npz"), **d)
    print("loader.npz:", len(NAMES), "trials; splits", [str(d["split%d" % i]) for i in range(len(NAMES))],
          "dist sum", float(d["distribution"].sum()))


if __name__ == "__main__":
    main()
