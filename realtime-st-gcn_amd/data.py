"""Trial loader format: the reference's on-disk layout for variable-length trials and its
directory dataset, restated for the GPU training/inference path.

Layout (data_prep/prep.py:15-45, prep_pkummd): per trial ``<split>/features/<name>.npy`` — float32
(C=3, L, V=25, M=2) — and ``<split>/labels/<name>.csv`` — one class per frame (np.savetxt float text);
``prep_pkummd(dir)`` builds it from the PKU-MMD release (``features/*.txt`` rows of 2 bodies x 25 joints x
xyz, ``labels/*.txt`` rows ``class,start,end,...``, ``cross-view.txt`` train list), like the reference.

``SkeletonDatasetFromDirectory(data_dir, label_dir, f_actions)`` (data_prep/dataset.py:57-131): items are
(data (3, L, 25) float32 — the first body — , labels (L,) int64), ``len``, and ``__get_distribution__(rank)``
the per-class frame counts.  MI355X additions: ``device=`` returns the trial already in HBM (pinned host
staging + a non-blocking copy on the current stream, so the next trial's read overlaps the GPU work), and
the class distribution is counted once at construction with numpy (no per-trial device round trips).
Files are read with loaders that execute nothing (np.load allow_pickle=False, numeric text parsing)."""
from __future__ import annotations

import os

import numpy as np
import torch


def _read_labels(path: str) -> np.ndarray:
    """Per-frame classes from a labels .csv (np.savetxt float text or plain ints), as int64 (dataset.py:112:
    pd.read_csv(header=None).values[:, 0] then np.int64)."""
    v = np.loadtxt(path, delimiter=",", dtype=np.float64, ndmin=2)
    return v[:, 0].astype(np.int64)


def _read_trial(path: str) -> np.ndarray:
    """(3, L, V, M) float .npy -> the first body (3, L, V) float32 (dataset.py:111)."""
    d = np.load(path, allow_pickle=False, mmap_mode="r")
    return np.ascontiguousarray(np.float32(d[:, :, :, 0]))


class SkeletonDatasetFromDirectory(torch.utils.data.Dataset):
    def __init__(self, data_dir, label_dir, f_actions, device=None):
        self.data = data_dir
        self.labels = label_dir
        self.device = torch.device(device) if device is not None else None
        # sorted file stems (dataset.py:89)
        self.dir_list = [f.split(".npy")[0] for f in sorted(os.listdir(self.data))]
        with open(f_actions, "r") as fa:
            actions = fa.read().split("\n")
        # 0th class is always the background action (dataset.py:97-100)
        self.actions = {i + 1: a for i, a in enumerate(actions)}
        self._dist = None

    def __len__(self):
        return len(self.dir_list)

    def __getitem__(self, index):
        name = self.dir_list[index]
        data = _read_trial(os.path.join(self.data, name + ".npy"))
        labels = _read_labels(os.path.join(self.labels, name + ".csv"))
        x, y = torch.from_numpy(data), torch.from_numpy(labels)
        if self.device is not None and self.device.type == "cuda":
            x = x.pin_memory().to(self.device, non_blocking=True)
            y = y.pin_memory().to(self.device, non_blocking=True)
        return x, y

    def __get_distribution__(self, rank):
        """Per-class frame counts over every trial (dataset.py:114-131), float32 on ``rank``."""
        if self._dist is None:
            C = len(self.actions)
            d = np.zeros(C, dtype=np.float64)
            for name in self.dir_list:
                lab = _read_labels(os.path.join(self.labels, name + ".csv"))
                lab = lab[(lab >= 0) & (lab < C)]
                d += np.bincount(lab, minlength=C)[:C]
            self._dist = torch.from_numpy(d.astype(np.float32))
        return self._dist.to(rank)


def prep_pkummd(dir):
    """PKU-MMD release -> the trial layout above (data_prep/prep.py:15-45): features (L, 150) text ->
    (3, L, 25, 2) float32 .npy; labels ``class,start,end,...`` -> per-frame classes (0 = background) .csv;
    split by cross-view.txt (second line split on ", " exactly as prep.py:17 does: no stripping, so an id
    that ends the line keeps its newline, never matches and its trial goes to 'val', as in the reference);
    the source files are removed."""
    with open(os.path.join(dir, "cross-view.txt")) as f:
        train = set(f.readlines()[1].split(", "))
    for split in ("train", "val"):
        for sub in ("features", "labels"):
            os.makedirs(os.path.join(dir, split, sub), exist_ok=True)
    for f_in in sorted(os.listdir(os.path.join(dir, "features"))):
        stem = f_in.split(".")[0]
        feat = np.loadtxt(os.path.join(dir, "features", f_in), dtype=np.float32, ndmin=2)
        feat = np.ascontiguousarray(np.transpose(feat.reshape(feat.shape[0], 2, 25, 3), (3, 0, 2, 1)))
        rows = np.loadtxt(os.path.join(dir, "labels", f_in), delimiter=",", dtype=np.int32, ndmin=2)
        d = np.zeros(feat.shape[1], dtype=np.int32)
        for r in rows:
            d[r[1]:r[2]] = r[0]
        split = "train" if stem in train else "val"
        with open(os.path.join(dir, split, "features", stem + ".npy"), "wb") as fo:
            np.save(fo, feat)
        with open(os.path.join(dir, split, "labels", stem + ".csv"), "w") as fo:
            np.savetxt(fo, d, delimiter=",")
        os.remove(os.path.join(dir, "features", f_in))
        os.remove(os.path.join(dir, "labels", f_in))
