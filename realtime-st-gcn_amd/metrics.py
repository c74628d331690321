"""Segment metrics on the GPU (utils/metrics/*.py): ``F1Score(rank, num_classes, overlap)``,
``EditScore(rank, num_classes)``, ``ConfusionMatrix(rank, num_classes)`` keep the reference's interface
(init_metric, __call__(labels, predicted) with (1, L) class tensors, reduce, value, save, log); the
per-trial work is one HIP kernel (metrics.hip: one wave per trial, bit-identical to the reference)."""
from __future__ import annotations

import torch

from . import _lib as L


def segment_metrics(labels, predicted, overlap, num_classes, confusion=None):
    """One trial: returns fp32 [K + 1] on the device (F1@overlap[k] ..., edit); adds the framewise counts
    into ``confusion`` (int64 [C][C], [predicted][label]) when given."""
    lab = labels.reshape(-1)
    pred = predicted.reshape(-1)
    L.require_device(lab)
    dev = lab.device
    if pred.numel() != lab.numel():
        raise RuntimeError(f"stgcn_amd: {pred.numel()} predictions for {lab.numel()} labels")
    lab = lab.to(torch.long).contiguous()
    pred = pred.to(device=dev, dtype=torch.long).contiguous()
    ov = torch.as_tensor(overlap, dtype=torch.float32).reshape(-1).to(dev).contiguous()
    K = ov.numel()
    Lf = lab.numel()
    work = torch.empty(max(1, L.lib().stgcn_segment_metrics_workspace(Lf) // 4), dtype=torch.int32, device=dev)
    out = torch.empty(K + 1, dtype=torch.float32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    if confusion is not None and (confusion.dtype != torch.int64 or not confusion.is_contiguous()):
        raise RuntimeError("stgcn_amd: confusion must be a contiguous int64 [C][C] tensor")
    L.check(L.lib().stgcn_segment_metrics(lab.data_ptr(), pred.data_ptr(), Lf, int(num_classes), ov.data_ptr(), K,
                                          work.data_ptr(), L.ptr(confusion), out.data_ptr(), status.data_ptr(),
                                          L.stream()), "segment_metrics")
    return out, status


class Metric:
    """utils/metrics/metric.py:4-47."""

    def __init__(self, rank, num_classes):
        self.num_classes = num_classes
        self.rank = rank

    def __call__(self):
        self.trial_id += 1

    def init_metric(self, num_trials):
        self.num_trials = num_trials
        self.trial_id = 0

    def value(self):
        return self.metric

    def reduce(self):
        return None


class F1Score(Metric):
    """utils/metrics/f1.py:6-67: per-trial F1@k, macro average over trials (NaN -> 0) in reduce()."""

    def __init__(self, rank, num_classes, overlap):
        super().__init__(rank, num_classes)
        self.overlap = torch.tensor(overlap, device=self.rank, dtype=torch.float32)

    def __call__(self, labels, predicted):
        out, _ = segment_metrics(labels, predicted, self.overlap, self.num_classes)
        self.metric[self.trial_id] = out[:-1]
        super().__call__()

    def init_metric(self, num_trials):
        super().init_metric(num_trials)
        self.metric = torch.zeros(self.num_trials, self.overlap.size(0), device=self.rank, dtype=torch.float32)

    def reduce(self):
        self.metric = self.metric.nan_to_num(0).mean(dim=0)

    def save(self, save_dir, suffix):
        import pandas as pd
        pd.DataFrame(torch.stack((self.overlap, self.metric)).cpu().numpy()).to_csv(
            "{0}/macro-F1@k{1}.csv".format(save_dir, suffix if suffix is not None else ""))

    def log(self):
        return "f1@k = {0}".format(self.metric.cpu().numpy())


class EditScore(Metric):
    """utils/metrics/edit.py:6-51."""

    def __call__(self, labels, predicted):
        out, status = segment_metrics(labels, predicted, [0.5], self.num_classes)
        if int(status.item()) != 0:
            raise RuntimeError("stgcn_amd: edit score supports up to 8192 segments in the shorter sequence")
        self.metric[self.trial_id] = out[-1:]
        super().__call__()

    def init_metric(self, num_trials):
        super().init_metric(num_trials)
        self.metric = torch.zeros(self.num_trials, 1, device=self.rank, dtype=torch.float32)

    def reduce(self):
        self.metric = self.metric.mean(dim=0)

    def save(self, save_dir, suffix):
        import pandas as pd
        pd.DataFrame(data={"edit": self.metric.cpu().numpy()}, index=[0]).to_csv(
            "{0}/edit{1}.csv".format(save_dir, suffix if suffix is not None else ""))

    def log(self):
        return "edit = {0}".format(self.metric.cpu().numpy())


class ConfusionMatrix(Metric):
    """utils/metrics/confusion.py:6-41: framewise counts [predicted][label] accumulated over trials."""

    def __call__(self, labels, predicted):
        for b in range(labels.shape[0]):
            segment_metrics(labels[b], predicted[b], [0.5], self.num_classes, confusion=self.metric)

    def init_metric(self, num_trials):
        super().init_metric(num_trials)
        self.metric = torch.zeros(self.num_classes, self.num_classes, device=self.rank, dtype=torch.int64)

    def save(self, save_dir, suffix):
        import pandas as pd
        pd.DataFrame(self.metric.cpu().numpy()).to_csv(
            "{0}/confusion-matrix{1}.csv".format(save_dir, suffix if suffix is not None else ""))

    def log(self):
        return None
