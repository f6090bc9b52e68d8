"""On-device classification metrics for the train.py drop-in.

The reference's train.py builds `torchmetrics.__dict__[name](task="multiclass", num_classes=C)`
(train.py:76-77) and calls `metric(pred_ids, labels)` once per eval repeat (train.py:132-133).
torchmetrics is not installed in this image, so these are restatements of its multiclass
defaults (torchmetrics 1.x: average="macro", top_k=1, multidim_average="global"): per-class
scores from the confusion counts, safe division (0 where a denominator is 0), and the macro mean
over the classes that occur in preds or target.  Parity unpinned (no torchmetrics to compare).

Everything stays on the device: one bincount of target*C + pred gives the confusion matrix.  Under
torch.distributed (one process per GPU) the confusion counts are all-reduced before
the scores are formed, so every rank reports the metric of the global evaluation set.
"""
from __future__ import annotations

import torch


def confusion(preds: torch.Tensor, target: torch.Tensor, num_classes: int) -> torch.Tensor:
    """[C, C] int64 counts, rows = target, columns = prediction."""
    p = preds.reshape(-1).long()
    t = target.reshape(-1).long()
    return torch.bincount(t * num_classes + p, minlength=num_classes * num_classes).view(num_classes, num_classes)


def _stat_scores(preds, target, num_classes, sync=True):
    cm = confusion(preds, target, num_classes)
    if sync:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(cm, op=dist.ReduceOp.SUM)
    cm = cm.double()
    tp = cm.diagonal()
    fp = cm.sum(0) - tp
    fn = cm.sum(1) - tp
    tn = cm.sum() - tp - fp - fn
    return tp, fp, fn, tn


def _sdiv(a, b):
    return torch.where(b > 0, a / b.clamp_min(1e-30), torch.zeros_like(a))


class _Multiclass:
    name = ""

    def __init__(self, task: str = "multiclass", num_classes: int = 2, average: str = "macro", sync: bool = True):
        if task != "multiclass":
            raise ValueError(f"{self.name}: only task='multiclass' is supported")
        if average not in ("macro", "micro"):
            raise ValueError(f"{self.name}: average must be 'macro' or 'micro'")
        self.num_classes, self.average, self.sync = int(num_classes), average, bool(sync)

    def cuda(self):                      # torchmetrics modules are moved with .cuda() (train.py:77)
        return self

    def to(self, *_a, **_k):
        return self

    def score(self, tp, fp, fn, tn):
        raise NotImplementedError

    def __call__(self, preds: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        tp, fp, fn, tn = _stat_scores(preds, target, self.num_classes, self.sync)
        if self.average == "micro":
            return self.score(tp.sum(), fp.sum(), fn.sum(), tn.sum()).float()
        s = self.score(tp, fp, fn, tn)
        present = (tp + fp + fn) > 0
        n = present.sum()
        return torch.where(n > 0, (s * present).sum() / n.clamp_min(1), torch.zeros_like(s.sum())).float()


class Accuracy(_Multiclass):
    name = "Accuracy"

    def score(self, tp, fp, fn, tn):
        return _sdiv(tp, tp + fn)


class Recall(_Multiclass):
    name = "Recall"

    def score(self, tp, fp, fn, tn):
        return _sdiv(tp, tp + fn)


class Precision(_Multiclass):
    name = "Precision"

    def score(self, tp, fp, fn, tn):
        return _sdiv(tp, tp + fp)


class F1Score(_Multiclass):
    name = "F1Score"

    def score(self, tp, fp, fn, tn):
        return _sdiv(2 * tp, 2 * tp + fp + fn)


class Specificity(_Multiclass):
    name = "Specificity"

    def score(self, tp, fp, fn, tn):
        return _sdiv(tn, tn + fp)


METRICS = {c.name: c for c in (Accuracy, Recall, Precision, F1Score, Specificity)}
