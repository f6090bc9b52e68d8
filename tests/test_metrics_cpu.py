"""eegfusion.metrics (torchmetrics multiclass restatement for the train.py drop-in): known answers
computed by hand from the confusion counts.  torchmetrics itself is absent: parity unpinned."""
import pytest
import torch


def test_known_answers_macro_micro():
    from eegfusion.metrics import METRICS
    preds = torch.tensor([0, 1, 1, 0])
    target = torch.tensor([0, 1, 0, 0])
    # class 0: tp 2, fp 0, fn 1; class 1: tp 1, fp 1, fn 0
    m = {k: float(c(task="multiclass", num_classes=2)(preds, target)) for k, c in METRICS.items()}
    assert m["Accuracy"] == pytest.approx((2 / 3 + 1) / 2)
    assert m["Recall"] == pytest.approx((2 / 3 + 1) / 2)
    assert m["Precision"] == pytest.approx((1 + 0.5) / 2)
    assert m["F1Score"] == pytest.approx((0.8 + 2 / 3) / 2)
    assert m["Specificity"] == pytest.approx((1 / 1 + 2 / 3) / 2)
    acc = METRICS["Accuracy"](task="multiclass", num_classes=2, average="micro")(preds, target)
    assert float(acc) == pytest.approx(0.75)


def test_absent_class_excluded_from_macro():
    from eegfusion.metrics import Accuracy
    # only class 0 appears anywhere among 3 classes: macro over present classes = 1.0
    assert float(Accuracy(num_classes=3)(torch.zeros(4, dtype=torch.long), torch.zeros(4, dtype=torch.long))) == 1.0


def test_train_parse_args_defaults():
    import train
    cfg = train.parse_args([])
    assert (cfg.batch_size, cfg.eps, cfg.n_eval, cfg.n_epochs, cfg.metrics) == (8, 2.0, 5, 50, "Accuracy")
    with pytest.raises(ValueError):
        from eegfusion.metrics import Accuracy
        Accuracy(task="binary")
