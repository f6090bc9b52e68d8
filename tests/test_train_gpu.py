"""train.py drop-in end to end on the GPU (SURVEY §8(f) #1, config C1's plumbing): feature files in
the reference's formats (written by this test), get_data -> get_model -> CE(sum) -> Adam for one
epoch, evaluation with repeated forwards, metrics, model.pth / results.pth."""
import types

import pytest
import torch

from test_data_cpu import _write_split

pytestmark = pytest.mark.gpu


def test_train_main_one_epoch(tmp_path, monkeypatch):
    import train
    for split in ("train", "test"):
        _write_split(tmp_path)
        (tmp_path / "x_EEG.csv").rename(tmp_path / f"{split}_EEG.csv")
        (tmp_path / "action" / "x_clip_v2.pickle").rename(tmp_path / "action" / f"{split}_clip_v2.pickle")
        (tmp_path / "EEG" / "x_bert.pickle").rename(tmp_path / "EEG" / f"{split}_bert.pickle")
    (tmp_path / "feature").mkdir()
    for p in list(tmp_path.iterdir()):
        if p.name != "feature":
            p.rename(tmp_path / "feature" / p.name)
    monkeypatch.chdir(tmp_path)
    train.set_seed(980616)
    cfg = train.parse_args(["-bs", "2", "-n", "1", "-ne", "2", "-m", "Accuracy,F1Score", "--exp", "t"])
    res = train.main(cfg)
    out = tmp_path / "experiment" / "t" / "test"
    assert (out / "results.pth").exists() and (out / "info.log").exists()
    saved = torch.load(out / "results.pth", weights_only=True)
    assert saved["pred"].shape == (5, 2) and saved["Accuracy"].shape == (2,) and saved["F1Score"].shape == (2,)
    assert torch.isfinite(saved["train_loss"]).all() and saved["train_loss"].numel() == 5
    assert 0.0 <= float(saved["Accuracy"].mean()) <= 1.0
    assert res["labels"].is_cuda
