"""custom_models/base_train.py (TrainAndTest, base_train.py:47-553) end to end on the GPU over
feature files in the reference's layout: one epoch of the 'lapacian_dropout' two-optimizer loop for
the TICA ('ti'), TTCA ('tt') and TISC (single_stream) models, and of 'NDP' (TICA_NonPrivate); the
record files and the best-F1 checkpoint.  TICA_NonPrivate (the ConcatModel computation under the
TICA signature, models.py:309-352) is checked against the reference-produced full_concat_tokens
fixture at 1e-4 fp32."""
import pytest
import torch

from custom_split import ACT_COEF, ACT_MODEL, EEG_COEF, EEG_MODEL, write_custom_split
from goldens import check_grads, det_params, load, rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pair,dp_mode,stream", [("ti", "lapacian_dropout", "double_stream"),
                                                 ("tt", "lapacian_dropout", "double_stream"),
                                                 ("ti", "lapacian_dropout", "single_stream"),
                                                 ("ti", "NDP", "double_stream")])
def test_train_and_test_one_epoch(tmp_path, monkeypatch, pair, dp_mode, stream):
    from custom_models.base_train import TrainAndTest
    write_custom_split(tmp_path, n=5)
    monkeypatch.chdir(tmp_path)
    job = TrainAndTest(batch_size=2, epochs=1)
    model = job.train("t", "run/", pair, dp_mode, EEG_MODEL, EEG_COEF, ACT_MODEL, ACT_COEF, stream, 1.0)
    rec = (tmp_path / "logs" / "t" / "run" / "whole_record.txt").read_text()
    assert rec.count("Epochs: 1") == 1 and "f_1 Score" in rec
    assert all(torch.isfinite(q).all() for q in model.parameters())
    has_dp = any(n == "DP" for n, _ in model.named_parameters())
    assert has_dp == (dp_mode == "lapacian_dropout")
    ck = tmp_path / "models" / "custom" / "t" / "run" / "best_f1.pickle"
    if ck.exists():
        sd = torch.load(ck, weights_only=True)
        assert set(sd) == set(model.state_dict())


def test_tica_nonprivate_matches_concat_fixture():
    from custom_models.models import TICA_NonPrivate
    _, fx = load("full_concat_tokens")
    torch.manual_seed(0)
    m = TICA_NonPrivate("bert-base-uncased", dropout=0.0)
    p = det_params("T", "concat", requires_grad=False)
    p.pop("DP", None)
    m.load_state_dict(p, strict=False)
    m = m.cuda().train()
    dev = "cuda"
    logits = m(torch.from_numpy(fx["title_input"]).to(dev), torch.from_numpy(fx["text_mask"]).to(dev),
               torch.from_numpy(fx["frame_input"]).to(dev), torch.from_numpy(fx["vedio_mask"]).to(dev))
    loss = torch.nn.CrossEntropyLoss(reduction="none")(logits, torch.from_numpy(fx["labels"]).to(dev)).sum()
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(logits.detach().cpu(), fx["logits"]) < 1e-4
    check_grads({n: q.grad for n, q in m.named_parameters()}, fx, 1e-4, skip=("DP",))
