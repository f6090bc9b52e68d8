"""configs[0] at its stated size on the HIP path (VERDICT r2 next #1b): ConcatModel at batch 32 over
padded token ids (L = 512) with train.py's CE sum, against the c1_batch32 fixture the reference
produced (tests/golden/make_golden.py gen_c1_batch32), fp32, deterministic weights, dropout 0:

  * the first dataset-order batch through the drop-in model: logits, loss and every recorded
    parameter gradient within 1e-4;
  * train.py itself, `-bs 32`, over a 64-sample split in the reference's file formats: the first
    training step's logits and loss match the reference's logits for the samples that step drew
    (train.py shuffles; the samples are identified by their CLIP vectors), within 1e-4."""
import numpy as np
import pytest
import torch

from c1_split import write_c1_split
from goldens import check_grads, det_params, load, rel_err

pytestmark = pytest.mark.gpu


def _det_concat_model():
    import model as drop_in
    m = drop_in.ConcatModel()
    cfg = m.engine.cfg
    cfg.hidden_dropout = cfg.attn_dropout = cfg.dec_dropout = 0.0      # the fixture runs p = 0
    m.load_state_dict(det_params("T", "concat", requires_grad=False), strict=False)
    return m


def test_c1_first_batch_logits_loss_grads():
    _, fx = load("c1_batch32")
    m = _det_concat_model().cuda().train()
    dev = "cuda"
    sel = slice(0, 32)
    x = (torch.from_numpy(fx["frame_input"][sel]).to(dev), torch.ones(32, 1, dtype=torch.long, device=dev),
         torch.from_numpy(fx["title_input"][sel]).to(dev), torch.from_numpy(fx["text_mask"][sel]).to(dev))
    logits = m(x, hard=True)
    loss = torch.nn.CrossEntropyLoss(reduction="none")(logits, torch.from_numpy(fx["labels"][sel]).to(dev)).sum()
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(logits.detach().cpu(), fx["logits_all"][sel]) < 1e-4
    assert abs(loss.item() - float(fx["loss"])) < 1e-4 * abs(float(fx["loss"]))
    check_grads({n: p.grad for n, p in m.named_parameters()}, fx, 1e-4)


def test_train_py_bs32_first_step(tmp_path, monkeypatch):
    import train
    feat = tmp_path / "feature"
    fx = write_c1_split(feat, "train")
    write_c1_split(feat, "test")
    monkeypatch.chdir(tmp_path)
    seen = []

    def get_model(cfg):
        m = _det_concat_model()
        m.eps = torch.tensor(cfg.eps).cuda()
        m = m.cuda()
        fwd = m.forward

        def capture(x, hard=True):
            out = fwd(x, hard)
            if m.training and not seen:
                seen.append((x[0].detach().cpu().clone(), out.detach().cpu().clone()))
            return out
        m.forward = capture
        return m

    monkeypatch.setattr(train, "get_model", get_model)
    train.set_seed(980616)
    cfg = train.parse_args(["-bs", "32", "-n", "1", "-ne", "1", "--exp", "c1"])
    res = train.main(cfg)
    frames, logits = seen[0]
    assert frames.shape == (32, 1, 512) and logits.shape == (32, 2)
    ref_frames = torch.from_numpy(fx["frame_input"])
    idx = [int(torch.nonzero((ref_frames == f).all(-1).all(-1)).view(-1)[0]) for f in frames]
    assert len(set(idx)) == 32                          # a shuffled batch of 32 distinct samples
    assert idx != list(range(32))                       # train.py's DataLoader(shuffle=True) drew it
    assert rel_err(logits, fx["logits_all"][idx]) < 1e-4
    loss0 = res["train_loss"][0]                        # CrossEntropyLoss(reduction='none') rows
    ref = float(fx["ce_all"][idx].astype(np.float64).sum())
    assert abs(float(loss0.sum()) - ref) < 1e-4 * abs(ref)
    assert len(res["train_loss"]) == 2                  # 64 samples / bs 32
    assert (tmp_path / "experiment" / "c1" / "test" / "results.pth").exists()
