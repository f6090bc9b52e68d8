"""PriGumbel-v1 (train_val.py:80-158) on the GPU against the reference's own
outputs (tests/golden/prigumbel_v1.npz: its forward and loss_function with the recorded [768, 2]
Gumbel draws and per-row Laplace draws injected), fp32, dropout 0:
  * the drop-in train_val.ConcatModel + train_val.loss_function (autograd across the engine node and
    the caller's torch expression on model.w): logits, loss and every gradient within 1e-4;
  * PriGumbelV1Trainer (fused alpha-scaled CE + eegf_v1_wloss privacy term): the same gradients and
    loss, and the Adam step;
  * Philox draws (no injection): finite, eval-mode masks are hard (straight-through), train-mode soft.
"""
import pytest
import torch

from goldens import check_grads, det_params, load, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(fx, ci):
    pre = f"c{ci}:"
    return {k[len(pre):]: v for k, v in fx.items() if k.startswith(pre)}


def _model(c, f):
    import train_val
    torch.manual_seed(0)
    m = train_val.ConcatModel(c["tau"], c["eps"], contract="W", dropout=0.0)
    p = det_params("W", "prigumbel_v1", requires_grad=False)
    p["w"] = torch.from_numpy(f["w"])
    m.load_state_dict(p, strict=False)
    m = m.cuda()
    m.train(not c["hard"])
    m.engine.injected = dict(v1_gumbels=torch.from_numpy(f["gumbels"]).to(DEV).contiguous(),
                             row_noise=torch.from_numpy(f["row_noise"]).to(DEV))
    return m


@pytest.mark.parametrize("ci", [0, 1, 2])
def test_v1_dropin_matches_reference(ci):
    import train_val
    cfg, fx = load("prigumbel_v1")
    c = cfg["cases"][ci]
    f = _case(fx, ci)
    m = _model(c, f)
    eeg, act = torch.from_numpy(f["eeg"]).to(DEV), torch.from_numpy(f["act"]).to(DEV)
    logits = m(act.unsqueeze(1), torch.ones(2, 1, device=DEV), eeg, torch.ones(2, 256, device=DEV))
    loss, _, _, _ = train_val.loss_function(logits, torch.from_numpy(f["labels"]).to(DEV).view(-1, 1), m, c["alpha"],
                                            c["eps"])
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(logits.detach().cpu(), f["logits"]) < 1e-4
    assert abs(loss.item() - float(f["loss"])) < 1e-4 * abs(float(f["loss"]))
    check_grads({n: q.grad for n, q in m.named_parameters()}, f, 1e-4)


@pytest.mark.parametrize("ci", [0, 2])
def test_v1_trainer_fused_loss(ci):
    from eegfusion.trainer import PriGumbelV1Trainer
    cfg, fx = load("prigumbel_v1")
    c = cfg["cases"][ci]
    f = _case(fx, ci)
    m = _model(c, f)
    eng = m.engine
    tr = PriGumbelV1Trainer(eng, alpha=c["alpha"], lr=1e-5)
    batch = {"eeg": torch.from_numpy(f["eeg"]).to(DEV), "act": torch.from_numpy(f["act"]).to(DEV)}
    w0 = m.w.detach().clone()
    orig_step = tr.opt.step
    grads = {}

    def capture(grad_scale=1.0):
        grads.update({n: eng.G(n).detach().clone() for n in ("w", "fc1.weight", "fc2.bias", "classifier.weight")})
        orig_step(grad_scale)

    tr.opt.step = capture
    loss, _ = tr.step(batch, torch.from_numpy(f["labels"]).to(DEV), training=not c["hard"])
    torch.cuda.synchronize()
    assert abs(float(loss.sum()) - float(f["loss"])) < 1e-4 * abs(float(f["loss"]))
    check_grads(grads, {k: v for k, v in f.items()
                        if k.split(":", 1)[-1] in grads or not k.startswith(("gsum:", "gnone:", "gabs:", "gfull:",
                                                                             "gpos:", "gval:"))}, 1e-4)
    assert not torch.equal(m.w.detach(), w0)


def test_v1_philox_draws():
    import train_val
    torch.manual_seed(3)
    m = train_val.ConcatModel(0.5, 1.0, contract="W", dropout=0.1).cuda()
    eeg = torch.randn(4, 64, 256, device=DEV)
    act = torch.randn(4, 32, device=DEV)
    m.train()
    out = m.forward_window(eeg, act)
    out.sum().backward()
    assert torch.isfinite(out).all() and torch.isfinite(m.w.grad).all() and m.w.grad.abs().sum() > 0
    m.eval()
    with torch.no_grad():
        e = m.forward_window(eeg, act)
    assert torch.isfinite(e).all()
