"""Pin the CPU oracle (oracle/fusion_oracle.py) against golden vectors produced by running the
reference itself (tests/golden/make_golden.py).  CPU only.

Tolerances: logits/features 2e-5 relative, gradients 1e-4 relative to each tensor's max |g|
(fp32 CPU vs fp32 CPU; differences are summation order and SDPA-vs-eager softmax).
"""
import numpy as np
import pytest
import torch

from goldens import check_grads, det_params, load, rel_err, w_values_dp
from oracle import fusion_oracle as O


def _grads(p):
    return {k: (v.grad if v.grad is not None else None) for k, v in p.items()}


def test_gate_head_cases():
    cfg, fx = load("gate_head")
    p0 = det_params("T", "prigumbel")
    head_p = {k: v for k, v in p0.items() if k.startswith(("fc_layers", "classifier"))}
    for ci, case in enumerate(cfg["cases"]):
        pre = f"c{ci}:"
        hp = {k: v.detach().clone().requires_grad_() for k, v in head_p.items()}
        pooled = torch.from_numpy(fx[pre + "pooled"]).requires_grad_()
        img = torch.from_numpy(fx[pre + "img"]).requires_grad_()
        cross = torch.from_numpy(fx[pre + "cross"]).requires_grad_()
        DP = torch.from_numpy(fx[pre + "DP"]).requires_grad_()
        f = O.minmax(torch.cat((pooled, img, cross), 1))
        g = O.prigumbel_gate(f, DP, torch.from_numpy(fx[pre + "noise"]), torch.from_numpy(fx[pre + "gumbels"]),
                             case["eps"], case["eps_mode"], case["hard"])
        logits = O.head(hp, g)
        loss, _ = O.cal_loss(logits, torch.from_numpy(fx[pre + "labels"]))
        loss.backward()
        assert rel_err(logits.detach(), fx[pre + "logits"]) < 2e-5, ci
        assert abs(loss.item() - float(fx[pre + "loss"])) < 1e-5
        for name, t in (("d_pooled", pooled), ("d_img", img), ("d_cross", cross), ("d_DP", DP)):
            assert rel_err(t.grad, fx[pre + name]) < 1e-4, (ci, name, rel_err(t.grad, fx[pre + name]))
        for n in ("fc_layers.0.bias", "fc_layers.2.bias", "classifier.weight", "classifier.bias"):
            assert rel_err(hp[n].grad.reshape(-1), fx[pre + "gfull:" + n]) < 1e-4, (ci, n)


def test_dp_guarantee():
    cfg, fx = load("dp_guarantee")
    out = O.dp_guarantee(torch.from_numpy(fx["feature"]), torch.from_numpy(fx["row_noise"]), True)
    assert rel_err(out, fx["out"]) < 1e-6


def _window_batch(fx):
    return dict(eeg=torch.from_numpy(fx["eeg"]), act=torch.from_numpy(fx["act"]))


@pytest.mark.parametrize("name", ["full_prigumbel_soft", "full_prigumbel_hard_wvalues"])
def test_full_prigumbel(name):
    cfg, fx = load(name)
    dp = w_values_dp() if cfg["dp"] == "w_values" else None
    p = det_params("W", "prigumbel", dp)
    pc = O.PathConfig(contract="W", variant="prigumbel", eps=cfg["eps"], eps_mode=cfg["eps_mode"], hard=cfg["hard"])
    logits, f, g = O.forward(p, _window_batch(fx), pc, noise=torch.from_numpy(fx["noise"]),
                             gumbels=torch.from_numpy(fx["gumbels"]), return_feature=True)
    loss, _ = O.cal_loss(logits, torch.from_numpy(fx["labels"]))
    loss.backward()
    assert rel_err(f[:, :768].detach(), fx["pooled"]) < 2e-5
    assert rel_err(f[:, 1536:].detach(), fx["cross"]) < 2e-5
    assert rel_err(g.detach(), fx["gated"]) < 2e-5
    assert rel_err(logits.detach(), fx["logits"]) < 2e-5
    check_grads(_grads(p), fx, 1e-4)


def test_full_priconcat():
    cfg, fx = load("full_priconcat")
    p = det_params("W", "priconcat")
    pc = O.PathConfig(contract="W", variant="priconcat", eps=cfg["eps"])
    logits = O.forward(p, _window_batch(fx), pc)
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(fx["labels"]))
    loss.backward()
    assert rel_err(logits.detach(), fx["logits"]) < 2e-5
    check_grads(_grads(p), fx, 1e-4)


def test_full_concat_tokens():
    cfg, fx = load("full_concat_tokens")
    p = det_params("T", "concat")
    pc = O.PathConfig(contract="T", variant="concat")
    batch = {k: torch.from_numpy(fx[k]) for k in ("title_input", "text_mask", "frame_input", "vedio_mask")}
    logits = O.forward(p, batch, pc)
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(fx["labels"]), reduction="sum")
    loss.backward()
    assert rel_err(logits.detach(), fx["logits"]) < 2e-5
    check_grads(_grads(p), fx, 1e-4)
