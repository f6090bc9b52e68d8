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


def test_full_priconcat_lap():
    """PriConcat with DP_guarantee('feature_all_lap') honoured (make_golden.gen_priconcat_lap_full)."""
    cfg, fx = load("full_priconcat_lap")
    p = det_params("W", "priconcat")
    pc = O.PathConfig(contract="W", variant="priconcat", eps=cfg["eps"], honor_dp_mode=True)
    logits = O.forward(p, _window_batch(fx), pc, row_noise=torch.from_numpy(fx["row_noise"]))
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(fx["labels"]))
    loss.backward()
    assert rel_err(logits.detach(), fx["logits"]) < 2e-5
    check_grads(_grads(p), fx, 1e-4)


def test_feawei_feature_pass():
    """The live feature pass of past_acc_feawei.py:103-124 (normalised fused features) and the
    float64 column mean of main2's stacked matrix (:141-156)."""
    cfg, fx = load("feawei_features")
    p = det_params("W", "prigumbel")
    pc = O.PathConfig(contract="W", variant="prigumbel")
    feats = []
    with torch.no_grad():
        for i in range(cfg["batches"]):
            pooled, img, cross = O.encoders(p, dict(eeg=torch.from_numpy(fx[f"eeg{i}"]),
                                                    act=torch.from_numpy(fx[f"act{i}"])), pc)
            feats.append(O.minmax(torch.cat((pooled, img, cross), 1)))
    f = torch.cat(feats).double().numpy()
    assert rel_err(f, fx["features"]) < 2e-5
    assert rel_err(f.mean(0), fx["mean_values"]) < 2e-5


def _two_pass_iteration(p, batch, labels, n1, g1, n2, g2, dp_opt, model_opt):
    """past_acc.py:194-212 on the oracle: pass 1 (hard=False) -> DP Adam, pass 2 (hard=True) -> model Adam."""
    dp_opt.zero_grad()
    O.cal_loss(O.forward(p, batch, O.PathConfig(contract="W", variant="prigumbel", hard=False), noise=n1,
                         gumbels=g1), labels)[0].backward()
    dp_opt.step()
    model_opt.zero_grad()
    loss2, _ = O.cal_loss(O.forward(p, batch, O.PathConfig(contract="W", variant="prigumbel", hard=True), noise=n2,
                                    gumbels=g2), labels)
    loss2.backward()
    model_opt.step()
    return loss2


def test_three_iterations():
    """Three two-optimizer iterations: oracle + torch Adam reproduce the reference's parameter deltas."""
    cfg, fx = load("three_iterations")
    p = det_params("W", "prigumbel", w_values_dp())
    before = {k: v.detach().clone() for k, v in p.items()}
    dp_opt = torch.optim.Adam([p["DP"]], lr=cfg["lr"])
    model_opt = torch.optim.Adam([v for k, v in p.items() if k != "DP"], lr=cfg["lr"])
    batch = _window_batch(fx)
    labels = torch.from_numpy(fx["labels"])
    for it in range(cfg["iters"]):
        t = {k: torch.from_numpy(fx[f"{k}_{it}"]) for k in ("noise1", "gumbels1", "noise2", "gumbels2")}
        loss2 = _two_pass_iteration(p, batch, labels, t["noise1"], t["gumbels1"], t["noise2"], t["gumbels2"],
                                    dp_opt, model_opt)
        assert abs(loss2.item() - float(fx[f"loss2_{it}"])) < 1e-5 * max(1.0, abs(float(fx[f"loss2_{it}"])))
    n_checked = 0
    for key in fx:
        if not key.startswith(("delta:", "dval:")):
            continue
        n = key.split(":", 1)[1]
        d = ((p[n].detach() - before[n]) / cfg["lr"]).reshape(-1).numpy()
        if key.startswith("dval:"):
            d = d[fx["dpos:" + n]]
        ref = fx[key]
        big = np.abs(ref) > 0.05
        assert big.any() and np.abs(d[big] - ref[big]).max() < 2e-3, (n, np.abs(d[big] - ref[big]).max())
        n_checked += 1
    assert n_checked >= 16


def _case(fx, ci):
    pre = f"c{ci}:"
    return {k[len(pre):]: v for k, v in fx.items() if k.startswith(pre)}


@pytest.mark.parametrize("ci", [0, 1, 2])
def test_prigumbel_v1(ci):
    """train_val.py PriGumbel-v1: the reference's forward + loss_function with its recorded Gumbel
    ([768, 2]) and per-row Laplace draws (make_golden.gen_prigumbel_v1)."""
    cfg, fx = load("prigumbel_v1")
    c = cfg["cases"][ci]
    f = _case(fx, ci)
    p = det_params("W", "prigumbel_v1")
    with torch.no_grad():
        p["w"].copy_(torch.from_numpy(f["w"]))
    pc = O.PathConfig(contract="W", variant="prigumbel_v1", eps=c["eps"], hard=c["hard"], tau=c["tau"])
    logits = O.forward(p, _window_batch(f), pc, gumbels=torch.from_numpy(f["gumbels"]),
                       row_noise=torch.from_numpy(f["row_noise"]))
    loss = O.loss_v1(logits, torch.from_numpy(f["labels"]), p["w"], c["alpha"], c["eps"])
    loss.backward()
    assert rel_err(logits.detach(), f["logits"]) < 2e-5
    assert abs(loss.item() - float(f["loss"])) < 1e-5
    check_grads(_grads(p), f, 1e-4)


@pytest.mark.parametrize("modal", ["ti", "it", "ii", "tt", "tisc"])
def test_modal_variants(modal):
    """custom_models/models.py TICA/ITCA/IICA/TTCA/TISC_LapDropout (reference-generated fixture):
    the oracle's encoders_modal + PriGumbel gate + head, injected Laplace / Gumbel draws."""
    from goldens import modal_case
    cfg, fx_all = load("modal_variants")
    fx = modal_case(fx_all, modal)
    p = det_params("T", "prigumbel", modal=modal)
    batch = {k: torch.from_numpy(fx[k]) for k in ("title_input", "text_mask", "title_input2", "text_mask2",
                                                  "frame_input", "frame_input2") if k in fx}
    logits = O.forward_modal(p, batch, modal, torch.from_numpy(fx["noise"]), torch.from_numpy(fx["gumbels"]),
                             cfg["eps"], cfg["hard"][modal])
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(fx["labels"]))
    loss.backward()
    assert rel_err(logits.detach(), fx["logits"]) < 2e-5
    check_grads(_grads(p), fx, 1e-4)
