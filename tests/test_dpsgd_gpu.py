"""DP-SGD on the engine (eegfusion/dpsgd.py, csrc/dpsgd.hip) against per-sample gradients of the
CPU oracle (oracle/fusion_oracle.py, pinned to the reference by tests/test_oracle_golden.py):

  * the per-sample gradient norms over the trainable set (ghost norms of the BERT layer's
    token-sequence Linears, LayerNorm / bias column sums, head row norms) and the clipped sum
    sum_b min(1, C / (norm_b + 1e-6)) grad_b, fp32, dropout 0, within 1e-4 relative, for the two
    reference configurations: main_0430.py:143-151 (contract T, padded token ids; layer[-1] +
    fc_layers + classifier) and base_train.py:322-331 (contract W; + pooler + visual_encoder);
  * DPOptimizer: p.grad = (clipped sum + N(0, (sigma C)^2)) / expected batch size — exact with
    sigma = 0, and the noise's mean / std at sigma > 0;
  * main_0430.train end to end: DP-SGD pretrain (Poisson batches, RDP accountant) then the
    fine-tune that loads the pretrain checkpoint with strict=False, on reference-format files.
Per-sample gradients of the oracle come from one autograd pass per sample (torch CPU fp32).
"""
import types

import numpy as np
import pytest
import torch

from goldens import det_params, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"
MAIN_0430 = ("bert.encoder.layer.11.", "fc_layers.", "classifier.")
BASE_TRAIN = ("bert.encoder.layer.11.", "bert.pooler.", "fc_layers.", "visual_encoder.", "classifier.")


def _token_batch(B=3, L=512, seed=5):
    g = torch.Generator().manual_seed(seed)
    lens = [51, 37, 60, 44][:B]
    ids = torch.zeros(B, L, dtype=torch.long)
    mask = torch.zeros(B, L, dtype=torch.long)
    for b, n in enumerate(lens):
        ids[b, :n] = torch.cat([torch.tensor([101]), torch.randint(1000, 1030, (n - 2,), generator=g),
                                torch.tensor([102])])
        mask[b, :n] = 1
    frame = torch.randn(B, 1, 512, generator=g) * 0.5
    labels = torch.tensor([1, 0, 1, 0][:B])
    return dict(title_input=ids, text_mask=mask, frame_input=frame, vedio_mask=torch.ones(B, 1, dtype=torch.long)), labels


def _window_batch(B=3, seed=6):
    g = torch.Generator().manual_seed(seed)
    return dict(eeg=torch.randn(B, 64, 256, generator=g), act=torch.randn(B, 32, generator=g) * 0.5), \
        torch.tensor([0, 1, 1, 0][:B])


def _oracle_per_sample(contract, batch, labels, prefixes):
    """per-sample gradients (of the per-sample CE) of the trainable parameters, oracle fp32"""
    from oracle import fusion_oracle as O
    p = det_params(contract, "priconcat", None, requires_grad=False)
    train = [k for k in p if k.startswith(prefixes)]
    for k in train:
        p[k].requires_grad_()
    pc = O.PathConfig(contract=contract, variant="priconcat")
    B = labels.shape[0]
    grads = []
    for b in range(B):
        sb = {k: v[b:b + 1] for k, v in batch.items()}
        loss = torch.nn.functional.cross_entropy(O.forward(p, sb, pc), labels[b:b + 1])
        grads.append(dict(zip(train, torch.autograd.grad(loss, [p[k] for k in train]))))
    return train, grads


def _zero_by_symmetry(name):
    """attention key biases: softmax shift invariance makes their gradient exactly 0 (the oracle and
    the reference hold fp residue only; tests/goldens.py check_grads treats them the same way)"""
    return name.endswith("attention.self.key.bias")


def _engine_model(contract, prefixes, C, dropout=0.0):
    from eegfusion.dpsgd import GradSampleModule
    from eegfusion.modules import PriConcatModel
    torch.manual_seed(0)
    m = PriConcatModel(types.SimpleNamespace(EPSILON=1.0), contract=contract, dropout=dropout)
    m.load_state_dict(det_params(contract, "priconcat", None, requires_grad=False), strict=False)
    for n, q in m.named_parameters():
        q.requires_grad = n.startswith(prefixes)
    return GradSampleModule(m.cuda().train(), max_grad_norm=C)


# LayerNorm gammas trainable with their betas frozen (the beta term must not enter the norm)
GAMMA_ONLY = ("bert.encoder.layer.11.attention.output.LayerNorm.weight", "bert.encoder.layer.11.output.LayerNorm.weight",
              "fc_layers.", "classifier.")


@pytest.mark.parametrize("cfg", ["main_0430_T", "base_train_W", "gamma_only_W"])
def test_per_sample_norms_and_clipped_sum(cfg):
    contract, prefixes = {"main_0430_T": ("T", MAIN_0430), "base_train_W": ("W", BASE_TRAIN),
                          "gamma_only_W": ("W", GAMMA_ONLY)}[cfg]
    batch, labels = _token_batch() if contract == "T" else _window_batch()
    train, grads = _oracle_per_sample(contract, batch, labels, prefixes)
    norms = torch.stack([torch.sqrt(sum((g[k].double() ** 2).sum() for k in train)) for g in grads])
    C = float(norms.median())                        # one sample clipped, one not, one at the edge
    clip = (C / (norms + 1e-6)).clamp(max=1.0)
    ref_sum = {k: sum(clip[b] * grads[b][k].double() for b in range(len(grads))) for k in train}

    wm = _engine_model(contract, prefixes, C)
    dev_batch = {k: v.to(DEV) for k, v in batch.items()}
    if contract == "T":
        logits = wm(dev_batch["frame_input"], dev_batch["vedio_mask"], dev_batch["title_input"], dev_batch["text_mask"])
    else:
        logits = wm._module.forward_window(dev_batch["eeg"], dev_batch["act"], True)
    torch.nn.functional.cross_entropy(logits, labels.to(DEV)).backward()
    torch.cuda.synchronize()
    psn = wm._module._dp["last_norms"].double().cpu()
    assert rel_err(psn.sqrt(), norms) < 1e-4, (psn.sqrt(), norms)
    assert rel_err(wm._module._dp["last_clip"].cpu(), clip) < 1e-4
    named = dict(wm._module.named_parameters())
    assert set(train) == {n for n, q in named.items() if q.requires_grad}
    bad = [(k, rel_err(named[k].grad.cpu(), ref_sum[k])) for k in train
           if not _zero_by_symmetry(k) and rel_err(named[k].grad.cpu(), ref_sum[k]) > 1e-4]
    assert not bad, bad[:5]
    assert all(named[k].grad.abs().max() < 1e-6 for k in train if _zero_by_symmetry(k))
    frozen = [n for n, q in named.items() if not q.requires_grad and q.grad is not None]
    assert not frozen, frozen[:3]


def test_private_backward_with_dropout():
    """The reference pretrain runs in train mode with dropout 0.1 (main_0430.py:176-187): the norm pass
    and the clipped-sum pass must replay the same hidden / attention dropout masks.  With C huge
    (clip = 1) the private gradient is the sum of the per-sample gradients; those are rebuilt by
    ordinary engine backwards of one sample's CE over the same forward (the same Philox offset,
    so the same masks), and the per-sample norms must match them, fp32 at 1e-4."""
    batch, labels = _window_batch()
    wm = _engine_model("W", BASE_TRAIN, 1e9, dropout=0.1)
    m = wm._module
    eeg, act, lab = batch["eeg"].to(DEV), batch["act"].to(DEV), labels.to(DEV)
    r0 = m.engine.rng_counter
    torch.nn.functional.cross_entropy(m.forward_window(eeg, act, True), lab).backward()
    torch.cuda.synchronize()
    named = dict(m.named_parameters())
    train = [n for n, q in named.items() if q.requires_grad]
    priv = {k: named[k].grad.detach().double().cpu().clone() for k in train}
    psn = m._dp["last_norms"].double().cpu().clone()
    dp_state, m._dp = m._dp, None
    per = []
    try:
        for b in range(labels.shape[0]):
            for q in m.parameters():
                q.grad = None
            m.engine.rng_counter = r0
            logits = m.forward_window(eeg, act, True)
            torch.nn.functional.cross_entropy(logits[b:b + 1], lab[b:b + 1]).backward()
            torch.cuda.synchronize()
            per.append({k: named[k].grad.detach().double().cpu().clone() for k in train})
    finally:
        m._dp = dp_state
    norms = torch.stack([sum((g[k] ** 2).sum() for k in train if not _zero_by_symmetry(k)) for g in per])
    assert rel_err(psn, norms) < 1e-4, (psn, norms)
    bad = [(k, rel_err(priv[k], sum(g[k] for g in per))) for k in train if not _zero_by_symmetry(k)]
    bad = [x for x in bad if x[1] > 1e-4]
    assert not bad, bad[:5]


@pytest.mark.parametrize("cls", ["IICA_LapDropout", "TISC_LapDropout"])
def test_shared_visual_encoder_refused(cls):
    """visual_encoder reached from two sites (IICA: both image tokens; TISC: the action token and the
    encoder input) cannot take the per-site norm sum: the norm pass must refuse, not under-clip."""
    from eegfusion import modules
    from eegfusion.dpsgd import GradSampleModule
    torch.manual_seed(0)
    m = getattr(modules, cls)(dropout=0.0)
    for n, q in m.named_parameters():
        q.requires_grad = n.startswith(("visual_encoder.", "fc_layers.", "classifier."))
    wm = GradSampleModule(m.cuda().train(), max_grad_norm=1.0)
    g = torch.Generator().manual_seed(3)
    img = [(torch.randn(2, 1, 512, generator=g) * 0.5).to(DEV) for _ in range(2)]
    one = torch.ones(2, 1, dtype=torch.long, device=DEV)
    if cls == "IICA_LapDropout":
        logits = wm(img[0], one, img[1], one, 1.0, False)
    else:
        batch, _ = _token_batch(B=2, L=128)
        logits = wm(batch["title_input"].to(DEV), batch["text_mask"].to(DEV), img[1], one, 1.0, True)
    with pytest.raises(NotImplementedError, match="two sites"):
        torch.nn.functional.cross_entropy(logits, torch.tensor([1, 0], device=DEV)).backward()


def test_dp_optimizer_sigma0_exact_and_noise_statistics():
    from eegfusion.dpsgd import DPOptimizer
    from eegfusion.optim import Adam
    batch, labels = _window_batch()
    train, grads = _oracle_per_sample("W", batch, labels, MAIN_0430)
    norms = torch.stack([torch.sqrt(sum((g[k].double() ** 2).sum() for k in train)) for g in grads])
    C = float(norms.min()) * 0.5                      # every sample clipped
    clip = (C / (norms + 1e-6)).clamp(max=1.0)
    wm = _engine_model("W", MAIN_0430, C)
    params = [q for q in wm.parameters()]
    opt = DPOptimizer(Adam(params, lr=1e-3), noise_multiplier=0.0, max_grad_norm=C, expected_batch_size=4)
    opt.zero_grad()
    logits = wm._module.forward_window(batch["eeg"].to(DEV), batch["act"].to(DEV), True)
    torch.nn.functional.cross_entropy(logits, labels.to(DEV)).backward()
    named = dict(wm._module.named_parameters())
    before = {k: named[k].detach().clone() for k in train}
    opt.step()
    torch.cuda.synchronize()
    for k in train:
        ref = sum(clip[b] * grads[b][k].double() for b in range(3)) / 4
        if _zero_by_symmetry(k):
            assert named[k].grad.abs().max() < 1e-6
            continue
        assert rel_err(named[k].grad.cpu(), ref) < 1e-4, k
        assert not torch.equal(named[k].detach(), before[k])
    # noise: zero gradients, sigma = 2, C = 0.5 -> std sigma C / expected = 0.25 on every element
    opt2 = DPOptimizer(Adam(params, lr=0.0), noise_multiplier=2.0, max_grad_norm=0.5, expected_batch_size=4)
    for k in train:
        named[k].grad.zero_()
    opt2.add_noise_and_scale()
    g = torch.cat([named[k].grad.reshape(-1) for k in train]).double()
    n = g.numel()
    assert n > 7e6
    assert abs(g.mean().item()) < 5 * 0.25 / n ** 0.5
    assert abs(g.std().item() / 0.25 - 1) < 2e-3
    frac = (g.abs() < 0.25).double().mean().item()         # P(|z| < 1) = 0.6827
    assert abs(frac - 0.682689) < 2e-3


def test_main_0430_pretrain_then_finetune(tmp_path, monkeypatch):
    """main_0430.train(pretrain=True) (DP-SGD, Poisson sampling, RDP accounting) then
    train(pretrain=False, load_stat=True) on reference-format feature files."""
    import main_0430
    from eegfusion.dpsgd import PrivacyEngine
    from test_data_cpu import _write_split
    _write_split(tmp_path, n=5)
    ds = main_0430.MultiModalDataset_ti(tmp_path / "x_EEG.csv", tmp_path / "action" / "x_clip_v2.pickle",
                                        tmp_path / "EEG" / "x_bert.pickle")
    args = types.SimpleNamespace(batch_size=2, learning_rate=1e-6, path=str(tmp_path / "run"), EPSILON=3.0,
                                 epochs=2, MAX_GRAD_NORM=0.1)
    torch.manual_seed(1)
    pe = PrivacyEngine()
    model, f1 = main_0430.train(args, ds, ds, main_0430.ConcatModel(args), pretrain=True, privacy_engine=pe)
    steps = 2 * 3                                      # epochs * len(DataLoader(5, bs 2))
    assert len(pe.accountant.history) == 1 and pe.accountant.history[0][2] == steps
    assert 0 < pe.get_epsilon(1 / 3) <= args.EPSILON
    rec = (tmp_path / "run" / "pretrain" / "whole_record.txt").read_text()
    assert rec.count("Epochs:") == 2
    trainable = {n for n, q in model.named_parameters() if q.requires_grad}
    assert trainable and all(n.startswith(("_module.bert.encoder.layer.11.", "_module.fc_layers.",
                                           "_module.classifier.")) for n in trainable)
    ck = tmp_path / "run" / "pretrain" / "best_f1.pickle"
    if ck.exists():                                    # saved only when F1 beat 0.5
        sd = torch.load(ck, weights_only=True)
        assert all(k.startswith("_module.") for k in sd)
    else:
        torch.save(model.state_dict(), ck)
    ft = main_0430.ConcatModel(args, dp_mode="feature_all_lap")
    _, f1b = main_0430.train(args, ds, ds, ft, pretrain=False, load_stat=True)
    assert (tmp_path / "run" / "whole_record.txt").read_text().count("Epochs:") == 2
    assert all(torch.isfinite(q).all() for q in ft.parameters())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("T", [64, 256, 512])
def test_norm_kernels_vs_float64(dt, T):
    """eegf_ghost_norm / eegf_seg_sqnorm / eegf_row_sqnorm against float64 torch on random operands."""
    from eegfusion import _lib
    s = torch.cuda.current_stream().cuda_stream
    code = 0 if dt == torch.float32 else 1
    tol = 1e-4 if dt == torch.float32 else 1e-2
    torch.manual_seed(T)
    S, Dx, Dy = 3, 768, 288
    X = torch.randn(S * T, Dx, device=DEV).to(dt)
    DY = torch.randn(S * T, Dy, device=DEV).to(dt)
    n = _lib.lib().eegf_ghost_norm_workspace(S, T)
    ws = torch.empty(n, device=DEV)
    out = torch.full((S,), 5.0, device=DEV)
    _lib.call("eegf_ghost_norm", code, S, T, Dx, Dy, X.data_ptr(), Dx, DY.data_ptr(), Dy, ws.data_ptr(), n, 1.0,
              out.data_ptr(), s)
    x64, y64 = X.double().view(S, T, Dx), DY.double().view(S, T, Dy)
    ref = torch.einsum("std,stk->sdk", y64, x64).pow(2).sum((1, 2)) + 5.0
    torch.cuda.synchronize()
    assert rel_err(out.cpu(), ref.cpu()) < tol
    # per-sample bias / LayerNorm gamma norms
    xs = torch.randn(S * T, Dy, device=DEV).to(dt)
    mean = torch.randn(S * T, device=DEV)
    rstd = torch.rand(S * T, device=DEV) + 0.5
    out2 = torch.zeros(S, device=DEV)
    _lib.call("eegf_seg_sqnorm", code, S, T, Dy, DY.data_ptr(), Dy, xs.data_ptr(), Dy, mean.data_ptr(),
              rstd.data_ptr(), 1, 0.0, out2.data_ptr(), s)
    xh = (xs.double() - mean.double()[:, None]) * rstd.double()[:, None]
    bias_t = (y64.sum(1) ** 2).sum(1)
    gamma_t = ((DY.double() * xh).view(S, T, Dy).sum(1) ** 2).sum(1)
    torch.cuda.synchronize()
    assert rel_err(out2.cpu(), (bias_t + gamma_t).cpu()) < tol
    # gamma-only (LN bias frozen) and bias-only (no LN statistics) terms
    _lib.call("eegf_seg_sqnorm", code, S, T, Dy, DY.data_ptr(), Dy, xs.data_ptr(), Dy, mean.data_ptr(),
              rstd.data_ptr(), 0, 0.0, out2.data_ptr(), s)
    torch.cuda.synchronize()
    assert rel_err(out2.cpu(), gamma_t.cpu()) < tol
    _lib.call("eegf_seg_sqnorm", code, S, T, Dy, DY.data_ptr(), Dy, None, 0, None, None, 1, 0.0, out2.data_ptr(), s)
    torch.cuda.synchronize()
    assert rel_err(out2.cpu(), bias_t.cpu()) < tol
    # one row per sample
    a = torch.randn(S, 100, device=DEV).to(dt)
    b = torch.randn(S, 40 * T, device=DEV).to(dt)[:, :70]
    out3 = torch.ones(S, device=DEV)
    _lib.call("eegf_row_sqnorm", code, S, 100, a.data_ptr(), 100, 70, b.data_ptr(), 40 * T, out3.data_ptr(), s)
    ref3 = 1 + (a.double() ** 2).sum(1) * (b.double() ** 2).sum(1)
    torch.cuda.synchronize()
    assert rel_err(out3.cpu(), ref3.cpu()) < tol
