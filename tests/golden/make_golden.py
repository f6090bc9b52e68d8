"""Generate golden vectors by running the REFERENCE itself (survey container only).

Imports the reference's own modules from /root/reference (read-only) — past_acc.py,
main_0430.py, model.py — with the survey's shims:
  * `opacus` stubbed (PrivacyEngine is not on the hot path), `transformers.AdamW` aliased;
  * `BertModel.from_pretrained('bert-base-uncased')` replaced by a local `BertModel(BertConfig())`
    constructor (bert-base geometry, sdpa attention) — no network fetch, weights then overwritten
    with closed-form deterministic values (oracle/detweights.py);
  * contract W: the reference's BERT call receives the EEG window in place of `title_input`; a
    wrapper applies the per-time-step `eeg_encoder` Linear(64,768) and calls the reference BertModel
    with `inputs_embeds=`; `visual_encoder` is Linear(32,768).  Everything downstream (decoder,
    fusion, min-max, Laplace/Gumbel gate, fc head) is the reference's own forward code.
  * dropout p=0 everywhere (the reference's dropout RNG cannot be replayed), Laplace noise
    injected through `model.noiser.sample`, Gumbel draws recorded from the reference's own
    `gumbel_softmax` call (by wrapping `Tensor.exponential_`).
The reference's pickled feature files are NOT loaded (no code-free loader exists for them):
contract-T fixtures use synthetic token ids / CLIP-like vectors of the same shapes.

Outputs: tests/golden/*.npz (inputs, injected draws, outputs, gradient checksums and samples).
Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import math
import sys
import types
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
REF = Path("/root/reference")
sys.path.insert(0, str(ROOT))
from oracle.detweights import det_tensor, sample_positions  # noqa: E402

SEED = 20240501
B_W, C_W, T_W, A_W = 2, 64, 256, 32


def import_reference():
    sys.modules.setdefault("opacus", types.SimpleNamespace(PrivacyEngine=object))
    import transformers
    from transformers import BertConfig, BertModel
    setattr(sys.modules["transformers"], "AdamW", torch.optim.AdamW)

    def _local(cls, name, *a, **k):
        return cls(BertConfig(attn_implementation="sdpa"))

    BertModel.from_pretrained = classmethod(_local)
    sys.path.insert(0, str(REF))
    import main_0430
    import model as ref_model
    import past_acc
    past_acc.device = torch.device("cpu")
    return past_acc, main_0430, ref_model


class WindowBert(nn.Module):
    """Contract W front-end around the reference BertModel."""

    def __init__(self, bert, eeg_encoder):
        super().__init__()
        self.bert = bert
        self.eeg_encoder = eeg_encoder

    def forward(self, input_ids=None, attention_mask=None, return_dict=False):
        emb = self.eeg_encoder(input_ids.transpose(1, 2))
        return self.bert(inputs_embeds=emb, attention_mask=attention_mask, return_dict=return_dict)


def canon(name: str) -> str:
    return name.replace("bert.bert.", "bert.").replace("bert.eeg_encoder.", "eeg_encoder.")


def prepare(m: nn.Module, contract: str, dp=None):
    if contract == "W":
        m.bert = WindowBert(m.bert, nn.Linear(C_W, 768))
        m.visual_encoder = nn.Linear(A_W, 768)
    with torch.no_grad():
        for n, p in m.named_parameters():
            cn = canon(n)
            if cn == "DP":
                p.copy_(torch.as_tensor(dp if dp is not None else np.zeros((1, 2304), np.float32)))
            else:
                p.copy_(torch.from_numpy(det_tensor(SEED, cn, tuple(p.shape))))
    for mod in m.modules():
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
        if isinstance(mod, nn.MultiheadAttention):
            mod.dropout = 0.0
    m.train()
    return m


class InjectedNoise:
    def __init__(self, noise):
        self.noise = noise

    def sample(self, shape):
        return self.noise.clone().view(*shape)


class RecordExp:
    """Records the Exp(1) draws of the reference's own F.gumbel_softmax call."""

    def __enter__(self):
        self.orig = torch.Tensor.exponential_
        self.draws = []
        rec = self

        def exp_(t, *a, **k):
            r = rec.orig(t, *a, **k)
            rec.draws.append(r.detach().clone())
            return r

        torch.Tensor.exponential_ = exp_
        return self

    def __exit__(self, *exc):
        torch.Tensor.exponential_ = self.orig


def grad_record(m):
    out = {}
    for n, p in m.named_parameters():
        cn = canon(n)
        g = p.grad
        if g is None:
            out[f"gnone:{cn}"] = np.array(1)
            continue
        g = g.detach().double().reshape(-1).numpy()
        out[f"gsum:{cn}"] = np.array(g.sum())
        out[f"gabs:{cn}"] = np.array(np.abs(g).sum())
        if g.size <= 4096:
            out[f"gfull:{cn}"] = g.astype(np.float32)
        else:
            pos = sample_positions(cn, g.size)
            out[f"gpos:{cn}"] = pos
            out[f"gval:{cn}"] = g[pos].astype(np.float32)
    return out


def laplace_noise(gen, shape):
    return torch.distributions.laplace.Laplace(torch.tensor([0.0]), torch.tensor([1.0])).sample(shape).view(*shape)


def window_inputs(gen):
    eeg = torch.randn(B_W, C_W, T_W, generator=gen)
    act = torch.randn(B_W, A_W, generator=gen) * 0.5
    return eeg, act


def save(name, cfg, arrays):
    arrays = {k: (v.detach().numpy() if torch.is_tensor(v) else v) for k, v in arrays.items()}
    np.savez_compressed(HERE / f"{name}.npz", config=np.array(json.dumps(cfg)), **arrays)
    print("wrote", name, sum(a.nbytes for a in arrays.values() if hasattr(a, "nbytes")), "bytes")


def w_values_dp():
    w = np.loadtxt(REF / "w_values.txt", delimiter=",", dtype=np.float64).reshape(1, -1)
    return np.log(w / (1 - w)).astype(np.float32)


# --------------------------------------------------------------------------- fixtures
def gen_prigumbel_full(past_acc, hard, tag, dp=None, eps=1.0):
    torch.manual_seed(7)
    gen = torch.Generator().manual_seed(11)
    m = prepare(past_acc.ConcatModel(eps), "W", dp)
    eeg, act = window_inputs(gen)
    frame = act.unsqueeze(1)
    vmask = torch.ones(B_W, 1, dtype=torch.long)
    tmask = torch.ones(B_W, T_W, dtype=torch.long)
    labels = torch.tensor([[1], [0]])
    noise = laplace_noise(gen, (B_W, 2304))
    m.noiser = InjectedNoise(noise)
    feats = {}
    m.fc_layers.register_forward_pre_hook(lambda mod, a: feats.__setitem__("gated", a[0].detach().clone()))
    m.multi_head_decoder.register_forward_hook(lambda mod, a, o: feats.__setitem__("cross", o.detach().permute(1, 0, 2).mean(1)))
    m.bert.register_forward_hook(lambda mod, a, o: feats.__setitem__("pooled", o[1].detach().clone()))
    with RecordExp() as rec:
        logits = m(frame, vmask, eeg, tmask, hard)
    loss, acc, _, _ = past_acc.cal_loss(logits, labels)
    loss.backward()
    gumbels = -torch.log(rec.draws[0])          # [2,B,2304] (the draws the reference used)
    cfg = dict(contract="W", variant="prigumbel", eps=eps, eps_mode="newfrac", hard=bool(hard), seed=SEED,
               B=B_W, C=C_W, T=T_W, A=A_W, dp="w_values" if dp is not None else "zeros")
    save(f"full_prigumbel_{tag}", cfg, dict(eeg=eeg, act=act, labels=labels.view(-1), noise=noise, gumbels=gumbels,
                                             logits=logits.detach(), loss=loss.detach(), pooled=feats["pooled"],
                                             cross=feats["cross"], gated=feats["gated"], **grad_record(m)))


def gen_priconcat_full(main_0430):
    torch.manual_seed(8)
    gen = torch.Generator().manual_seed(12)
    args = types.SimpleNamespace(EPSILON=1.0)
    m = prepare(main_0430.ConcatModel(args, dp_mode="feature_all_lap"), "W")
    eeg, act = window_inputs(gen)
    labels = torch.tensor([0, 1])
    logits = m(act.unsqueeze(1), torch.ones(B_W, 1, dtype=torch.long), eeg, torch.ones(B_W, T_W, dtype=torch.long))
    loss = nn.functional.cross_entropy(logits, labels)
    loss.backward()
    cfg = dict(contract="W", variant="priconcat", eps=1.0, honor_dp_mode=False, seed=SEED, B=B_W, C=C_W, T=T_W, A=A_W)
    save("full_priconcat", cfg, dict(eeg=eeg, act=act, labels=labels, logits=logits.detach(), loss=loss.detach(),
                                     **grad_record(m)))


def gen_concat_tokens(ref_model):
    """model.py ConcatModel (contract T, L=512) — C1's model on synthetic token ids."""
    torch.manual_seed(9)
    gen = torch.Generator().manual_seed(13)
    m = prepare(ref_model.ConcatModel(), "T")
    B, L = 2, 512
    lens = [51, 37]
    ids = torch.zeros(B, L, dtype=torch.long)
    mask = torch.zeros(B, L, dtype=torch.long)
    for b, n in enumerate(lens):
        body = torch.randint(1000, 1030, (n - 2,), generator=gen)
        ids[b, :n] = torch.cat([torch.tensor([101]), body, torch.tensor([102])])
        mask[b, :n] = 1
    frame = torch.randn(B, 1, 512, generator=gen) * 0.5
    vmask = torch.ones(B, 1, dtype=torch.long)
    labels = torch.tensor([1, 0])
    logits = m((frame, vmask, ids, mask), hard=True)
    loss = nn.CrossEntropyLoss(reduction="none")(logits, labels).sum()     # train.py:69,110-111
    loss.backward()
    cfg = dict(contract="T", variant="concat", seed=SEED, B=B, L=L)
    save("full_concat_tokens", cfg, dict(title_input=ids, text_mask=mask, frame_input=frame, vedio_mask=vmask,
                                         labels=labels, logits=logits.detach(), loss=loss.detach(), **grad_record(m)))


class Const(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, *a, **k):
        return self.fn(*a, **k)


def gen_gate_head(past_acc, ref_model, main_0430):
    """Fusion (concat + min-max) + privacy stage + fc head through the reference's own forward,
    with the encoders replaced by leaves (B=4).  One case per (eps, hard, DP init)."""
    gen = torch.Generator().manual_seed(21)
    B = 4
    cases = [("zeros", 1.0, False), ("zeros", 1.0, True), ("w_values", 0.1, False), ("w_values", 1.0, True),
             ("w_values", 3.0, False), ("w_values", 5.0, True), ("w_values", 10.0, False), ("w_values", 10.0, True)]
    out = {}
    for ci, (dpname, eps, hard) in enumerate(cases):
        pooled = (torch.randn(B, 768, generator=gen) * 0.5).requires_grad_()
        img = (torch.randn(B, 1, 768, generator=gen) * 0.5).requires_grad_()
        cross = (torch.randn(1, B, 768, generator=gen) * 0.5).requires_grad_()
        m = past_acc.ConcatModel(eps)
        prepare(m, "T", w_values_dp() if dpname == "w_values" else None)
        m.bert = Const(lambda **k: (torch.zeros(B, 1, 768), pooled))
        m.visual_encoder = Const(lambda x: img)
        m.multi_head_decoder = Const(lambda **k: cross)
        noise = laplace_noise(gen, (B, 2304))
        m.noiser = InjectedNoise(noise)
        labels = torch.randint(0, 2, (B,), generator=gen)
        with RecordExp() as rec:
            logits = m(None, torch.ones(B, 1), None, None, hard)
        loss, _, _, _ = past_acc.cal_loss(logits, labels.view(-1, 1))
        loss.backward()
        pre = f"c{ci}:"
        out.update({pre + "pooled": pooled.detach(), pre + "img": img.detach().squeeze(1),
                    pre + "cross": cross.detach().squeeze(0), pre + "noise": noise,
                    pre + "gumbels": -torch.log(rec.draws[0]), pre + "labels": labels,
                    pre + "DP": m.DP.detach().clone(), pre + "logits": logits.detach(), pre + "loss": loss.detach(),
                    pre + "d_pooled": pooled.grad, pre + "d_img": img.grad.squeeze(1), pre + "d_cross": cross.grad.squeeze(0),
                    pre + "d_DP": m.DP.grad.clone()})
        for n in ("fc_layers.0.weight", "fc_layers.2.weight"):
            g = dict(m.named_parameters())[n].grad.reshape(-1).double().numpy()
            out[pre + "gsum:" + n] = np.array(g.sum())
            pos = sample_positions(n, g.size)
            out[pre + "gpos:" + n] = pos
            out[pre + "gval:" + n] = g[pos].astype(np.float32)
        for n in ("fc_layers.0.bias", "fc_layers.2.bias", "classifier.weight", "classifier.bias"):
            out[pre + "gfull:" + n] = dict(m.named_parameters())[n].grad.reshape(-1)
    cfg = dict(cases=[dict(dp=d, eps=e, hard=h, eps_mode="newfrac") for d, e, h in cases], B=B, seed=SEED)
    save("gate_head", cfg, out)

    # PriConcat DP_guarantee('feature_all_lap') (main_0430.py:76-85), called directly.
    f = torch.randn(B, 2304, generator=gen)
    torch.manual_seed(31)
    y = main_0430.DP_guarantee(f.clone(), 1.0, dp_mode="feature_all_lap")
    torch.manual_seed(31)
    row_noise = torch.distributions.laplace.Laplace(torch.tensor([0.0]), torch.tensor([1.0 / 1.0])).sample([B])
    save("dp_guarantee", dict(eps=1.0, B=B), dict(feature=f, out=y, row_noise=row_noise.view(-1)))


def gen_adam_two_optimizer(past_acc):
    """One PriGumbel iteration of past_acc.main2's loop body (:194-212) with the reference's two
    Adam optimizers (lr 1e-6): parameter deltas / lr recorded for DP and the head."""
    torch.manual_seed(10)
    gen = torch.Generator().manual_seed(14)
    m = prepare(past_acc.ConcatModel(1.0), "W", w_values_dp())
    eeg, act = window_inputs(gen)
    frame, vmask, tmask = act.unsqueeze(1), torch.ones(B_W, 1, dtype=torch.long), torch.ones(B_W, T_W, dtype=torch.long)
    labels = torch.tensor([[0], [1]])
    n1, n2 = laplace_noise(gen, (B_W, 2304)), laplace_noise(gen, (B_W, 2304))
    DP_params = [p for n, p in m.named_parameters() if "DP" in n]
    model_params = [p for n, p in m.named_parameters() if "DP" not in n]
    lr = 1e-6
    model_opt, dp_opt = torch.optim.Adam(model_params, lr=lr), torch.optim.Adam(DP_params, lr=lr)
    before = {canon(n): p.detach().clone() for n, p in m.named_parameters()}
    dp_opt.zero_grad()
    m.noiser = InjectedNoise(n1)
    with RecordExp() as r1:
        loss1, _, _, _ = past_acc.cal_loss(m(frame, vmask, eeg, tmask, hard=False), labels)
    loss1.backward()
    dp_opt.step()
    model_opt.zero_grad()
    m.noiser = InjectedNoise(n2)
    with RecordExp() as r2:
        loss2, _, _, _ = past_acc.cal_loss(m(frame, vmask, eeg, tmask, hard=True), labels)
    loss2.backward()
    model_opt.step()
    out = dict(eeg=eeg, act=act, labels=labels.view(-1), noise1=n1, noise2=n2, gumbels1=-torch.log(r1.draws[0]),
               gumbels2=-torch.log(r2.draws[0]), loss1=loss1.detach(), loss2=loss2.detach())
    for n, p in m.named_parameters():
        cn = canon(n)
        if cn in ("DP", "classifier.weight", "classifier.bias", "fc_layers.2.bias", "bert.pooler.dense.bias",
                  "multi_head_decoder.layers.2.norm3.weight"):
            out["delta:" + cn] = ((p.detach() - before[cn]) / lr).reshape(-1)
    save("two_optimizer_step", dict(lr=lr, eps=1.0, seed=SEED, B=B_W, C=C_W, T=T_W, A=A_W, dp="w_values"), out)


def gen_adam_three_iters(past_acc):
    """Three PriGumbel iterations of past_acc.main2's loop body (:194-212) with the reference's two
    Adam optimizers (lr 1e-6).  After the first Adam step delta/lr is no longer ~-sign(g), so the
    deltas of iterations 2-3 check the moment estimates; recorded for DP, the head, one BERT layer's
    Q/K/V/out/FFN matrices (sampled positions) and the decoder's in_proj matrices (sampled)."""
    torch.manual_seed(40)
    gen = torch.Generator().manual_seed(41)
    m = prepare(past_acc.ConcatModel(1.0), "W", w_values_dp())
    eeg, act = window_inputs(gen)
    frame, vmask, tmask = act.unsqueeze(1), torch.ones(B_W, 1, dtype=torch.long), torch.ones(B_W, T_W, dtype=torch.long)
    labels = torch.tensor([[1], [0]])
    lr = 1e-6
    DP_params = [p for n, p in m.named_parameters() if "DP" in n]
    model_params = [p for n, p in m.named_parameters() if "DP" not in n]
    model_opt, dp_opt = torch.optim.Adam(model_params, lr=lr), torch.optim.Adam(DP_params, lr=lr)
    before = {canon(n): p.detach().clone() for n, p in m.named_parameters()}
    out = dict(eeg=eeg, act=act, labels=labels.view(-1))
    for it in range(3):
        n1, n2 = laplace_noise(gen, (B_W, 2304)), laplace_noise(gen, (B_W, 2304))
        dp_opt.zero_grad()
        m.noiser = InjectedNoise(n1)
        with RecordExp() as r1:
            loss1, _, _, _ = past_acc.cal_loss(m(frame, vmask, eeg, tmask, hard=False), labels)
        loss1.backward()
        dp_opt.step()
        model_opt.zero_grad()
        m.noiser = InjectedNoise(n2)
        with RecordExp() as r2:
            loss2, _, _, _ = past_acc.cal_loss(m(frame, vmask, eeg, tmask, hard=True), labels)
        loss2.backward()
        model_opt.step()
        out.update({f"noise1_{it}": n1, f"noise2_{it}": n2, f"gumbels1_{it}": -torch.log(r1.draws[0]),
                    f"gumbels2_{it}": -torch.log(r2.draws[0]), f"loss1_{it}": loss1.detach(),
                    f"loss2_{it}": loss2.detach()})
    full = ("DP", "classifier.weight", "classifier.bias", "fc_layers.2.bias", "bert.pooler.dense.bias",
            "multi_head_decoder.layers.2.norm3.weight", "bert.encoder.layer.5.attention.self.query.bias",
            "bert.encoder.layer.5.output.LayerNorm.weight")
    sampled = tuple(f"bert.encoder.layer.5.{k}" for k in (
        "attention.self.query.weight", "attention.self.key.weight", "attention.self.value.weight",
        "attention.output.dense.weight", "intermediate.dense.weight", "output.dense.weight")) + (
        "multi_head_decoder.layers.0.self_attn.in_proj_weight", "multi_head_decoder.layers.0.multihead_attn.in_proj_weight",
        "eeg_encoder.weight", "fc_layers.0.weight")
    for n, p in m.named_parameters():
        cn = canon(n)
        d = ((p.detach() - before[cn]) / lr).reshape(-1)
        if cn in full:
            out["delta:" + cn] = d
        elif cn in sampled:
            pos = sample_positions(cn, d.numel())
            out["dpos:" + cn] = pos
            out["dval:" + cn] = d[torch.from_numpy(pos)]
    save("three_iterations", dict(lr=lr, eps=1.0, seed=SEED, B=B_W, C=C_W, T=T_W, A=A_W, dp="w_values", iters=3), out)


def gen_priconcat_lap_full(main_0430):
    """PriConcat with DP_guarantee('feature_all_lap') honoured (the build's honor_dp_mode=True, SURVEY
    App. A.2): the reference's ConcatModel.forward (main_0430.py:108-123) with its DP_guarantee call
    routed to dp_mode='feature_all_lap' (main_0430.py:76-85); the per-row Laplace draw is taken under
    a fixed seed and recorded by re-drawing under the same seed."""
    torch.manual_seed(42)
    gen = torch.Generator().manual_seed(43)
    args = types.SimpleNamespace(EPSILON=1.0)
    m = prepare(main_0430.ConcatModel(args, dp_mode="feature_all_lap"), "W")
    eeg, act = window_inputs(gen)
    labels = torch.tensor([1, 0])
    orig = main_0430.DP_guarantee

    def honoured(feature, EPSILON, dp_mode=None):
        torch.manual_seed(77)
        return orig(feature, EPSILON, dp_mode="feature_all_lap")

    main_0430.DP_guarantee = honoured
    try:
        logits = m(act.unsqueeze(1), torch.ones(B_W, 1, dtype=torch.long), eeg, torch.ones(B_W, T_W, dtype=torch.long))
    finally:
        main_0430.DP_guarantee = orig
    torch.manual_seed(77)
    row_noise = torch.distributions.laplace.Laplace(torch.tensor([0.0]), torch.tensor([1.0])).sample([B_W]).view(-1)
    loss = nn.functional.cross_entropy(logits, labels)
    loss.backward()
    cfg = dict(contract="W", variant="priconcat_lap", eps=1.0, honor_dp_mode=True, seed=SEED, B=B_W, C=C_W, T=T_W,
               A=A_W)
    save("full_priconcat_lap", cfg, dict(eeg=eeg, act=act, labels=labels, row_noise=row_noise, logits=logits.detach(),
                                         loss=loss.detach(), **grad_record(m)))


def gen_feawei_features():
    """The live feature pass of the feawei initialisation: past_acc_feawei.ConcatModel.forward
    (:103-124) returns the min-max normalised fused feature; main2 (:127-148) stacks the batches
    into a float64 matrix whose column mean (:156) feeds the DP init.  Two batches of B=2."""
    import past_acc_feawei
    torch.manual_seed(44)
    gen = torch.Generator().manual_seed(45)
    m = prepare(past_acc_feawei.ConcatModel(), "W")
    weight = np.empty((0, 2304))
    out = {}
    for i in range(2):
        eeg, act = window_inputs(gen)
        with torch.no_grad():
            feature = m(act.unsqueeze(1), torch.ones(B_W, 1, dtype=torch.long), eeg,
                        torch.ones(B_W, T_W, dtype=torch.long), hard=False)
        weight = np.vstack((weight, feature.detach().cpu().numpy()))
        out[f"eeg{i}"], out[f"act{i}"] = eeg, act
    out["features"] = weight
    out["mean_values"] = np.mean(weight, axis=0)
    save("feawei_features", dict(contract="W", seed=SEED, B=B_W, batches=2, C=C_W, T=T_W, A=A_W), out)


def gen_prigumbel_v1():
    """PriGumbel-v1 (train_val.py:125-158) through the reference's own forward and loss_function
    (:80-93): Gumbel draws recorded from its F.gumbel_softmax call ([768, 2], one pair per feature),
    the per-row Laplace draws of Lap_noise recorded from Laplace.sample.  w set to a spread of values
    in (0.05, 0.95) (the reference initialises torch.rand(768)).  Cases: train mode (soft mask) and
    eval mode (hard, straight-through), tau 0.5 / 0.01, eps 1, alpha 0.2 (the 'good results' run,
    train_val.py:547-549)."""
    import train_val
    from torch.distributions.laplace import Laplace
    out = {}
    cases = [(0.5, False), (0.01, True), (0.01, False)]
    for ci, (tau, hard) in enumerate(cases):
        torch.manual_seed(50 + ci)
        gen = torch.Generator().manual_seed(60 + ci)
        m = prepare(train_val.ConcatModel(tau, 1.0), "W")
        with torch.no_grad():
            m.w.copy_(torch.from_numpy((0.05 + 0.9 * (np.arange(768) % 97) / 96.0).astype(np.float32)))
        if hard:
            m.eval()
        eeg, act = window_inputs(gen)
        labels = torch.tensor([[1], [0]])
        lap = []
        orig = Laplace.sample

        def rec(self, shape=torch.Size()):
            r = orig(self, shape)
            lap.append(r.detach().clone())
            return r

        Laplace.sample = rec
        try:
            with RecordExp() as re_:
                logits = m(act.unsqueeze(1), torch.ones(B_W, 1, dtype=torch.long), eeg,
                           torch.ones(B_W, T_W, dtype=torch.long))
        finally:
            Laplace.sample = orig
        loss, _, _, _ = train_val.loss_function(logits, labels, m, 0.2, 1.0)
        loss.backward()
        pre = f"c{ci}:"
        out.update({pre + "eeg": eeg, pre + "act": act, pre + "labels": labels.view(-1),
                    pre + "w": m.w.detach().clone(), pre + "gumbels": -torch.log(re_.draws[0]),
                    pre + "row_noise": lap[0].view(-1), pre + "logits": logits.detach(), pre + "loss": loss.detach()})
        out.update({pre + k: v for k, v in grad_record(m).items()})
    save("prigumbel_v1", dict(cases=[dict(tau=t, hard=h, eps=1.0, alpha=0.2) for t, h in cases], contract="W",
                              seed=SEED, B=B_W, C=C_W, T=T_W, A=A_W), out)


def import_custom_models():
    """python/src/custom_models/models.py (opacus stubbed, BertModel.from_pretrained local — the
    shims of import_reference, which must run first)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_custom_models", REF / "python/src/custom_models/models.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def gen_modal_variants():
    """custom_models/models.py:84-272 — TTCA / ITCA / IICA / TISC_LapDropout (and TICA for the same
    inputs) on contract-T style inputs: token ids [B, 128] with real lengths, CLIP-like vectors
    [B, 1, 512]; eps 1.0, soft gate (hard for TISC), injected Laplace noise, recorded Gumbel draws,
    CE mean.  Batch keys follow the engine (title_input / text_mask / frame_input, *2 for the
    second input of the pair)."""
    cm = import_custom_models()
    B, L = 2, 128
    out = {}
    for ci, (modal, cls, hard) in enumerate((("ti", "TICA_LapDropout", False), ("it", "ITCA_LapDropout", False),
                                             ("ii", "IICA_LapDropout", False), ("tt", "TTCA_LapDropout", False),
                                             ("tisc", "TISC_LapDropout", True))):
        torch.manual_seed(30 + ci)
        gen = torch.Generator().manual_seed(40 + ci)
        m = getattr(cm, cls)() if modal == "ii" else getattr(cm, cls)("bert-base-uncased")
        m = prepare(m, "T")
        ids, masks = [], []
        for lens in ([51, 37], [40, 66]):
            i_ = torch.zeros(B, L, dtype=torch.long)
            m_ = torch.zeros(B, L, dtype=torch.long)
            for b, n in enumerate(lens):
                i_[b, :n] = torch.cat([torch.tensor([101]), torch.randint(1000, 1030, (n - 2,), generator=gen),
                                       torch.tensor([102])])
                m_[b, :n] = 1
            ids.append(i_)
            masks.append(m_)
        img = [torch.randn(B, 1, 512, generator=gen) * 0.5 for _ in range(2)]
        one = torch.ones(B, 1, dtype=torch.long)
        labels = torch.tensor([1, 0])
        noise = laplace_noise(gen, (B, 2304))
        m.noiser = InjectedNoise(noise)
        if modal == "ti":
            args, batch = (ids[0], masks[0], img[1], one), dict(title_input=ids[0], text_mask=masks[0], frame_input=img[1])
        elif modal == "it":
            args, batch = (img[0], one, ids[1], masks[1]), dict(title_input=ids[1], text_mask=masks[1], frame_input=img[0])
        elif modal == "ii":
            args, batch = (img[0], one, img[1], one), dict(frame_input=img[0], frame_input2=img[1])
        elif modal == "tt":
            args, batch = (ids[0], masks[0], ids[1], masks[1]), dict(title_input=ids[0], text_mask=masks[0],
                                                                   title_input2=ids[1], text_mask2=masks[1])
        else:
            args, batch = (ids[0], masks[0], img[1], one), dict(title_input=ids[0], text_mask=masks[0], frame_input=img[1])
        with RecordExp() as rec:
            logits = m(*args, 1.0, hard)
        loss = nn.functional.cross_entropy(logits, labels)
        loss.backward()
        pre = f"{modal}:"
        out.update({pre + k: v for k, v in batch.items()})
        out.update({pre + "labels": labels, pre + "noise": noise, pre + "gumbels": -torch.log(rec.draws[0]),
                    pre + "logits": logits.detach(), pre + "loss": loss.detach()})
        out.update({pre + k: v for k, v in grad_record(m).items()})
        print("modal", modal, float(loss))
    save("modal_variants", dict(modals=["ti", "it", "ii", "tt", "tisc"], hard=dict(ti=False, it=False, ii=False, tt=False,
                                                                                  tisc=True),
                                eps=1.0, contract="T", B=B, L=L, seed=SEED), out)


def c1_split(n=64, L=512, seed=70):
    """A synthetic split in the reference's feature formats for configs[0] (train.py -bs 32): token ids
    with real lengths drawn around the measured 33-65 distribution (mean 51.3), CLS/SEP,
    EEG-digit-like ids; CLIP-like vectors (std 0.5); labels ~ Bernoulli(0.66) with two NaN rows
    (data.py:29-32 maps them to 0).  Returned as arrays (the fixture stores these, and the test writes
    the CSV / pickles from them)."""
    g = torch.Generator().manual_seed(seed)
    lens = (torch.randn(n, generator=g) * 7.0 + 51.3).round().clamp(33, 65).long()
    ids = torch.zeros(n, L, dtype=torch.long)
    mask = torch.zeros(n, L, dtype=torch.long)
    for b in range(n):
        k = int(lens[b])
        ids[b, :k] = torch.cat([torch.tensor([101]), torch.randint(1015, 1025, (k - 2,), generator=g),
                                torch.tensor([102])])
        mask[b, :k] = 1
    clip = (torch.randn(n, 512, generator=g) * 0.5).float()
    labels = (torch.rand(n, generator=g) < 0.66).double()
    labels[[5, 40]] = float("nan")
    return ids, mask, clip, labels


def write_split(d: Path, prefix: str, ids, mask, clip, labels):
    """the reference's formats: feature/{prefix}_EEG.csv (an 'EEG' text column + 'label'),
    feature/action/{prefix}_clip_v2.pickle (ndarray [N, 512] f32), feature/EEG/{prefix}_bert.pickle
    (list of BatchEncoding with 1-D 'input_ids' / 'attention_mask' lists)."""
    import pickle

    import pandas as pd
    from transformers import BatchEncoding
    (d / "action").mkdir(parents=True, exist_ok=True)
    (d / "EEG").mkdir(parents=True, exist_ok=True)
    pd.DataFrame({"EEG": [" ".join(map(str, r[r > 0].tolist())) for r in ids],
                  "label": labels.numpy()}).to_csv(d / f"{prefix}_EEG.csv", index=False)
    with open(d / "action" / f"{prefix}_clip_v2.pickle", "wb") as f:
        pickle.dump(clip.numpy(), f)
    enc = [BatchEncoding({"input_ids": ids[i].tolist(), "attention_mask": mask[i].tolist()}) for i in range(len(ids))]
    with open(d / "EEG" / f"{prefix}_bert.pickle", "wb") as f:
        pickle.dump(enc, f)


def gen_c1_batch32(ref_model):
    """configs[0]: model.py ConcatModel under train.py's loss (CrossEntropyLoss(reduction='none'), .sum(),
    train.py:69,110-111) at batch 32, contract T (L = 512 padded token ids).  The split is read back
    through the reference's own data.MultiModalDataset_ti (data.py:7-34) from files in its formats, so
    the loader is pinned too.  Per-sample logits / CE of all 64 samples (batches of 32 in dataset order;
    no op couples samples, so a sample's logits do not depend on its batch), the CE-sum loss and every
    parameter gradient of the first dataset-order batch.  Deterministic weights, dropout p = 0."""
    import tempfile

    import data as ref_data
    torch.manual_seed(71)
    ids, mask, clip, labels = c1_split()
    with tempfile.TemporaryDirectory() as td:
        write_split(Path(td), "train", ids, mask, clip, labels)
        ds = ref_data.MultiModalDataset_ti(f"{td}/train_EEG.csv", f"{td}/action/train_clip_v2.pickle",
                                           f"{td}/EEG/train_bert.pickle")
        items = [ds[i] for i in range(len(ds))]
    m = prepare(ref_model.ConcatModel(), "T")
    crit = nn.CrossEntropyLoss(reduction="none")
    logits_all, ce_all, loss0 = [], [], None
    for b0 in (0, 32):
        (frame, vmask, tids, tmask), lab = torch.utils.data.default_collate(items[b0:b0 + 32])
        lab = lab.view(-1)
        logits = m((frame, vmask, tids, tmask), hard=True)
        ce = crit(logits, lab)
        if b0 == 0:
            loss0 = ce.sum()
            loss0.backward()
        logits_all.append(logits.detach())
        ce_all.append(ce.detach())
    loaded_labels = torch.cat([it[1] for it in items]).view(-1)
    cfg = dict(contract="T", variant="concat", seed=SEED, B=32, N=64, L=512, loss="CE sum (train.py:69,110-111)")
    save("c1_batch32", cfg, dict(title_input=ids, text_mask=mask, frame_input=clip.unsqueeze(1),
                                 labels_csv=labels, labels=loaded_labels, logits_all=torch.cat(logits_all),
                                 ce_all=torch.cat(ce_all), loss=loss0.detach(), **grad_record(m)))


if __name__ == "__main__":
    torch.set_num_threads(8)
    past_acc, main_0430, ref_model = import_reference()
    if len(sys.argv) > 1:                       # e.g. `make_golden.py c1_batch32`: only those fixtures
        for name in sys.argv[1:]:
            fn = globals()[f"gen_{name}"]
            fn(ref_model) if name == "c1_batch32" else fn()
        sys.exit(0)
    np.savez_compressed(HERE / "w_values_dp.npz", DP=w_values_dp())
    gen_gate_head(past_acc, ref_model, main_0430)
    gen_prigumbel_full(past_acc, hard=False, tag="soft")
    gen_prigumbel_full(past_acc, hard=True, tag="hard_wvalues", dp=w_values_dp())
    gen_priconcat_full(main_0430)
    gen_concat_tokens(ref_model)
    gen_adam_two_optimizer(past_acc)
    # round 2 (appended so the fixtures above are regenerated bit-identically)
    gen_adam_three_iters(past_acc)
    gen_priconcat_lap_full(main_0430)
    gen_feawei_features()
    gen_prigumbel_v1()
    gen_modal_variants()
    # round 3
    gen_c1_batch32(ref_model)
