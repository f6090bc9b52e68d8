"""Training-mode parity WITH dropout (p = 0.1 at every reference site) — HIP engine vs the CPU oracle.

The oracle (oracle/fusion_oracle.py) runs the reference computation with its dropout sites routed
through a replay hook that applies the HIP path's own Philox masks (tests/philox_ref.py, pinned to
the Random123 known-answer vectors by test_philox_cpu.py).  Everything else — weights, EEG/action
inputs, Laplace/Gumbel draws — is the golden fixture the reference produced.  Tolerance: logits and
every parameter gradient within 1e-4 relative to that tensor's max |value| (fp32 compute).

Engine element/offset conventions per site (engine.py; R = the forward's rng base):
  emb R+1 | attn_out R+10+3i | ffn_out R+11+3i | attn_probs R+12+3i (attention stream)
  dec_sa R+100+8d | dec_ca R+101+8d | dec_ff R+102+8d | dec_sa_w R+103+8d | dec_ca_probs R+104+8d |
  dec_ff_inner R+105+8d; element = row-major flat index of the dropped tensor (attn_probs: the
  [B, H, L, L] numbering of philox_ref.attn_probs_mask / attention.hip attn_call).
"""
import numpy as np
import pytest
import torch

from goldens import det_params, load, rel_err
from oracle import fusion_oracle as O
from philox_ref import attn_mask, attn_probs_mask, drop_mask

pytestmark = pytest.mark.gpu

P_DROP = 0.1
R0 = 5 << 12


def replay(seed: int, R: int, p: float):
    def fn(site, x):
        kind = site[0]
        i = site[1] if len(site) > 1 else 0
        off, stream = {
            # LayerNorm-fused sites (emb, attn_out, ffn_out, dec_sa/ca/ff) draw from the Philox-7
            # 16-bit stream shared with the attention probabilities (layernorm.hip ln_keep)
            "emb": (R + 1, attn_mask), "attn_out": (R + 10 + 3 * i, attn_mask),
            "ffn_out": (R + 11 + 3 * i, attn_mask), "attn_probs": (R + 12 + 3 * i, "probs"),
            "dec_sa": (R + 100 + 8 * i, attn_mask), "dec_ca": (R + 101 + 8 * i, attn_mask),
            "dec_ff": (R + 102 + 8 * i, attn_mask), "dec_sa_w": (R + 103 + 8 * i, drop_mask),
            "dec_ca_probs": (R + 104 + 8 * i, drop_mask), "dec_ff_inner": (R + 105 + 8 * i, drop_mask),
        }[kind]
        e = np.arange(x.numel(), dtype=np.uint64)
        m = attn_probs_mask(seed, off, e, p, x.shape[-1]) if stream == "probs" else stream(seed, off, e, p)
        return x * torch.from_numpy(m).view(x.shape).to(x.dtype)
    return fn


@pytest.mark.parametrize("hard", [False, True])
def test_prigumbel_training_with_dropout_matches_oracle(hard):
    from eegfusion.modules import PriGumbelModel
    cfg, fx = load("full_prigumbel_soft")
    torch.manual_seed(0)
    m = PriGumbelModel(cfg["eps"], contract="W", dropout=P_DROP)
    p = det_params("W", "prigumbel", None, requires_grad=False)
    m.load_state_dict(p, strict=False)
    m = m.cuda().train()
    dev = "cuda"
    noise, gumbels = torch.from_numpy(fx["noise"]), torch.from_numpy(fx["gumbels"])
    m.engine.injected = dict(noise=noise.to(dev), gumbels=gumbels.to(dev).contiguous())
    eeg, act, labels = (torch.from_numpy(fx[k]) for k in ("eeg", "act", "labels"))
    m.engine.rng_counter = R0
    logits = m.forward_window(eeg.to(dev), act.to(dev), hard)
    torch.nn.functional.cross_entropy(logits, labels.to(dev)).backward()
    torch.cuda.synchronize()

    pr = det_params("W", "prigumbel", None, requires_grad=True)
    O.set_dropout_replay(replay(m.engine.cfg.seed, R0, P_DROP))
    try:
        ref = O.forward(pr, dict(eeg=eeg, act=act), O.PathConfig(contract="W", variant="prigumbel", eps=cfg["eps"],
                                                                 hard=hard), noise=noise, gumbels=gumbels)
    finally:
        O.set_dropout_replay(None)
    torch.nn.functional.cross_entropy(ref, labels).backward()

    # dropout is really on: the result differs from the p = 0 golden logits
    assert rel_err(ref.detach(), fx["logits"]) > 1e-3 or hard
    assert rel_err(logits.detach().cpu(), ref.detach()) < 1e-4
    grads = dict(m.named_parameters())
    bad = []
    for n, t in pr.items():
        if t.grad is None or n not in grads:
            continue
        g = grads[n].grad
        gref = t.grad
        if float(gref.abs().max()) == 0.0:
            assert g is None or float(g.abs().max()) < 1e-12, n
            continue
        if n.endswith("attention.self.key.bias"):
            # structurally zero (softmax is shift-invariant per query): both sides are rounding noise;
            # bound it against the scale of the sibling query-bias gradient instead
            scale = float(pr[n.replace(".key.", ".query.")].grad.abs().max())
            assert float(g.abs().max()) < 1e-4 * scale and float(gref.abs().max()) < 1e-4 * scale, n
            continue
        e = rel_err(g.detach().cpu(), gref)
        if e > 1e-4:
            bad.append((e, n))
    assert not bad, sorted(bad)[-5:]
