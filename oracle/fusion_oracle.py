"""CPU oracle for the EEG+action fusion training path — TEST INFRASTRUCTURE ONLY.

A plain torch fp32 restatement (no `transformers`, no HIP) of the reference computation,
used by tests/, `__graft_entry__.smoke()` and the `cpu_baseline` leg of bench.py as the checker.
Device-agnostic: on CPU tensors it is the golden-pinned oracle; on GPU tensors (plain ATen fp32
ops, TF32 off) the same functions check the production step at full size
(tests/test_fullsize_oracle_gpu.py).
The product path (eeg-multimodal_amd/eegfusion) never imports this module.

Pinned against golden vectors produced by running the reference itself in the survey container
(tests/golden/make_golden.py → tests/golden/*.npz; checked by tests/test_oracle_golden.py).

Follows, line by line:
  * BERT encoder: transformers 5.15.0 `modeling_bert.py` BertEmbeddings :53-106 (word/pos/type +
    LayerNorm 1e-12), BertSelfAttention :139-199 (12 heads x 64, scale 1/8, additive key mask),
    BertSelfOutput :282-293, BertIntermediate/BertOutput :325-351 (GELU-erf), BertPooler :451-462.
  * decoder: torch 2.10 `nn/modules/transformer.py` TransformerDecoderLayer (post-norm, ReLU,
    d_ff 2048, LN 1e-5) :1100-1200 and `F.multi_head_attention_forward` (literal q/k/v form).
  * fusion + privacy: model.py:34-64, past_acc.py:108-139, main_0430.py:76-123,
    python/src/custom_models/models.py:56-82.
  * gumbel_softmax: torch/nn/functional.py gumbel_softmax (soft + straight-through hard).
  * Laplace sampling: torch/distributions/laplace.py:83-86 (u ~ U[eps-1, 1); loc - scale*sign(u)*log1p(-|u|)).
Dropout: p=0 against the reference's golden vectors (its draws come from torch's RNG and cannot be
replayed).  For training-mode parity with dropout on, `set_dropout_replay(fn)` installs a hook called
at every dropout site of the reference — fn(site, x) -> dropout(x) — through which a test replays the
HIP path's Philox masks (tests/test_dropout_parity_gpu.py).  Sites, in reference order:
  ("emb",)               BertEmbeddings.dropout                    modeling_bert.py:107
  ("attn_probs", i)      dropout(attn_weights)                     modeling_bert.py:131
  ("attn_out", i)        BertSelfOutput.dropout                    modeling_bert.py:291
  ("ffn_out", i)         BertOutput.dropout                        modeling_bert.py:349
  ("dec_sa_w", d)        self-attention weight dropout (SDPA dropout_p)   transformer.py:1158-1176
  ("dec_sa", d)          dropout1                                  transformer.py:1174
  ("dec_ca_probs", d)    cross-attention weight dropout            transformer.py:1177-1196
  ("dec_ca", d)          dropout2                                  transformer.py:1194
  ("dec_ff_inner", d)    _ff_block's self.dropout                  transformer.py:1198
  ("dec_ff", d)          dropout3                                  transformer.py:1199
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

HID, NHEAD, DHEAD, FFN, NLAYER = 768, 12, 64, 3072, 12
DEC_FF, DEC_LAYERS = 2048, 3
LN_BERT, LN_DEC = 1e-12, 1e-5
FUSED = 3 * HID


@dataclass
class PathConfig:
    contract: str = "W"          # "W": window (eeg [B,C,T] f32, act [B,32]); "T": token ids (L=512) + CLIP [B,1,512]
    variant: str = "prigumbel"   # "concat" (model.py), "priconcat" (main_0430.py), "prigumbel" (past_acc.py)
    eps: float = 1.0
    eps_mode: str = "newfrac"    # "newfrac": 1/ln((e^eps-w)/(1-w)) (past_acc.py:132); "new": ln(...) (model.py:57)
    hard: bool = False
    honor_dp_mode: bool = False  # PriConcat: apply DP_guarantee('feature_all_lap') (main_0430.py:76-85)
    tau: float = 1.0             # PriGumbel-v1 gumbel_softmax temperature (train_val.py:95)


_DROP = None


def set_dropout_replay(fn) -> None:
    """fn(site: tuple, x: Tensor) -> Tensor, or None for no dropout (the default)."""
    global _DROP
    _DROP = fn


def _drop(site, x):
    return x if _DROP is None else _DROP(site, x)


# ------------------------------------------------------------------------------ BERT (a4)
def _ln(x, w, b, eps):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def _lin(x, p, name):
    return F.linear(x, p[name + ".weight"], p.get(name + ".bias"))


def bert_embeddings(p, *, input_ids=None, inputs_embeds=None):
    """BertEmbeddings.forward (modeling_bert.py:68-106): word|embeds + type[0] + pos, LN 1e-12."""
    pre = "bert.embeddings."
    if inputs_embeds is None:
        inputs_embeds = p[pre + "word_embeddings.weight"][input_ids]
    L = inputs_embeds.shape[1]
    x = inputs_embeds + p[pre + "token_type_embeddings.weight"][0] + p[pre + "position_embeddings.weight"][:L]
    return _drop(("emb",), _ln(x, p[pre + "LayerNorm.weight"], p[pre + "LayerNorm.bias"], LN_BERT))


def bert_layer(p, i, h, key_bias):
    """BertLayer (modeling_bert.py:354-417) with eager attention (:111-136) semantics."""
    pre = f"bert.encoder.layer.{i}."
    B, L, _ = h.shape

    def heads(t):
        return t.view(B, L, NHEAD, DHEAD).transpose(1, 2)

    q = heads(_lin(h, p, pre + "attention.self.query"))
    k = heads(_lin(h, p, pre + "attention.self.key"))
    v = heads(_lin(h, p, pre + "attention.self.value"))
    s = q @ k.transpose(-1, -2) * (DHEAD ** -0.5) + key_bias[:, None, None, :]
    ctx = (_drop(("attn_probs", i), s.softmax(-1)) @ v).transpose(1, 2).reshape(B, L, HID)
    a = _ln(_drop(("attn_out", i), _lin(ctx, p, pre + "attention.output.dense")) + h,
            p[pre + "attention.output.LayerNorm.weight"], p[pre + "attention.output.LayerNorm.bias"], LN_BERT)
    f = F.gelu(_lin(a, p, pre + "intermediate.dense"))
    return _ln(_drop(("ffn_out", i), _lin(f, p, pre + "output.dense")) + a,
               p[pre + "output.LayerNorm.weight"], p[pre + "output.LayerNorm.bias"], LN_BERT)


def bert(p, emb, attention_mask):
    """BertModel.forward (modeling_bert.py:623-686) → (sequence_output, pooled_output)."""
    key_bias = torch.zeros(attention_mask.shape, dtype=emb.dtype, device=emb.device)
    key_bias = key_bias.masked_fill(attention_mask == 0, torch.finfo(emb.dtype).min)
    h = emb
    for i in range(NLAYER):
        h = bert_layer(p, i, h, key_bias)
    pooled = torch.tanh(_lin(h[:, 0], p, "bert.pooler.dense"))
    return h, pooled


# -------------------------------------------------------------------------- decoder (a5)
def mha_literal(x, mem, in_w, in_b, out_w, out_b, key_padding_mask, site=None):
    """F.multi_head_attention_forward, batch-major: x [B,Lq,E], mem [B,S,E]; mask True = ignore."""
    B, Lq, E = x.shape
    S = mem.shape[1]
    wq, wk, wv = in_w.chunk(3)
    bq, bk, bv = in_b.chunk(3)
    q = F.linear(x, wq, bq).view(B, Lq, NHEAD, DHEAD).transpose(1, 2)
    k = F.linear(mem, wk, bk).view(B, S, NHEAD, DHEAD).transpose(1, 2)
    v = F.linear(mem, wv, bv).view(B, S, NHEAD, DHEAD).transpose(1, 2)
    s = (q * DHEAD ** -0.5) @ k.transpose(-1, -2)
    if key_padding_mask is not None:
        s = s.masked_fill(key_padding_mask[:, None, None, :], float("-inf"))
    w = s.softmax(-1)
    if site is not None:
        w = _drop(site, w)
    ctx = (w @ v).transpose(1, 2).reshape(B, Lq, E)
    return F.linear(ctx, out_w, out_b)


def decoder_layer(p, i, x, mem, mem_pad, tgt_pad):
    """TransformerDecoderLayer.forward, norm_first=False (transformer.py:1158-1200)."""
    pre = f"multi_head_decoder.layers.{i}."
    sa = mha_literal(x, x, p[pre + "self_attn.in_proj_weight"], p[pre + "self_attn.in_proj_bias"],
                     p[pre + "self_attn.out_proj.weight"], p[pre + "self_attn.out_proj.bias"], tgt_pad,
                     site=("dec_sa_w", i))
    x = _ln(x + _drop(("dec_sa", i), sa), p[pre + "norm1.weight"], p[pre + "norm1.bias"], LN_DEC)
    ca = mha_literal(x, mem, p[pre + "multihead_attn.in_proj_weight"], p[pre + "multihead_attn.in_proj_bias"],
                     p[pre + "multihead_attn.out_proj.weight"], p[pre + "multihead_attn.out_proj.bias"], mem_pad,
                     site=("dec_ca_probs", i))
    x = _ln(x + _drop(("dec_ca", i), ca), p[pre + "norm2.weight"], p[pre + "norm2.bias"], LN_DEC)
    ff = _lin(_drop(("dec_ff_inner", i), F.relu(_lin(x, p, pre + "linear1"))), p, pre + "linear2")
    return _ln(x + _drop(("dec_ff", i), ff), p[pre + "norm3.weight"], p[pre + "norm3.bias"], LN_DEC)


def decoder(p, tgt, mem, mem_mask, tgt_mask):
    """multi_head_decoder(tgt, memory, tgt_key_padding_mask, memory_key_padding_mask)
    followed by .permute(1,0,2).mean(dim=1) (model.py:40-44).  mem_mask / tgt_mask None: no mask
    (TTCA / IICA call the decoder without masks, models.py:107-108, :196-197)."""
    x = tgt
    for i in range(DEC_LAYERS):
        x = decoder_layer(p, i, x, mem, None if mem_mask is None else mem_mask == 0,
                          None if tgt_mask is None else tgt_mask == 0)
    return x.mean(dim=1)


def encoder_layer(p, i, x):
    """TransformerEncoderLayer.forward, norm_first=False, ReLU, d_ff 2048, LN 1e-5 (torch 2.10
    transformer.py TransformerEncoderLayer; TISC_LapDropout, models.py:227-228): x [B,S,E]."""
    pre = f"multi_head_encoder.layers.{i}."
    sa = mha_literal(x, x, p[pre + "self_attn.in_proj_weight"], p[pre + "self_attn.in_proj_bias"],
                     p[pre + "self_attn.out_proj.weight"], p[pre + "self_attn.out_proj.bias"], None,
                     site=("enc_sa_w", i))
    x = _ln(x + _drop(("enc_sa", i), sa), p[pre + "norm1.weight"], p[pre + "norm1.bias"], LN_DEC)
    ff = _lin(_drop(("enc_ff_inner", i), F.relu(_lin(x, p, pre + "linear1"))), p, pre + "linear2")
    return _ln(x + _drop(("enc_ff", i), ff), p[pre + "norm2.weight"], p[pre + "norm2.bias"], LN_DEC)


# ------------------------------------------ modality variants (custom_models/models.py:84-272)
# Batch keys (the engine's): title_input / text_mask = the first BERT input, title_input2 /
# text_mask2 the second (TTCA), frame_input / frame_input2 the CLIP-vector inputs [B,1,512].
MODALS = ("ti", "it", "ii", "tt", "tisc")


def encoders_modal(p, batch, modal):
    """-> the three fused features in the variant's concat order.
    ti   TICA_LapDropout  (models.py:28-82):   BERT(eeg txt) | visual(act img) | decoder(act img; eeg seq)
    it   ITCA_LapDropout  (models.py:130-175): visual(eeg img) | BERT(act txt) | decoder(eeg img; act seq)
    ii   IICA_LapDropout  (models.py:176-214): visual(eeg img) | visual(act img) | decoder(eeg img; act img)
    tt   TTCA_LapDropout  (models.py:84-129):  BERT(eeg txt) | BERT(act txt) | decoder(act seq; eeg seq), no masks
    tisc TISC_LapDropout  (models.py:215-272): BERT(eeg txt) | visual(act img) | encoder([mean(eeg seq), act img])"""
    if modal == "ti":
        emb = bert_embeddings(p, input_ids=batch["title_input"])
        seq, pooled = bert(p, emb, batch["text_mask"])
        vis = _lin(batch["frame_input"], p, "visual_encoder")
        return pooled, vis.squeeze(1), decoder(p, vis, seq, batch["text_mask"], batch.get("vedio_mask"))
    if modal == "it":
        emb = bert_embeddings(p, input_ids=batch["title_input"])
        seq, pooled = bert(p, emb, batch["text_mask"])
        vis = _lin(batch["frame_input"], p, "visual_encoder")
        return vis.squeeze(1), pooled, decoder(p, vis, seq, batch["text_mask"], batch.get("vedio_mask"))
    if modal == "ii":
        ve = _lin(batch["frame_input"], p, "visual_encoder")
        va = _lin(batch["frame_input2"], p, "visual_encoder")
        return ve.squeeze(1), va.squeeze(1), decoder(p, ve, va, None, None)
    if modal == "tt":
        se, pe = bert(p, bert_embeddings(p, input_ids=batch["title_input"]), batch["text_mask"])
        sa, pa = bert(p, bert_embeddings(p, input_ids=batch["title_input2"]), batch["text_mask2"])
        return pe, pa, decoder(p, sa, se, None, None)
    if modal == "tisc":
        se, pe = bert(p, bert_embeddings(p, input_ids=batch["title_input"]), batch["text_mask"])
        va = _lin(batch["frame_input"], p, "visual_encoder")
        x = torch.cat((se.mean(dim=1).unsqueeze(1), va), dim=1)     # [B, 2, 768] (batch-major)
        for i in range(DEC_LAYERS):
            x = encoder_layer(p, i, x)
        return pe, va.squeeze(1), x.mean(dim=1)
    raise ValueError(modal)


def forward_modal(p, batch, modal, noise, gumbels, eps=1.0, hard=False):
    """the *_LapDropout forward after the encoders (models.py:69-82): min-max, PriGumbel newfrac gate,
    fc head."""
    f = torch.cat(encoders_modal(p, batch, modal), dim=1)
    g = prigumbel_gate(minmax(f), p["DP"], noise, gumbels, eps, "newfrac", hard)
    return head(p, g)


# --------------------------------------------------------------------- fusion + privacy
def minmax(f):
    """Row-wise min-max normalisation, no epsilon (model.py:47-50; past_acc.py:121-123)."""
    fmin = f.min(dim=-1, keepdim=True)[0]
    fmax = f.max(dim=-1, keepdim=True)[0]
    return (f - fmin) / (fmax - fmin)


def eps_hat(w, eps, mode):
    a = torch.tensor(math.exp(eps), dtype=torch.float32)
    r = ((a - w) / (1 - w)).log()
    return 1.0 / r if mode == "newfrac" else r


def gumbel_softmax_injected(logits, gumbels, hard, tau=1.0, dim=0):
    """torch.nn.functional.gumbel_softmax with the -log(Exp(1)) draws supplied."""
    y_soft = ((logits + gumbels) / tau).softmax(dim)
    if not hard:
        return y_soft
    index = y_soft.max(dim, keepdim=True)[1]
    y_hard = torch.zeros_like(logits).scatter_(dim, index, 1.0)
    return y_hard - y_soft.detach() + y_soft


def prigumbel_gate(feature, DP, noise, gumbels, eps, mode, hard):
    """past_acc.py:130-136 / models.py:73-79."""
    w = torch.sigmoid(DP)
    y = feature + noise * eps_hat(w, eps, mode)
    logits = torch.stack((w, 1 - w)).repeat(1, feature.shape[0], 1)
    mask = gumbel_softmax_injected(logits, gumbels, hard)
    return (y * mask).sum(0)


def dp_guarantee(feature, row_noise, honor):
    """main_0430.py:76-85: identity for dp_mode=None (as ConcatModel.forward calls it, :118);
    'feature_all_lap': min-max then one Laplace(0, 1/eps) scalar per row."""
    if not honor:
        return feature
    return minmax(feature) + row_noise.view(-1, 1)


def laplace_from_uniform(u, scale=1.0):
    """torch Laplace.rsample (laplace.py:83-86) given u ~ U[finfo.eps - 1, 1)."""
    return -scale * u.sign() * torch.log1p(-u.abs())


def head(p, f):
    """fc_layers + classifier (model.py:24-32,62-63)."""
    h = torch.relu(_lin(f, p, "fc_layers.0"))
    h = torch.tanh(_lin(h, p, "fc_layers.2"))
    return _lin(h, p, "classifier")


# --------------------------------------------------------------- PriGumbel-v1 (train_val.py)
def gumbel_dropout_v1(x, w, gumbels, tau, hard):
    """train_val.py:95-101: logits [768, 2] = (w, 1 - w) (raw w), F.gumbel_softmax over dim -1 with
    the -log Exp(1) draws [768, 2] supplied; mask = column 1; x * mask / (1 - w)."""
    logits = torch.stack((w, 1 - w), dim=1)
    mask = gumbel_softmax_injected(logits, gumbels, hard, tau=tau, dim=-1)[:, 1]
    return x * mask / (1.0 - w)


def head_v1(p, f, gumbels, row_noise, tau, hard):
    """train_val.py:153-157: relu(fc1) -> fc2 -> gumbel dropout -> Lap_noise (:114-123: row min-max +
    one Laplace(0, 1/eps) draw per row) -> classifier."""
    x = _lin(torch.relu(_lin(f, p, "fc1")), p, "fc2")
    res = gumbel_dropout_v1(x, p["w"], gumbels, tau, hard)
    return _lin(minmax(res) + row_noise.view(-1, 1), p, "classifier")


def loss_v1(logits, labels, w, alpha, eps):
    """train_val.py:80-93: alpha * CE(mean) + max_j((1 - w_j) e^eps + w_j)."""
    return alpha * F.cross_entropy(logits, labels) + ((1 - w) * math.exp(eps) + w).max(dim=0)[0]


# ------------------------------------------------------------------------- feawei init
def feawei_dp_init(features, k=1.0, zscore=True, base=(0.4, 0.5, 0.3)):
    """DP initialisation from a feature pass, numpy as in the reference:
    features [N, 2304] (the reference vstacks them into a float64 array, past_acc_feawei.py:141-144);
    mean_values = np.mean(weight, axis=0); z-score with np.std (past_acc.py:100, k = 1) or raw
    (past_acc_feawei.py:153-163, k = 5); w_init = 1 - F.sigmoid(torch.tensor(k * z, float32));
    DP = cat(full(0.4), full(0.5), full(0.3)) + w_init - 0.5 (past_acc.py:101-103)."""
    import numpy as np
    weight = np.vstack((np.empty((0, features.shape[1])), np.asarray(features)))
    mean_values = np.mean(weight, axis=0)
    if zscore:
        mean_values = (mean_values - np.mean(mean_values)) / np.std(mean_values)
    w_init = 1 - F.sigmoid(torch.tensor(k * mean_values, dtype=torch.float32))
    blk = features.shape[1] // len(base)
    dp0 = torch.cat([torch.full((1, blk), float(b)) for b in base], dim=1)
    return dp0 + w_init.unsqueeze(0) - 0.5


# ---------------------------------------------------------------------------- full path
def encoders(p, batch, cfg: PathConfig):
    """→ (pooled [B,768], img [B,768], cross [B,768])."""
    if cfg.contract == "W":
        eeg, act = batch["eeg"], batch["act"]                      # [B,C,T], [B,A]
        tokens = eeg.transpose(1, 2)                               # time-major [B,T,C]
        emb = bert_embeddings(p, inputs_embeds=_lin(tokens, p, "eeg_encoder"))
        mask = batch.get("eeg_mask", torch.ones(eeg.shape[0], eeg.shape[2], dtype=torch.long, device=eeg.device))
        vis = _lin(act.unsqueeze(1), p, "visual_encoder")          # [B,1,768]
        vmask = torch.ones(eeg.shape[0], 1, dtype=torch.long, device=eeg.device)
    else:
        emb = bert_embeddings(p, input_ids=batch["title_input"])
        mask = batch["text_mask"]
        vis = _lin(batch["frame_input"], p, "visual_encoder")
        vmask = batch["vedio_mask"]
    seq, pooled = bert(p, emb, mask)
    cross = decoder(p, vis, seq, mask, vmask)
    return pooled, vis.squeeze(1), cross


def forward(p, batch, cfg: PathConfig, noise=None, gumbels=None, row_noise=None, return_feature=False):
    pooled, img, cross = encoders(p, batch, cfg)
    f = torch.cat((pooled, img, cross), dim=1)                     # [B,2304]: EEG || action || cross
    if cfg.variant == "prigumbel_v1":
        logits = head_v1(p, f, gumbels, row_noise, cfg.tau, cfg.hard)
        return (logits, f, None) if return_feature else logits
    if cfg.variant == "priconcat":
        g = dp_guarantee(f, row_noise, cfg.honor_dp_mode)
    elif cfg.variant == "concat":
        g = minmax(f)
    else:
        g = prigumbel_gate(minmax(f), p["DP"], noise, gumbels, cfg.eps, cfg.eps_mode, cfg.hard)
    logits = head(p, g)
    return (logits, f, g) if return_feature else logits


def cal_loss(logits, labels):
    """past_acc.py:71-77 (mean CE, argmax accuracy)."""
    loss = F.cross_entropy(logits, labels)
    acc = (logits.argmax(1) == labels).float().mean()
    return loss, acc


# -------------------------------------------------------------- parameter inventory
def param_shapes(contract: str = "W", variant: str = "prigumbel", eeg_channels=64, act_dim=32,
                 modal: str = "ti") -> dict:
    """state_dict names/shapes of the path (reference names, SURVEY Appendix A.6 / probe7); `modal`
    selects a custom_models variant's module set (no BERT for ii, no visual encoder for tt, the
    TransformerEncoder instead of the decoder for tisc)."""
    s = {}
    if modal != "ii":
        _bert_shapes(s)
    if contract == "W":
        s["eeg_encoder.weight"] = (HID, eeg_channels)
        s["eeg_encoder.bias"] = (HID,)
        s["visual_encoder.weight"] = (HID, act_dim)
        s["visual_encoder.bias"] = (HID,)
    elif modal != "tt":
        s["visual_encoder.weight"] = (HID, 512)
        s["visual_encoder.bias"] = (HID,)
    if modal == "tisc":
        for pre in ["multi_head_encoderlayer."] + [f"multi_head_encoder.layers.{i}." for i in range(DEC_LAYERS)]:
            s[pre + "self_attn.in_proj_weight"] = (3 * HID, HID)
            s[pre + "self_attn.in_proj_bias"] = (3 * HID,)
            s[pre + "self_attn.out_proj.weight"] = (HID, HID)
            s[pre + "self_attn.out_proj.bias"] = (HID,)
            s[pre + "linear1.weight"] = (DEC_FF, HID)
            s[pre + "linear1.bias"] = (DEC_FF,)
            s[pre + "linear2.weight"] = (HID, DEC_FF)
            s[pre + "linear2.bias"] = (HID,)
            for n in ("norm1", "norm2"):
                s[pre + n + ".weight"] = (HID,)
                s[pre + n + ".bias"] = (HID,)
    else:
        _decoder_shapes(s)
    _head_shapes(s, variant)
    return s


def _bert_shapes(s):
    e = "bert.embeddings."
    s[e + "word_embeddings.weight"] = (30522, HID)
    s[e + "position_embeddings.weight"] = (512, HID)
    s[e + "token_type_embeddings.weight"] = (2, HID)
    s[e + "LayerNorm.weight"] = (HID,)
    s[e + "LayerNorm.bias"] = (HID,)
    for i in range(NLAYER):
        pre = f"bert.encoder.layer.{i}."
        for n in ("attention.self.query", "attention.self.key", "attention.self.value", "attention.output.dense"):
            s[pre + n + ".weight"] = (HID, HID)
            s[pre + n + ".bias"] = (HID,)
        for n in ("attention.output.LayerNorm", "output.LayerNorm"):
            s[pre + n + ".weight"] = (HID,)
            s[pre + n + ".bias"] = (HID,)
        s[pre + "intermediate.dense.weight"] = (FFN, HID)
        s[pre + "intermediate.dense.bias"] = (FFN,)
        s[pre + "output.dense.weight"] = (HID, FFN)
        s[pre + "output.dense.bias"] = (HID,)
    s["bert.pooler.dense.weight"] = (HID, HID)
    s["bert.pooler.dense.bias"] = (HID,)


def _decoder_shapes(s):
    for pre in ["multi_head_decoderlayer."] + [f"multi_head_decoder.layers.{i}." for i in range(DEC_LAYERS)]:
        for a in ("self_attn", "multihead_attn"):
            s[pre + a + ".in_proj_weight"] = (3 * HID, HID)
            s[pre + a + ".in_proj_bias"] = (3 * HID,)
            s[pre + a + ".out_proj.weight"] = (HID, HID)
            s[pre + a + ".out_proj.bias"] = (HID,)
        s[pre + "linear1.weight"] = (DEC_FF, HID)
        s[pre + "linear1.bias"] = (DEC_FF,)
        s[pre + "linear2.weight"] = (HID, DEC_FF)
        s[pre + "linear2.bias"] = (HID,)
        for n in ("norm1", "norm2", "norm3"):
            s[pre + n + ".weight"] = (HID,)
            s[pre + n + ".bias"] = (HID,)


def _head_shapes(s, variant):
    if variant == "prigumbel_v1":
        s["classifier.weight"] = (2, HID)
        s["classifier.bias"] = (2,)
        s["w"] = (HID,)
        s["fc1.weight"] = (FUSED, FUSED)
        s["fc1.bias"] = (FUSED,)
        s["fc2.weight"] = (HID, FUSED)
        s["fc2.bias"] = (HID,)
        return
    s["fc_layers.0.weight"] = (FUSED, FUSED)
    s["fc_layers.0.bias"] = (FUSED,)
    s["fc_layers.2.weight"] = (HID, FUSED)
    s["fc_layers.2.bias"] = (HID,)
    s["classifier.weight"] = (2, HID)
    s["classifier.bias"] = (2,)
    if variant in ("prigumbel", "concat"):
        s["DP"] = (1, FUSED)
