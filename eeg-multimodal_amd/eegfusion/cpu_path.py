"""The fusion path on the host CPU, for models whose parameters live in host memory.

BASELINE configs[0] ("ConcatModel on feature/train_EEG.csv + feature/action, batch 32, CPU PyTorch via
train.py (plumbing, no GPU)") and SURVEY §8(f)#1 ask that the drop-in run where no GPU exists
(`model.py:11-12` hard-codes `.cuda()`).  A model is on this path only when its parameter arena is
in host memory — a model moved to a GPU always runs libeegfusion.so, and a GPU process whose library
is missing fails at the first launch; nothing here is a fallback for a device model.

This is the reference computation in plain torch ops over the model's own parameters (autograd gives
the gradients), contract T and W, variants concat / priconcat(_lap) / prigumbel, the "ti" pairing:
  * BERT (modeling_bert.py:53-462 of the container's transformers 5.15): embeddings + LN(1e-12),
    12 layers of SDPA self-attention with the additive key mask, out-proj + residual + LN, GELU(erf)
    FFN + residual + LN, tanh pooler over CLS; dropout at the reference's sites;
  * the 3-layer post-norm TransformerDecoder (torch/nn/modules/transformer.py:1100-1200) through
    F.multi_head_attention_forward over the registered decoder parameters;
  * concat, row min-max (model.py:46-50), the privacy stage (past_acc.py:130-136 / main_0430.py:76-85),
    fc_layers + classifier.
Right-padded token batches are cut to their longest real sequence before BERT: padded keys carry the
mask bias (exp underflows to exactly 0), padded queries reach nothing the loss reads (the pooler takes
CLS, the decoder masks padded memory), so the logits are those of the padded computation.  Laplace and
Gumbel draws come from torch's generators as in the reference (`engine.injected` draws are honoured,
as on the device path).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

HID, NHEAD = 768, 12


def _lin(x, mod):
    return F.linear(x, mod.weight, mod.bias)


def _ln(x, mod, eps):
    return F.layer_norm(x, (x.shape[-1],), mod.weight, mod.bias, eps)


def _bert(model, cfg, batch, training):
    """-> (sequence output [B, L, 768], pooled [B, 768], key mask [B, L] int64)"""
    bert = model.bert
    emb = bert.embeddings
    p_h, p_a = (cfg.hidden_dropout, cfg.attn_dropout) if training else (0.0, 0.0)
    if cfg.contract == "W":
        eeg = batch["eeg"]                                           # [B, C, T] channel x time
        x = _lin(eeg.transpose(1, 2), model.eeg_encoder)             # time-major tokens -> inputs_embeds
        B, L = x.shape[:2]
        mask = torch.ones(B, L, dtype=torch.long)
    else:
        ids, mask = batch["title_input"], batch["text_mask"]
        lens = mask.sum(1)
        right_padded = bool((mask == (torch.arange(mask.shape[1]) < lens[:, None]).long()).all())
        # cut to the longest real sequence only where no dropout is drawn: F.dropout / SDPA dropout over
        # the cut tensors would consume torch's global RNG differently from the reference's padded run,
        # so every later draw (noise, gate, DataLoader order) would stop being seed-for-seed comparable
        if right_padded and int(lens.min()) > 0 and p_h == 0.0 and p_a == 0.0:
            keep = int(lens.max())
            ids, mask = ids[:, :keep], mask[:, :keep]
        B, L = ids.shape
        x = F.embedding(ids, emb.word_embeddings.weight)
    x = x + emb.position_embeddings.weight[:L] + emb.token_type_embeddings.weight[0]
    h = F.dropout(_ln(x, emb.LayerNorm, 1e-12), p_h, training)
    bias = (1.0 - mask[:, None, None, :].to(h.dtype)) * torch.finfo(h.dtype).min
    for lay in bert.encoder.layer:
        sa = lay.attention.self

        def heads(t):
            return t.view(B, L, NHEAD, HID // NHEAD).transpose(1, 2)
        q, k, v = heads(_lin(h, sa.query)), heads(_lin(h, sa.key)), heads(_lin(h, sa.value))
        ctx = F.scaled_dot_product_attention(q, k, v, attn_mask=bias, dropout_p=p_a if training else 0.0)
        ctx = ctx.transpose(1, 2).reshape(B, L, HID)
        a = _ln(F.dropout(_lin(ctx, lay.attention.output.dense), p_h, training) + h, lay.attention.output.LayerNorm,
                1e-12)
        f = F.gelu(_lin(a, lay.intermediate.dense))
        h = _ln(F.dropout(_lin(f, lay.output.dense), p_h, training) + a, lay.output.LayerNorm, 1e-12)
    pooled = torch.tanh(_lin(h[:, 0], bert.pooler.dense))
    return h, pooled, mask


def _mha(x, mem, attn, key_padding_mask, p, training):
    """nn.MultiheadAttention(batch_first=False) over [S, B, E] tensors (torch's own functional form)"""
    out, _ = F.multi_head_attention_forward(
        x, mem, mem, HID, NHEAD, attn.in_proj_weight, attn.in_proj_bias, None, None, False, p,
        attn.out_proj.weight, attn.out_proj.bias, training=training, key_padding_mask=key_padding_mask,
        need_weights=False)
    return out


def _decoder(model, tgt, mem, mem_mask, tgt_mask, p, training):
    """TransformerDecoder(TransformerDecoderLayer(768, 12), 3), post-norm, ReLU FFN 2048, LN 1e-5
    (model.py:20-21,40-44): tgt [1, B, 768] (the action token), memory [L, B, 768]."""
    x = tgt
    for lay in model.multi_head_decoder.layers:
        x = _ln(x + F.dropout(_mha(x, x, lay.self_attn, tgt_mask == 0, p, training), p, training), lay.norm1, 1e-5)
        x = _ln(x + F.dropout(_mha(x, mem, lay.multihead_attn, mem_mask == 0, p, training), p, training), lay.norm2,
                1e-5)
        ff = _lin(F.dropout(F.relu(_lin(x, lay.linear1)), p, training), lay.linear2)
        x = _ln(x + F.dropout(ff, p, training), lay.norm3, 1e-5)
    return x


def _minmax(f):
    lo = torch.min(f, dim=-1, keepdim=True)[0]
    hi = torch.max(f, dim=-1, keepdim=True)[0]
    return (f - lo) / (hi - lo)


def _privacy(model, cfg, f, hard):
    variant = cfg.variant
    inj = model.engine.injected or {}
    if variant == "concat":
        return _minmax(f)
    if variant == "priconcat":
        return f                                                     # DP_guarantee(dp_mode=None): identity
    if variant == "priconcat_lap":
        g = _minmax(f)
        row = inj.get("row_noise")
        if row is None:
            lap = torch.distributions.laplace.Laplace(torch.tensor([0.0]), torch.tensor([1.0 / cfg.eps]))
            row = lap.sample([f.shape[0]])
        return g + row.view(-1, 1).to(g)
    # prigumbel (past_acc.py:130-136)
    g = _minmax(f)
    w = torch.sigmoid(model.DP)
    noise = inj.get("noise")
    if noise is None:
        noise = model.noiser.sample(g.shape).view(*g.shape)
    a = math.exp(cfg.eps)
    r = ((a - w) / (1 - w)).log()
    eps_hat = 1 / r if cfg.eps_mode == "newfrac" else r
    y = g + noise.to(g) * eps_hat
    logits = torch.stack((w, 1 - w)).repeat(1, g.shape[0], 1)
    gum = inj.get("gumbels")
    if gum is None:
        mask = F.gumbel_softmax(logits, hard=hard, dim=0)
    else:                                                            # F.gumbel_softmax with recorded draws
        soft = ((logits + gum.to(g)) / cfg.tau).softmax(0)
        if hard:
            idx = soft.max(0, keepdim=True)[1]
            mask = torch.zeros_like(soft).scatter_(0, idx, 1.0) - soft.detach() + soft
        else:
            mask = soft
    return (y * mask).sum(0)


def forward(model, batch: dict, hard: bool, return_feature: bool = False):
    """logits [B, 2] (and the privacy stage's input/output with return_feature) of `model` on host
    tensors; gradients by autograd over the model's parameters."""
    cfg = model.engine.cfg
    if cfg.modal != "ti" or cfg.variant == "prigumbel_v1":
        raise NotImplementedError(f"eegfusion host path: modal {cfg.modal!r} / variant {cfg.variant!r} run on the "
                                  "GPU only; move the model with .cuda()")
    if getattr(model, "_dp", None) is not None:
        raise NotImplementedError("eegfusion host path: DP-SGD per-sample norms run on the GPU only")
    training = model.training
    seq, pooled, mask = _bert(model, cfg, batch, training)
    if cfg.contract == "W":
        vis = _lin(batch["act"].unsqueeze(1), model.visual_encoder)          # [B, 1, 768]
        vmask = torch.ones(vis.shape[0], 1, dtype=torch.long)
    else:
        vis = _lin(batch["frame_input"], model.visual_encoder)
        vmask = batch.get("vedio_mask", torch.ones(vis.shape[0], 1, dtype=torch.long)).reshape(vis.shape[0], 1)
    p = cfg.dec_dropout if training else 0.0
    cross = _decoder(model, vis.permute(1, 0, 2), seq.permute(1, 0, 2), mask, vmask, p, training)
    cross = cross.permute(1, 0, 2).mean(dim=1)
    f = torch.cat((pooled, vis.squeeze(1), cross), dim=1)                    # EEG || action || cross
    g = _privacy(model, cfg, f, hard)
    h = torch.tanh(_lin(torch.relu(_lin(g, model.fc_layers[0])), model.fc_layers[2]))
    logits = _lin(h, model.classifier)
    return (logits, f, g) if return_feature else logits
