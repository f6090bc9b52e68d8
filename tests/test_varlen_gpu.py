"""Contract T pad skipping: BERT over the packed real tokens of right-padded
sequences must give the padded computation's outputs (the reference masks padded keys,
/root/reference/model.py:37-43; padded query rows never reach the loss).

Checks, all through the C-ABI:
  * eegf_attn_varlen_fwd/bwd against the dense kernels on the padded layout with the key mask
    (same Philox numbering, so also with attention dropout): real rows within 2e-5 (fp32) /
    1e-2 relative (bf16), pad rows zero;
  * eegf_seq_lengths / eegf_varlen_embed / eegf_varlen_rows against torch;
  * whole models: packed vs padded engine (fp32, dropout 0: logits 1e-5, every gradient 1e-4
    relative; bf16: cosine >= 0.999) and the reference golden vectors with packing on.
"""
import numpy as np
import pytest
import torch

from goldens import check_grads, det_params, load, rel_err

pytestmark = pytest.mark.gpu

H, DH = 12, 64


def _lib():
    from eegfusion import _lib
    return _lib


def _s():
    return torch.cuda.current_stream().cuda_stream


def _plan(lens, L):
    cu = np.zeros(len(lens) + 1, np.int32)
    cu[1:] = np.cumsum(lens)
    T = int(cu[-1])
    return torch.from_numpy(cu).cuda(), T, (T + 255) // 256 * 256


LENS = [1, 37, 64, 65, 200, 256, 257, 512]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attn_varlen_matches_padded(dt, p):
    L, B = 512, len(LENS)
    lib = _lib()
    code = lib.F32 if dt == torch.float32 else lib.BF16
    torch.manual_seed(3)
    cu, T, R = _plan(LENS, L)
    qkv_pad = torch.randn(B, L, 3 * H * DH, device="cuda").to(dt)
    mask = torch.zeros(B, L, dtype=torch.int64, device="cuda")
    for b, n in enumerate(LENS):
        mask[b, :n] = 1
    kbias = torch.empty(B, L, device="cuda")
    lib.call("eegf_key_bias", B * L, mask.data_ptr(), kbias.data_ptr(), _s())
    qkv_pk = torch.zeros(R, 3 * H * DH, device="cuda", dtype=dt)
    for b, n in enumerate(LENS):
        qkv_pk[cu[b]:cu[b] + n] = qkv_pad[b, :n]
    # dense reference on the padded layout
    out_d = torch.empty(B, L, H * DH, device="cuda", dtype=dt)
    lse_d = torch.empty(B, H, L, device="cuda")
    lib.call("eegf_attn_fwd", code, B, H, L, qkv_pad.data_ptr(), 3 * H * DH, kbias.data_ptr(), 0.125, p, 11, 5,
             out_d.data_ptr(), H * DH, lse_d.data_ptr(), None, _s())
    out_v = torch.full((R, H * DH), float("nan"), device="cuda").to(dt)
    lse_v = torch.empty(B, H, L, device="cuda")
    lib.call("eegf_attn_varlen_fwd", code, B, H, L, cu.data_ptr(), T, R, qkv_pk.data_ptr(), 3 * H * DH, None, 0.125, p, 11, 5,
             out_v.data_ptr(), H * DH, lse_v.data_ptr(), _s())
    dout_pad = torch.randn(B, L, H * DH, device="cuda").to(dt)
    dout_pk = torch.zeros(R, H * DH, device="cuda", dtype=dt)
    for b, n in enumerate(LENS):
        dout_pk[cu[b]:cu[b] + n] = dout_pad[b, :n]
        dout_pad[b, n:] = 0                       # padded queries carry no gradient (unused outputs)
    dq_d = torch.empty_like(qkv_pad)
    ws_d = torch.empty(max(lib.lib().eegf_attn_bwd_workspace(B, L), 1), device="cuda")
    lib.call("eegf_attn_bwd", code, B, H, L, qkv_pad.data_ptr(), 3 * H * DH, kbias.data_ptr(), 0.125, p, 11, 5,
             out_d.data_ptr(), dout_pad.data_ptr(), H * DH, lse_d.data_ptr(), None, dq_d.data_ptr(), ws_d.data_ptr(), _s())
    dq_v = torch.full((R, 3 * H * DH), float("nan"), device="cuda").to(dt)
    ws_v = torch.empty(max(lib.lib().eegf_attn_varlen_bwd_workspace(R, L), 1), device="cuda")
    lib.call("eegf_attn_varlen_bwd", code, B, H, L, cu.data_ptr(), T, R, qkv_pk.data_ptr(), 3 * H * DH, None, 0.125, p, 11, 5,
             out_v.data_ptr(), dout_pk.data_ptr(), H * DH, lse_v.data_ptr(), dq_v.data_ptr(), ws_v.data_ptr(), _s())
    torch.cuda.synchronize()
    tol = 2e-5 if dt == torch.float32 else 1e-2
    for b, n in enumerate(LENS):
        o_ref, o = out_d[b, :n].double(), out_v[cu[b]:cu[b] + n].double()
        assert (o - o_ref).abs().max().item() <= tol * max(1.0, o_ref.abs().max().item()), (b, n)
        assert torch.allclose(lse_v[b, :, :n], lse_d[b, :, :n], rtol=1e-5, atol=1e-4)
        g_ref, g = dq_d[b, :n].double(), dq_v[cu[b]:cu[b] + n].double()
        assert (g - g_ref).abs().max().item() <= tol * max(1.0, g_ref.abs().max().item()), (b, n)
    assert torch.count_nonzero(out_v[T:].float()) == 0 and torch.count_nonzero(dq_v[T:].float()) == 0


def test_varlen_front_end_kernels():
    lib = _lib()
    B, L, W = 5, 128, 768
    lens = [3, 128, 1, 77, 64]
    torch.manual_seed(1)
    mask = torch.zeros(B, L, dtype=torch.int64, device="cuda")
    for b, n in enumerate(lens):
        mask[b, :n] = 1
    buf = torch.empty(B + 1, dtype=torch.int32, device="cuda")
    lib.call("eegf_seq_lengths", B, L, mask.data_ptr(), buf.data_ptr(), buf[B:].data_ptr(), _s())
    torch.cuda.synchronize()
    assert buf[:B].tolist() == lens and buf[B].item() == 0
    mask2 = mask.clone()
    mask2[1, 5] = 0                                  # a hole: not right-padded
    lib.call("eegf_seq_lengths", B, L, mask2.data_ptr(), buf.data_ptr(), buf[B:].data_ptr(), _s())
    torch.cuda.synchronize()
    assert buf[B].item() == 1 and buf[1].item() == 127
    cu, T, R = _plan(lens, L)
    ids = torch.randint(0, 1000, (B, L), device="cuda")
    word = torch.randn(1000, W, device="cuda")
    pos = torch.randn(L, W, device="cuda")
    for dt in (torch.float32, torch.bfloat16):
        code = lib.F32 if dt == torch.float32 else lib.BF16
        out = torch.full((R, W), 7.0, device="cuda").to(dt)
        idp = torch.full((R,), -5, dtype=torch.int64, device="cuda")
        lib.call("eegf_varlen_embed", code, B, L, W, cu.data_ptr(), T, R, ids.data_ptr(), word.data_ptr(), pos.data_ptr(),
                 out.data_ptr(), idp.data_ptr(), _s())
        pad = torch.randn(B * L, W, device="cuda").to(dt)
        back = torch.full((R, W), 3.0, device="cuda").to(dt)
        lib.call("eegf_varlen_rows", code, B, L, W, cu.data_ptr(), T, R, pad.data_ptr(), W, back.data_ptr(), W, 0, _s())
        unp = torch.full((B * L, W), 3.0, device="cuda").to(dt)
        lib.call("eegf_varlen_rows", code, B, L, W, cu.data_ptr(), T, R, back.data_ptr(), W, unp.data_ptr(), W, 1, _s())
        torch.cuda.synchronize()
        for b, n in enumerate(lens):
            r0 = int(cu[b])
            ref = (word[ids[b, :n]] + pos[:n]).to(dt)
            assert torch.equal(out[r0:r0 + n], ref)
            assert torch.equal(idp[r0:r0 + n], ids[b, :n])
            assert torch.equal(back[r0:r0 + n], pad[b * L:b * L + n])
            assert torch.equal(unp[b * L:b * L + n], pad[b * L:b * L + n])
            assert torch.count_nonzero(unp[b * L + n:(b + 1) * L].float()) == 0
        assert torch.count_nonzero(out[T:].float()) == 0 and torch.count_nonzero(back[T:].float()) == 0
        assert torch.count_nonzero(idp[T:]) == 0


def _tokens_batch(lens, L, seed=0):
    g = torch.Generator().manual_seed(seed)
    B = len(lens)
    ids = torch.randint(1000, 30000, (B, L), generator=g)
    ids[:, 0] = 101
    mask = torch.zeros(B, L, dtype=torch.int64)
    for b, n in enumerate(lens):
        mask[b, :n] = 1
        ids[b, n:] = 0
    frame = torch.randn(B, 1, 512, generator=g) * 0.5
    vmask = torch.ones(B, 1, dtype=torch.int64)
    labels = torch.randint(0, 2, (B,), generator=g)
    dev = "cuda"
    return (frame.to(dev), vmask.to(dev), ids.to(dev), mask.to(dev)), labels.to(dev)


def _run_concat(x, labels, varlen, dtype):
    from eegfusion.modules import ConcatModel
    torch.manual_seed(0)
    m = ConcatModel(contract="T", dropout=0.0)
    m.load_state_dict(det_params("T", "concat", requires_grad=False), strict=False)
    m = m.cuda().train()
    if dtype != torch.float32:
        m.set_compute_dtype(dtype)
    m.engine.cfg.varlen = varlen
    logits = m(x, hard=True)
    torch.nn.CrossEntropyLoss(reduction="none")(logits, labels).sum().backward()
    torch.cuda.synchronize()
    return logits.detach().double().cpu(), {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()
                                            if p.grad is not None}


def test_concat_tokens_packed_equals_padded_fp32():
    x, labels = _tokens_batch([51, 37, 512, 1, 130, 256], 512)
    lp, gp = _run_concat(x, labels, False, torch.float32)
    lv, gv = _run_concat(x, labels, True, torch.float32)
    assert rel_err(lv, lp.numpy()) < 1e-5
    assert set(gp) == set(gv)
    for n in gp:
        if n.endswith("attention.self.key.bias"):
            # structurally zero (a per-head constant shift of every score cancels in the softmax):
            # both hold fp residue only, checked against the scale of the query-bias gradient
            scale = gp[n.replace("key.bias", "query.bias")].abs().max().item()
            assert gv[n].abs().max().item() <= 1e-4 * scale and gp[n].abs().max().item() <= 1e-4 * scale, n
            continue
        den = max(gp[n].abs().max().item(), 1e-30)
        assert (gv[n] - gp[n]).abs().max().item() / den < 1e-4, n


def test_concat_tokens_packed_equals_padded_bf16():
    x, labels = _tokens_batch([65, 33, 48, 60] * 4, 512, seed=2)
    lp, gp = _run_concat(x, labels, False, torch.bfloat16)
    lv, gv = _run_concat(x, labels, True, torch.bfloat16)
    assert rel_err(lv, lp.numpy()) < 2e-2
    for n in ("bert.encoder.layer.0.attention.self.query.weight", "bert.encoder.layer.11.output.dense.weight",
              "bert.embeddings.word_embeddings.weight", "bert.embeddings.position_embeddings.weight",
              "fc_layers.0.weight"):
        a, b = gv[n].flatten(), gp[n].flatten()
        cos = (a @ b / (a.norm() * b.norm())).item()
        assert cos >= 0.999, (n, cos)


@pytest.mark.parametrize("varlen", [False, True])
def test_concat_tokens_golden_packed_and_padded(varlen):
    """the reference's own golden vectors (real lengths 51 / 37 of 512) with packing on and off"""
    from eegfusion.modules import ConcatModel
    cfg, fx = load("full_concat_tokens")
    torch.manual_seed(0)
    m = ConcatModel(contract="T", dropout=0.0)
    m.load_state_dict(det_params("T", "concat", requires_grad=False), strict=False)
    m = m.cuda().train()
    m.engine.cfg.varlen = varlen
    dev = "cuda"
    x = tuple(torch.from_numpy(fx[k]).to(dev) for k in ("frame_input", "vedio_mask", "title_input", "text_mask"))
    logits = m(x, hard=True)
    loss = torch.nn.CrossEntropyLoss(reduction="none")(logits, torch.from_numpy(fx["labels"]).to(dev)).sum()
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(logits.detach().cpu(), fx["logits"]) < 1e-4
    check_grads({n: p.grad for n, p in m.named_parameters()}, fx, 1e-4)
