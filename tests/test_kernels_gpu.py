"""GPU numerics of the non-GEMM kernels against float64 torch references of the same op.

Tolerances: fp32 ≤ 1e-4 relative to the reference's max magnitude (fp32 storage / fp32 math);
bf16 ≤ 3e-2 relative (bf16 storage, fp32 math).
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DT = [torch.float32, torch.bfloat16]


def _tol(dt):
    return 1e-4 if dt == torch.float32 else 3e-2


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _lib():
    from eegfusion import _lib
    return _lib


def _s():
    return torch.cuda.current_stream().cuda_stream


def _code(dt):
    return 0 if dt == torch.float32 else 1


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_layernorm_fwd_bwd(dt, mode):
    L = _lib()
    torch.manual_seed(0)
    R, W = 300, 768
    x = torch.randn(R, W, device="cuda").to(dt)
    r = torch.randn(R, W, device="cuda").to(dt)
    g = (1 + 0.1 * torch.randn(W, device="cuda"))
    b = 0.1 * torch.randn(W, device="cuda")
    y = torch.empty_like(x)
    s = torch.empty_like(x)
    mean = torch.empty(R, device="cuda")
    rstd = torch.empty(R, device="cuda")
    p = 0.0 if mode == 0 else 0.25
    L.call("eegf_ln_fwd", _code(dt), R, W, x.data_ptr(), r.data_ptr(), None, 1, None, g.data_ptr(), b.data_ptr(),
           1e-12, p, mode, 123, 7, y.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(), _s())
    torch.cuda.synchronize()
    # recover the dropout masks from the kernel output (scale 1/(1-p) or 0)
    xd, rd = x.double(), r.double()
    if mode == 1:
        m = ((s.double() - rd) != 0).double() / (1 - p)      # dropped lanes store s == r exactly
        assert abs(1 - (1 - p) * m.mean().item() - p) < 0.02
        from philox_ref import attn_mask                      # element-exact: the Philox-7 16-bit stream
        want = torch.from_numpy(attn_mask(123, 7, np.arange(R * W, dtype=np.uint64), p) > 0).view(R, W)
        got = (m > 0).cpu()
        # bf16: a kept x*scale below half an ulp of r rounds s back to r and reads as dropped
        assert torch.equal(got, want) if dt == torch.float32 else not (got & ~want).any()
        v = xd * m + rd
        assert _rel(s, v) < _tol(dt)
    else:
        v = xd + rd
    ref = F.layer_norm(v, (W,), g.double(), b.double(), 1e-12)
    if mode == 2:
        kept = y.double().abs() > 0
        assert abs(1 - kept.double().mean().item() - p) < 0.02
        from philox_ref import attn_mask
        want = torch.from_numpy(attn_mask(123, 7, np.arange(R * W, dtype=np.uint64), p) > 0).view(R, W)
        assert torch.equal(kept.cpu(), want) if dt == torch.float32 else not (kept.cpu() & ~want).any()
        ref = torch.where(kept, ref / (1 - p), torch.zeros_like(ref))
    assert _rel(y, ref) < _tol(dt)
    # backward vs autograd (mode 0 only: masks already checked)
    if mode == 0:
        vv = v.clone().requires_grad_()
        gg = g.double().clone().requires_grad_()
        bb = b.double().clone().requires_grad_()
        out = F.layer_norm(vv, (W,), gg, bb, 1e-12)
        dy = torch.randn(R, W, device="cuda").to(dt)
        out.backward(dy.double())
        dx = torch.empty_like(x)
        rpb = L.lib().eegf_ln_bwd_partial_rows(R)          # the ABI's block size (include/eegfusion.h)
        nb = (R + rpb - 1) // rpb
        part = torch.empty(2, nb, W, device="cuda")
        L.call("eegf_ln_bwd", _code(dt), R, W, dy.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
               g.data_ptr(), 0.0, 0, 0, 0, dx.data_ptr(), None, part[0].data_ptr(), part[1].data_ptr(), _s())
        torch.cuda.synchronize()
        assert _rel(dx, vv.grad) < _tol(dt) * 3
        assert _rel(part[0].sum(0), gg.grad) < _tol(dt)
        assert _rel(part[1].sum(0), bb.grad) < _tol(dt)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("with_r,with_tables", [(True, False), (False, True), (True, True)])
def test_layernorm768_matches_generic(mode, with_r, with_tables):
    """bf16 768-wide rows take ln_fwd768_kernel (16-B accesses, eegf_tune key 10); it must keep exactly
    the generic kernel's dropout elements and agree on every output within bf16 rounding, at the bench
    row count (65536 rows: 16 rows per wave with the next row's loads in flight)."""
    L = _lib()
    torch.manual_seed(1)
    R, W = 65536, 768
    x = torch.randn(R, W, device="cuda").to(torch.bfloat16)
    r = torch.randn(R, W, device="cuda").to(torch.bfloat16) if with_r else None
    tab = torch.randn(256, W, device="cuda") if with_tables else None
    tab2 = torch.randn(W, device="cuda") if with_tables else None
    g = 1 + 0.1 * torch.randn(W, device="cuda")
    b = 0.1 * torch.randn(W, device="cuda")
    p = 0.0 if mode == 0 else 0.1
    outs = []
    for kern in (1, 0):
        old = L.lib().eegf_tune(10, kern)
        y, s = torch.empty_like(x), torch.empty_like(x)
        mean, rstd = torch.empty(R, device="cuda"), torch.empty(R, device="cuda")
        L.call("eegf_ln_fwd", 1, R, W, x.data_ptr(), r.data_ptr() if with_r else None,
               tab.data_ptr() if with_tables else None, 256, tab2.data_ptr() if with_tables else None,
               g.data_ptr(), b.data_ptr(), 1e-12, p, mode, 99, 5, y.data_ptr(), s.data_ptr(), mean.data_ptr(),
               rstd.data_ptr(), _s())
        torch.cuda.synchronize()
        L.lib().eegf_tune(10, old)
        outs.append((y, s, mean, rstd))
    (y1, s1, m1, r1), (y0, s0, m0, r0) = outs
    if mode == 2:
        assert torch.equal(y1 == 0, y0 == 0)
    # the residual sum (mode 1: dropout applied before it) is the same fp32 expression rounded once:
    # identical, which also pins the mode-1 keep elements
    assert torch.equal(s1, s0)
    assert _rel(m1, m0) < 1e-5 and _rel(r1, r0) < 1e-5
    assert (y1.float() - y0.float()).abs().max().item() <= 2 * 2 ** -8 * y0.float().abs().max().item()


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("period", [1, 6, 256])
def test_colsum(dt, period):
    L = _lib()
    rows, W = 1536, 300
    x = torch.randn(rows, W, device="cuda").to(dt)
    out = torch.randn(period, W, device="cuda")
    ws = torch.empty(1 << 22, device="cuda")
    ref = out.double() * 0.5 + x.double().view(rows // period if rows % period == 0 else -1, period, W).sum(0) \
        if rows % period == 0 else None
    if ref is None:
        ref = out.double() * 0.5
        for p in range(period):
            ref[p] += x.double()[p::period].sum(0)
    L.call("eegf_colsum", _code(dt), x.data_ptr(), W, rows, W, period, ws.data_ptr(), ws.numel(), out.data_ptr(),
           0.5, _s())
    torch.cuda.synchronize()
    assert _rel(out, ref) < 1e-5


def _attn_ref(qkv, B, L, kbias, zmask=None):
    q, k, v = qkv.double().view(B, L, 3, 12, 64).unbind(2)
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    s = q @ k.transpose(-1, -2) / 8.0
    if kbias is not None:
        s = s + kbias.double()[:, None, None, :]
    p = s.softmax(-1)
    if zmask is not None:            # dropout(attention_probs) with the kernel's Philox mask
        p = p * zmask
    return (p @ v).transpose(1, 2).reshape(B, L, 768)


def _check_bits(bits, z, B, L):
    """keep bits [B*12][L][L/32] (bit t of word j <-> key 32j+t) == the replayed Philox keep mask"""
    w = bits.view(B, 12, L, L // 32).to(torch.int64) & 0xFFFFFFFF
    t = torch.arange(32, device=w.device)
    keep = ((w[..., None] >> t) & 1).view(B, 12, L, L)
    assert torch.equal(keep.bool(), z > 0)


def _attn_mask(B, L, p, seed, offset):
    from philox_ref import attn_probs_mask
    e = torch.arange(B * 12 * L * L, dtype=torch.int64).numpy()
    return torch.from_numpy(attn_probs_mask(seed, offset, e, p, L)).view(B, 12, L, L).cuda()


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("L", [256, 512])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("pdrop", [0.0, 0.25])
@pytest.mark.parametrize("use_bits", [False, True])
def test_attention_fwd_bwd(dt, L, masked, pdrop, use_bits):
    lib = _lib()
    torch.manual_seed(1)
    B = 2
    qkv = torch.randn(B, L, 2304, device="cuda").to(dt)
    kbias = None
    if masked:
        lens = [L // 3, L]
        mask = torch.zeros(B, L, dtype=torch.long, device="cuda")
        for i, n in enumerate(lens):
            mask[i, :n] = 1
        kbias = torch.empty(B, L, device="cuda")
        lib.call("eegf_key_bias", B * L, mask.data_ptr(), kbias.data_ptr(), _s())
    out = torch.empty(B, L, 768, device="cuda", dtype=dt)
    lse = torch.empty(B, 12, L, device="cuda")
    bits = torch.zeros(B * 12 * L * L // 32, device="cuda", dtype=torch.int32)
    seed, off = 77, 5
    lib.call("eegf_attn_fwd", _code(dt), B, 12, L, qkv.data_ptr(), 2304, None if kbias is None else kbias.data_ptr(),
             0.125, pdrop, seed, off, out.data_ptr(), 768, lse.data_ptr(), bits.data_ptr() if use_bits else None, _s())
    torch.cuda.synchronize()
    qr = qkv.double().clone().requires_grad_()
    z = _attn_mask(B, L, pdrop, seed, off) if pdrop > 0 else None
    if z is not None and use_bits:     # the stored keep bits are the Philox mask
        _check_bits(bits, z, B, L)
    if z is not None:
        assert abs((z > 0).double().mean().item() - (1 - pdrop)) < 0.01
    ref = _attn_ref(qr, B, L, kbias, z)
    assert _rel(out, ref) < _tol(dt)
    dout = torch.randn(B, L, 768, device="cuda").to(dt)
    ref.backward(dout.double())
    dqkv = torch.empty_like(qkv)
    ws_n = lib.lib().eegf_attn_bwd_workspace(B, L)
    ws = torch.empty(max(ws_n, 1), device="cuda")
    lib.call("eegf_attn_bwd", _code(dt), B, 12, L, qkv.data_ptr(), 2304, None if kbias is None else kbias.data_ptr(),
             0.125, pdrop, seed, off, out.data_ptr(), dout.data_ptr(), 768, lse.data_ptr(),
             bits.data_ptr() if use_bits else None, dqkv.data_ptr(), ws.data_ptr(), _s())
    torch.cuda.synchronize()
    for sl, name in ((slice(0, 768), "dq"), (slice(768, 1536), "dk"), (slice(1536, 2304), "dv")):
        e = _rel(dqkv[..., sl], qr.grad[..., sl])
        assert e < _tol(dt) * 3, (name, e)


@pytest.mark.parametrize("pdrop", [1e-6, 0.1])
def test_attention256_exports_keep_bits(pdrop):
    """The L = 256 forward with a drop_bits buffer (the engine's path with cfg.attn_bits / EEGF_ATTN_BITS=1): identical output
    bits to the forward without it, the exported mask equals the Philox replay (p = 1e-6 < 2^-16: every
    probability kept, all-ones words), and the backward reading the bits equals the one regenerating."""
    lib = _lib()
    torch.manual_seed(3)
    B, L = 3, 256
    qkv = torch.randn(B, L, 2304, device="cuda").to(torch.bfloat16)
    dout = torch.randn(B, L, 768, device="cuda").to(torch.bfloat16)
    ws = torch.empty(max(lib.lib().eegf_attn_bwd_workspace(B, L), 1), device="cuda")
    res = {}
    for use_bits in (False, True):
        out = torch.empty(B, L, 768, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B, 12, L, device="cuda")
        bits = torch.zeros(B * 12 * L * L // 32, device="cuda", dtype=torch.int32)
        dqkv = torch.empty_like(qkv)
        bp = bits.data_ptr() if use_bits else None
        lib.call("eegf_attn_fwd", _code(torch.bfloat16), B, 12, L, qkv.data_ptr(), 2304, None, 0.125, pdrop, 11, 4,
                 out.data_ptr(), 768, lse.data_ptr(), bp, _s())
        lib.call("eegf_attn_bwd", _code(torch.bfloat16), B, 12, L, qkv.data_ptr(), 2304, None, 0.125, pdrop, 11, 4,
                 out.data_ptr(), dout.data_ptr(), 768, lse.data_ptr(), bp, dqkv.data_ptr(), ws.data_ptr(), _s())
        torch.cuda.synchronize()
        res[use_bits] = (out, lse, dqkv, bits)
    assert torch.equal(res[False][0], res[True][0]) and torch.equal(res[False][1], res[True][1])
    assert torch.equal(res[False][2], res[True][2])
    bits = res[True][3]
    if pdrop < 2.0 ** -16:
        assert bool((bits == -1).all())
    else:
        _check_bits(bits, _attn_mask(B, L, pdrop, 11, 4), B, L)


@pytest.mark.parametrize("dt", DT)
def test_xattn_mixed_dtypes(dt):
    """bf16 memory with fp32 query/context (mixed-precision engine)."""
    lib = _lib()
    torch.manual_seed(9)
    B, S = 2, 256
    mem = torch.randn(B, S, 768, device="cuda").to(torch.bfloat16)
    qp = 0.05 * torch.randn(B, 12, 768, device="cuda")
    probs = torch.empty(B, 12, S, device="cuda")
    cc = torch.empty(B, 12, 768, device="cuda")
    ws = torch.empty(B * 12 * S, device="cuda")
    lib.call("eegf_xattn_fwd", 1, 0, B, S, mem.data_ptr(), qp.data_ptr(), None, 0.0, 0, 0, ws.data_ptr(),
             probs.data_ptr(), None, cc.data_ptr(), _s())
    torch.cuda.synchronize()
    p = torch.einsum("bhc,bjc->bhj", qp.double(), mem.double()).softmax(-1)
    assert _rel(cc, torch.einsum("bhj,bjc->bhc", p, mem.double())) < 1e-5


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("S,pdrop,masked", [(256, 0.0, False), (256, 0.3, False), (100, 0.0, True), (300, 0.2, True)])
def test_xattn_fwd_bwd(dt, S, pdrop, masked):
    """Reduced cross-attention (scores, softmax, dropout(p), context, s = sum p~) and its backward
    (dM, dq', with a gradient on s) vs float64 autograd with the replayed Philox mask."""
    from philox_ref import drop_mask
    lib = _lib()
    torch.manual_seed(2)
    B = 3
    seed, off = 1234, 99
    mem = torch.randn(B, S, 768, device="cuda").to(dt)
    qp = (0.05 * torch.randn(B, 12, 768, device="cuda")).to(dt)
    kbias = None
    if masked:
        kbias = torch.zeros(B, S, device="cuda")
        kbias[0, S // 2:] = -1e30
    probs = torch.empty(B, 12, S, device="cuda")
    psum = torch.empty(B, 12, device="cuda")
    cc = torch.empty(B, 12, 768, device="cuda", dtype=dt)
    ws = torch.empty(B * 12 * S, device="cuda")
    lib.call("eegf_xattn_fwd", _code(dt), _code(dt), B, S, mem.data_ptr(), qp.data_ptr(),
             None if kbias is None else kbias.data_ptr(), pdrop, seed, off, ws.data_ptr(), probs.data_ptr(),
             psum.data_ptr(), cc.data_ptr(), _s())
    torch.cuda.synchronize()
    m = mem.double().clone().requires_grad_()
    q = qp.double().clone().requires_grad_()
    sc = torch.einsum("bhc,bjc->bhj", q, m)
    if kbias is not None:
        sc = sc + kbias.double()[:, None, :]
    p = sc.softmax(-1)
    z = torch.ones_like(p)
    if pdrop > 0:
        z = torch.from_numpy(drop_mask(seed, off, torch.arange(B * 12 * S).numpy(), pdrop)).view(B, 12, S).cuda()
    pt = p * z
    c = torch.einsum("bhj,bjc->bhc", pt, m)
    s = pt.sum(-1)
    assert _rel(probs, p) < _tol(dt)
    assert _rel(cc, c) < _tol(dt)
    if pdrop > 0:
        assert _rel(psum, s) < 1e-5
    dc = torch.randn(B, 12, 768, device="cuda").to(dt)
    dps = torch.randn(B, 12, device="cuda")
    (c * dc.double()).sum().add((s * dps.double()).sum() if pdrop > 0 else 0.0).backward()
    dmem = torch.randn_like(mem)
    dmem0 = dmem.double().clone()
    dqp = torch.empty_like(qp)
    lib.call("eegf_xattn_bwd", _code(dt), _code(dt), B, S, mem.data_ptr(), qp.data_ptr(), probs.data_ptr(),
             dps.data_ptr() if pdrop > 0 else None, dc.data_ptr(), pdrop, seed, off, ws.data_ptr(), dmem.data_ptr(),
             1.0, dqp.data_ptr(), _s())
    torch.cuda.synchronize()
    assert _rel(dmem.double() - dmem0, m.grad) < _tol(dt) * 3
    assert _rel(dqp, q.grad) < _tol(dt) * 3


@pytest.mark.parametrize("S,pdrop", [(256, 0.1), (256, 0.0), (100, 0.2), (300, 0.0), (7, 0.3)])
def test_xattn_fwd_mixed_mfma(S, pdrop):
    """The engine's cross-attention context (bf16 memory, fp32 query / context) on the fp32-MFMA kernel
    (eegf_tune key 19 = 1) vs float64 with the replayed Philox mask, and vs the VALU kernel (key 19 = 0):
    identical probabilities and s = sum p~ (same softmax code), the context within fp32 summation order."""
    from philox_ref import drop_mask
    lib = _lib()
    torch.manual_seed(6)
    B, seed, off = 3, 31, 2
    mem = torch.randn(B, S, 768, device="cuda").to(torch.bfloat16)
    qp = 0.05 * torch.randn(B, 12, 768, device="cuda")
    tune = lib.lib().eegf_tune
    tune.argtypes = [lib.i32, lib.i32]
    out = {}
    for key in (1, 0):
        probs = torch.empty(B, 12, S, device="cuda")
        psum = torch.empty(B, 12, device="cuda")
        cc = torch.empty(B, 12, 768, device="cuda")
        ws = torch.empty(B * 12 * S, device="cuda")
        old = tune(19, key)
        try:
            lib.call("eegf_xattn_fwd", 1, 0, B, S, mem.data_ptr(), qp.data_ptr(), None, pdrop, seed, off,
                     ws.data_ptr(), probs.data_ptr(), psum.data_ptr(), cc.data_ptr(), _s())
            torch.cuda.synchronize()
        finally:
            tune(19, old)
        out[key] = (probs, psum, cc)
    p = torch.einsum("bhc,bjc->bhj", qp.double(), mem.double()).softmax(-1)
    z = torch.ones_like(p)
    if pdrop > 0:
        z = torch.from_numpy(drop_mask(seed, off, torch.arange(B * 12 * S).numpy(), pdrop)).view(B, 12, S).cuda()
    c = torch.einsum("bhj,bjc->bhc", p * z, mem.double())
    assert torch.equal(out[1][0], out[0][0]) and torch.equal(out[1][1], out[0][1])
    assert _rel(out[1][2], c) < 1e-5 and _rel(out[1][2], out[0][2]) < 1e-5


@pytest.mark.parametrize("S,pdrop,beta", [(256, 0.1, 1.0), (256, 0.0, 0.0), (100, 0.2, 1.0), (300, 0.0, 1.0), (7, 0.3, 0.0)])
def test_xattn_bwd_mixed_mfma(S, pdrop, beta):
    """The engine's cross-attention backward (bf16 memory, fp32 query / context gradient) on the fp32-MFMA
    kernel (eegf_tune key 19 = 1) vs float64 autograd with the replayed Philox mask, and vs the VALU kernel
    (key 19 = 0): the same fp32 products summed in another order."""
    from philox_ref import drop_mask
    lib = _lib()
    torch.manual_seed(5)
    B, seed, off = 3, 77, 5
    mem = torch.randn(B, S, 768, device="cuda").to(torch.bfloat16)
    qp = 0.05 * torch.randn(B, 12, 768, device="cuda")
    probs = torch.empty(B, 12, S, device="cuda")
    psum = torch.empty(B, 12, device="cuda")
    cc = torch.empty(B, 12, 768, device="cuda")
    ws = torch.empty(B * 12 * S, device="cuda")
    lib.call("eegf_xattn_fwd", 1, 0, B, S, mem.data_ptr(), qp.data_ptr(), None, pdrop, seed, off, ws.data_ptr(),
             probs.data_ptr(), psum.data_ptr(), cc.data_ptr(), _s())
    torch.cuda.synchronize()
    m = mem.double().clone().requires_grad_()
    q = qp.double().clone().requires_grad_()
    p = torch.einsum("bhc,bjc->bhj", q, m).softmax(-1)
    z = torch.ones_like(p)
    if pdrop > 0:
        z = torch.from_numpy(drop_mask(seed, off, torch.arange(B * 12 * S).numpy(), pdrop)).view(B, 12, S).cuda()
    pt = p * z
    c = torch.einsum("bhj,bjc->bhc", pt, m)
    dc = torch.randn(B, 12, 768, device="cuda")
    dps = torch.randn(B, 12, device="cuda")
    (c * dc.double()).sum().add((pt.sum(-1) * dps.double()).sum() if pdrop > 0 else 0.0).backward()
    dmem0 = torch.randn_like(mem)
    out = {}
    for key in (1, 0):
        tune = lib.lib().eegf_tune
        tune.argtypes = [lib.i32, lib.i32]
        old = tune(19, key)
        try:
            dmem = dmem0.clone()
            dqp = torch.empty_like(qp)
            lib.call("eegf_xattn_bwd", 1, 0, B, S, mem.data_ptr(), qp.data_ptr(), probs.data_ptr(),
                     dps.data_ptr() if pdrop > 0 else None, dc.data_ptr(), pdrop, seed, off, ws.data_ptr(),
                     dmem.data_ptr(), beta, dqp.data_ptr(), _s())
            torch.cuda.synchronize()
        finally:
            tune(19, old)
        out[key] = (dmem, dqp)
    for key, (dmem, dqp) in out.items():
        ref_m = m.grad + beta * dmem0.double()
        assert _rel(dmem, ref_m) < 1e-2, key                 # bf16 output: one rounding
        assert _rel(dqp, q.grad) < 1e-5, key                 # fp32 output
    assert _rel(out[1][1], out[0][1]) < 1e-5
    assert (out[1][0].double() - out[0][0].double()).abs().max() <= 2 * 2.0 ** -8 * out[0][0].double().abs().max()


def test_head_bias_fwd_bwd():
    lib = _lib()
    torch.manual_seed(4)
    B = 37
    x = torch.randn(B, 768, device="cuda")
    bias = torch.randn(768, device="cuda")
    s = torch.rand(B, 12, device="cuda")
    ref = x.double() + bias.double() * s.double().repeat_interleave(64, 1)
    lib.call("eegf_head_bias_fwd", B, 768, 64, x.data_ptr(), bias.data_ptr(), s.data_ptr(), _s())
    torch.cuda.synchronize()
    assert _rel(x, ref) < 1e-6
    dx = torch.randn(B, 768, device="cuda")
    ds = torch.empty(B, 12, device="cuda")
    dbias = torch.randn(768, device="cuda")
    db0 = dbias.double().clone()
    lib.call("eegf_head_bias_bwd", B, 768, 64, dx.data_ptr(), bias.data_ptr(), s.data_ptr(), ds.data_ptr(),
             dbias.data_ptr(), 1.0, _s())
    torch.cuda.synchronize()
    assert _rel(ds, (dx.double() * bias.double()).view(B, 12, 64).sum(-1)) < 1e-5
    assert _rel(dbias.double() - db0, (dx.double() * s.double().repeat_interleave(64, 1)).sum(0)) < 1e-5


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("group", [1, 64])
def test_dropout_grouped(dt, group):
    from philox_ref import drop_mask
    lib = _lib()
    torch.manual_seed(5)
    n, p, seed, off = 256 * 768, 0.1, 31, 17
    x = torch.randn(n, device="cuda").to(dt)
    x0 = x.double().clone()
    lib.call("eegf_dropout", _code(dt), n, group, p, seed, off, x.data_ptr(), _s())
    torch.cuda.synchronize()
    mk = torch.from_numpy(drop_mask(seed, off, (torch.arange(n) // group).numpy(), p)).cuda()
    assert abs((mk > 0).double().mean().item() - (1 - p)) < 0.02 if group == 1 else True
    assert _rel(x, x0 * mk) < _tol(dt)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("hard", [False, True])
@pytest.mark.parametrize("eps", [0.1, 1.0, 3.0, 5.0, 10.0])      # BASELINE configs[4] sweep
def test_fusion_prigumbel_injected(dt, hard, eps):
    """Fusion kernel vs the oracle gate on injected draws (fp64 autograd of the same formulas)."""
    import sys
    from oracle import fusion_oracle as O
    lib = _lib()
    torch.manual_seed(3)
    B = 5
    parts = [torch.randn(B, 768, device="cuda").to(dt) for _ in range(3)]
    DP = 0.5 * torch.randn(1, 2304, device="cuda")
    noise = O.laplace_from_uniform(torch.rand(B, 2304, device="cuda") * 2 - 1).float()
    gumb = -torch.log(-torch.log(torch.rand(2, B, 2304, device="cuda").clamp(1e-6, 1 - 1e-6)))
    out = torch.empty(B, 2304, device="cuda", dtype=dt)
    xn = torch.empty(B, 2304, device="cuda")
    amin = torch.empty(B, dtype=torch.int32, device="cuda")
    amax = torch.empty_like(amin)
    rg = torch.empty(B, device="cuda")
    lib.call("eegf_fusion_fwd", _code(dt), B, 3, parts[0].data_ptr(), 768, parts[1].data_ptr(), 768,
             parts[2].data_ptr(), 768, DP.data_ptr(), noise.data_ptr(), gumb.data_ptr(), None, int(hard), 0,
             math.exp(eps), 1 / eps, 0, 0, out.data_ptr(), xn.data_ptr(), amin.data_ptr(), amax.data_ptr(),
             rg.data_ptr(), _s())
    torch.cuda.synchronize()
    ps = [p.double().clone().requires_grad_() for p in parts]
    dp = DP.double().clone().requires_grad_()
    f = O.minmax(torch.cat(ps, 1))
    ref = O.prigumbel_gate(f, dp, noise.double(), gumb.double(), eps, "newfrac", hard)
    assert _rel(out, ref) < _tol(dt)
    dout = torch.randn(B, 2304, device="cuda").to(dt)
    ref.backward(dout.double())
    d = [torch.empty_like(p) for p in parts]
    ddp = torch.empty(B, 2304, device="cuda")
    lib.call("eegf_fusion_bwd", _code(dt), B, 3, dout.data_ptr(), xn.data_ptr(), amin.data_ptr(), amax.data_ptr(),
             rg.data_ptr(), DP.data_ptr(), noise.data_ptr(), gumb.data_ptr(), int(hard), 0, math.exp(eps), 0, 0,
             d[0].data_ptr(), 768, d[1].data_ptr(), 768, d[2].data_ptr(), 768, ddp.data_ptr(), _s())
    torch.cuda.synchronize()
    for a, b in zip(d, ps):
        assert _rel(a, b.grad) < _tol(dt) * 3
    assert _rel(ddp.sum(0, keepdim=True), dp.grad) < _tol(dt) * 3


@pytest.mark.parametrize("dt", DT)
def test_fusion_philox_statistics(dt):
    """Without injected draws the kernel's Laplace noise has the Laplace(0,1) law."""
    lib = _lib()
    B = 256
    z = torch.zeros(B, 768, device="cuda", dtype=dt)
    z[:, 0] = 1.0                                   # min 0, max 1 -> xn = input
    DP = torch.zeros(1, 2304, device="cuda")        # w = 0.5
    out = torch.empty(B, 2304, device="cuda", dtype=dt)
    xn = torch.empty(B, 2304, device="cuda")
    ai = torch.empty(B, dtype=torch.int32, device="cuda")
    rg = torch.empty(B, device="cuda")
    eps = 1.0
    lib.call("eegf_fusion_fwd", _code(dt), B, 3, z.data_ptr(), 768, z.data_ptr(), 768, z.data_ptr(), 768,
             DP.data_ptr(), None, None, None, 0, 0, math.exp(eps), 1.0, 42, 0, out.data_ptr(), xn.data_ptr(),
             ai.data_ptr(), ai.data_ptr(), rg.data_ptr(), _s())
    torch.cuda.synchronize()
    eh = 1.0 / math.log((math.e - 0.5) / 0.5)
    n = ((out.double() - xn.double()) / eh)[:, 1:]
    assert abs(n.mean().item()) < 0.02
    assert abs(n.abs().mean().item() - 1.0) < 0.03      # E|Laplace(0,1)| = 1
    assert abs(n.var().item() - 2.0) < 0.1              # Var = 2


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("reduction", [0, 1])
def test_cross_entropy(dt, reduction):
    lib = _lib()
    B = 300
    z = torch.randn(B, 2, device="cuda").to(dt)
    y = torch.randint(0, 2, (B,), device="cuda")
    loss = torch.empty(1, device="cuda")
    corr = torch.empty(1, dtype=torch.int32, device="cuda")
    dz = torch.empty_like(z)
    lib.call("eegf_cross_entropy", _code(dt), B, 2, z.data_ptr(), y.data_ptr(), reduction, 1.0, loss.data_ptr(),
             corr.data_ptr(), dz.data_ptr(), _s())
    torch.cuda.synchronize()
    zr = z.double().clone().requires_grad_()
    ref = F.cross_entropy(zr, y, reduction="mean" if reduction == 0 else "sum")
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-4 * max(1, abs(ref.item()))
    assert corr.item() == (z.float().argmax(1) == y).sum().item()
    assert _rel(dz, zr.grad) < _tol(dt)


def test_adam_matches_torch():
    lib = _lib()
    torch.manual_seed(4)
    n = 10000 + 3
    p = torch.randn(n, device="cuda")
    p_ref = p.clone().requires_grad_()
    opt = torch.optim.Adam([p_ref], lr=1e-3, weight_decay=0.01)
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    shadow = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    for step in range(1, 4):
        g = torch.randn(n, device="cuda")
        p_ref.grad = g.clone()
        opt.step()
        lib.call("eegf_adam", n, p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), shadow.data_ptr(), 1e-3, 0.9,
                 0.999, 1e-8, 0.01, 1.0, step, _s())
    torch.cuda.synchronize()
    assert (p - p_ref.detach()).abs().max().item() < 1e-6
    # grad_scale: a step over an all-reduced sum of 4 ranks equals the step over the averaged gradient
    # bitwise (the 1/N product is the fp32 product torch's mul_ stores)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    g = torch.randn(n, device="cuda")
    g4 = g.mul(0.25)
    lib.call("eegf_adam", n, p.data_ptr(), g4.data_ptr(), m.data_ptr(), v.data_ptr(), None, 1e-3, 0.9,
             0.999, 1e-8, 0.01, 1.0, 4, _s())
    lib.call("eegf_adam", n, p2.data_ptr(), g.data_ptr(), m2.data_ptr(), v2.data_ptr(), None, 1e-3, 0.9,
             0.999, 1e-8, 0.01, 0.25, 4, _s())
    torch.cuda.synchronize()
    assert torch.equal(p, p2) and torch.equal(m, m2) and torch.equal(v, v2)
    assert (shadow.float() - p).abs().max().item() <= 1e-2 * p.abs().max().item()
    # eegf_adam_consume: bitwise the same step, and the gradient left zero (ragged tail included)
    p3, m3, v3, g3 = p.clone(), m.clone(), v.clone(), g.clone()
    lib.call("eegf_adam", n, p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), None, 1e-3, 0.9,
             0.999, 1e-8, 0.01, 1.0, 5, _s())
    lib.call("eegf_adam_consume", n, p3.data_ptr(), g3.data_ptr(), m3.data_ptr(), v3.data_ptr(), None, 1e-3, 0.9,
             0.999, 1e-8, 0.01, 1.0, 5, _s())
    torch.cuda.synchronize()
    assert torch.equal(p, p3) and torch.equal(m, m3) and torch.equal(v, v3)
    assert not bool(g3.any()) and bool(g.any())


@pytest.mark.parametrize("dt", DT)
def test_window_tokens(dt):
    lib = _lib()
    eeg = torch.randn(3, 64, 256, device="cuda")
    tok = torch.empty(3 * 256, 64, device="cuda", dtype=dt)
    lib.call("eegf_window_tokens", _code(dt), 3, 64, 256, eeg.data_ptr(), tok.data_ptr(), _s())
    torch.cuda.synchronize()
    assert torch.equal(tok, eeg.transpose(1, 2).reshape(-1, 64).to(dt))


@pytest.mark.parametrize("pdrop", [0.0, 0.1])
@pytest.mark.parametrize("mode", [1, 3])
def test_attention_l256_persistent(pdrop, mode):
    """L = 256 bf16 path with more (b, h) items than workgroups: every persistent workgroup runs
    several items (next-item K/V/Q prefetch, chunk stream across items).  mode (eegf_tune key 2):
    1 = persistent forward, 3 = persistent forward and backward (default)."""
    lib = _lib()
    lib.lib().eegf_tune.argtypes = [lib.i32, lib.i32]
    old = lib.lib().eegf_tune(2, mode)
    try:
        _attention_l256(lib, pdrop)
    finally:
        lib.lib().eegf_tune(2, old)


def _attention_l256(lib, pdrop):
    torch.manual_seed(4)
    B, L, dt = 24, 256, torch.bfloat16
    qkv = torch.randn(B, L, 2304, device="cuda").to(dt)
    out = torch.empty(B, L, 768, device="cuda", dtype=dt)
    lse = torch.empty(B, 12, L, device="cuda")
    seed, off = 123, 9
    lib.call("eegf_attn_fwd", _code(dt), B, 12, L, qkv.data_ptr(), 2304, None, 0.125, pdrop, seed, off,
             out.data_ptr(), 768, lse.data_ptr(), None, _s())
    torch.cuda.synchronize()
    qr = qkv.double().clone().requires_grad_()
    z = _attn_mask(B, L, pdrop, seed, off) if pdrop > 0 else None
    ref = _attn_ref(qr, B, L, None, z)
    assert _rel(out, ref) < _tol(dt)
    q, k, _ = qkv.double().view(B, L, 3, 12, 64).unbind(2)
    s = (q.transpose(1, 2) @ k.transpose(1, 2).transpose(-1, -2)) / 8.0
    assert (lse.double() - torch.logsumexp(s, -1)).abs().max().item() < 1e-2
    dout = torch.randn(B, L, 768, device="cuda").to(dt)
    ref.backward(dout.double())
    dqkv = torch.full_like(qkv, float("nan"))
    lib.call("eegf_attn_bwd", _code(dt), B, 12, L, qkv.data_ptr(), 2304, None, 0.125, pdrop, seed, off,
             out.data_ptr(), dout.data_ptr(), 768, lse.data_ptr(), None, dqkv.data_ptr(), None, _s())
    torch.cuda.synchronize()
    for sl, name in ((slice(0, 768), "dq"), (slice(768, 1536), "dk"), (slice(1536, 2304), "dv")):
        e = _rel(dqkv[..., sl], qr.grad[..., sl])
        assert e < _tol(dt) * 3, (name, e)


def test_colsum_batch():
    """eegf_colsum_batch: many independent column sums (fp32 / bf16 sources, strided rows, ragged
    widths) in one launch, accumulated onto dst, bitwise reproducible."""
    import struct
    lib = _lib()
    torch.manual_seed(21)
    specs = [(torch.float32, 1024, 768, 768), (torch.bfloat16, 256, 2304, 2304), (torch.float32, 37, 100, 130),
             (torch.bfloat16, 5, 1, 8), (torch.float32, 256, 2, 2),
             # 4-column vector form: ragged row counts (tails of the 64-row unroll), partial last block
             (torch.float32, 37, 100, 128), (torch.float32, 8192, 72, 72), (torch.bfloat16, 1000, 300, 304),
             (torch.bfloat16, 70, 6, 8)]
    srcs, dsts, refs, rows_d, blk = [], [], [], [], 0
    one = struct.unpack("<i", struct.pack("<f", 1.0))[0]
    for dt, rows, width, ld in specs:
        x = torch.randn(rows, ld, device="cuda").to(dt)
        d = torch.randn(width, device="cuda")
        refs.append(d.double() + x[:, :width].double().sum(0))
        srcs.append(x)
        dsts.append(d)
        rows_d.append([x.data_ptr(), d.data_ptr(), ld, rows, width | (_code(dt) << 32), one | (blk << 32)])
        blk += (width + 63) // 64
    desc = torch.tensor(rows_d, dtype=torch.int64, device="cuda")
    lib.call("eegf_colsum_batch", len(specs), desc.data_ptr(), blk, _s())
    torch.cuda.synchronize()
    for d, r in zip(dsts, refs):
        assert (d.double() - r).abs().max().item() <= 1e-4 * (1 + r.abs().max().item())
