"""GPU numerics of the MFMA GEMM (eegf_gemm) against a float64 torch reference of the same op.

Tolerances: fp32 path ≤ 1e-4·(1+|ref|) per element (exact-f32 MFMA, k-permuted summation);
bf16 path ≤ 2e-2·max|ref| (bf16 operands, fp32 accumulation).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _k():
    from eegfusion import kernels
    return kernels


def _gelu_grad(x):
    return 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5


def _ref_epi(v, epi, bias, aux, scale):
    if epi in ("bias", "bias_gelu", "bias_relu", "bias_tanh", "bias_gelu_d"):
        v = v + bias.double()
    if epi == "bias_gelu":
        return torch.nn.functional.gelu(v), v
    if epi == "bias_gelu_d":
        return torch.nn.functional.gelu(v), _gelu_grad(v)
    if epi == "mul_aux":
        return v * aux.double(), None
    if epi == "bias_relu":
        return torch.relu(v), None
    if epi == "bias_tanh":
        return torch.tanh(v), None
    if epi == "dgelu":
        x = aux.double()
        g = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
        return v * g, None
    if epi == "drelu":
        return v * (aux.double() > 0) * scale, None
    if epi == "dtanh":
        return v * (1 - aux.double() ** 2), None
    return v, None


def _check(out, ref, dt):
    out = out.double()
    if dt == torch.float32:
        err = ((out - ref).abs() / (1 + ref.abs())).max().item()
        assert err <= 1e-4, err
    else:
        err = (out - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
        assert err <= 2e-2, err


SHAPES = [(256, 768, 768), (300, 200, 96), (128, 2, 768), (64, 2304, 2304), (1000, 130, 72), (33, 17, 8)]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("layout", ["fwd", "dgrad", "wgrad", "tn"])
def test_gemm_layouts(dt, M, N, K, layout):
    k = _k()
    torch.manual_seed(0)
    dev = "cuda"
    # logical A[M,K], B[K,N]
    A = torch.randn(M, K, device=dev).to(dt)
    B = torch.randn(K, N, device=dev).to(dt)
    ref = A.double() @ B.double()
    outdt = torch.float32 if (dt == torch.float32 or layout == "wgrad") else dt
    C = torch.empty(M, N, device=dev, dtype=outdt)
    if layout == "fwd":        # A [M,K] row-major, B stored [N,K]
        Bs = B.t().contiguous()
        k.gemm(A, Bs, C, M=M, N=N, K=K, a_kc=1, b_kc=1, lda=K, ldb=K, ldc=N)
    elif layout == "dgrad":    # A [M,K], B stored [K,N]
        k.gemm(A, B.contiguous(), C, M=M, N=N, K=K, a_kc=1, b_kc=0, lda=K, ldb=N, ldc=N)
    elif layout == "wgrad":    # A stored [K,M], B stored [K,N]
        k.gemm(A.t().contiguous(), B.contiguous(), C, M=M, N=N, K=K, a_kc=0, b_kc=0, lda=M, ldb=N, ldc=N)
    else:                      # A stored [K,M], B stored [N,K]
        k.gemm(A.t().contiguous(), B.t().contiguous(), C, M=M, N=N, K=K, a_kc=0, b_kc=1, lda=M, ldb=K, ldc=N)
    torch.cuda.synchronize()
    _check(C, ref, dt if outdt != torch.float32 or dt == torch.float32 else torch.bfloat16)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("epi", ["bias", "bias_gelu", "bias_relu", "bias_tanh", "bias_gelu_d"])
def test_gemm_fwd_epilogues(dt, epi):
    k = _k()
    torch.manual_seed(1)
    M, N, K = 260, 300, 192
    x = (torch.randn(M, K, device="cuda") * 0.3).to(dt)
    w = (torch.randn(N, K, device="cuda") * 0.3).to(dt)
    b = torch.randn(N, device="cuda")
    aux = torch.empty(M, N, device="cuda", dtype=dt) if epi in ("bias_gelu", "bias_gelu_d") else None
    out = k.linear(x, w, b, epi=epi, aux=aux)
    torch.cuda.synchronize()
    ref, pre = _ref_epi(x.double() @ w.double().t(), epi, b, None, 1.0)
    _check(out, ref, dt)
    if pre is not None:
        _check(aux, pre, dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("epi", ["dgelu", "drelu", "dtanh", "mul_aux"])
def test_gemm_dgrad_epilogues(dt, epi):
    k = _k()
    torch.manual_seed(2)
    M, N, K = 260, 300, 192
    dy = torch.randn(M, N, device="cuda").to(dt)
    w = (torch.randn(N, K, device="cuda") * 0.2).to(dt)
    aux = torch.randn(M, K, device="cuda").to(dt)
    if epi == "dtanh":
        aux = torch.tanh(aux.float()).to(dt)
    out = k.linear_dgrad(dy, w, epi=epi, aux=aux, epi_scale=1.25)
    torch.cuda.synchronize()
    ref, _ = _ref_epi(dy.double() @ w.double(), epi, None, aux, 1.25)
    _check(out, ref, dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_wgrad_beta_and_batch(dt):
    k = _k()
    torch.manual_seed(3)
    M, N, K = 515, 96, 136
    dy = torch.randn(M, N, device="cuda").to(dt)
    x = torch.randn(M, K, device="cuda").to(dt)
    dw = torch.randn(N, K, device="cuda")
    ref = dw.double() * 0.5 + dy.double().t() @ x.double()
    k.linear_wgrad(dy, x, dw, beta=0.5)
    torch.cuda.synchronize()
    _check(dw, ref, dt)
    # batched (z) strided: 3 independent products
    Z = 3
    A = torch.randn(Z, 70, 64, device="cuda").to(dt)
    B = torch.randn(Z, 50, 64, device="cuda").to(dt)
    C = torch.empty(Z, 70, 50, device="cuda", dtype=torch.float32 if dt == torch.float32 else dt)
    k.gemm(A, B, C, M=70, N=50, K=64, a_kc=1, b_kc=1, lda=64, ldb=64, ldc=50, batch=Z,
           sA=70 * 64, sB=50 * 64, sC=70 * 50)
    torch.cuda.synchronize()
    _check(C, A.double() @ B.double().transpose(1, 2), dt)


@pytest.mark.parametrize("akc,bkc", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_gemm_batched_splitk(akc, bkc, beta):
    """Batched plain fp32 GEMMs on an under-filled grid split K (slabs [split][batch][M][N] and a batched
    fixed-order reduction): the decoder's per-head dq[b, h 64 + i] = sum_c dqp[b, h, c] Wk[h 64 + i, c],
    C batches as column blocks of one row-major matrix (strideC = 64, ldc = 768)."""
    k = _k()
    torch.manual_seed(9)
    Z, M, N, K = 12, 256, 64, 768
    A = torch.randn(Z, M, K, device="cuda") if akc else torch.randn(Z, K, M, device="cuda")
    B = torch.randn(Z, N, K, device="cuda") if bkc else torch.randn(Z, K, N, device="cuda")
    C = torch.randn(M, Z * N, device="cuda")
    ref = (A.double() if akc else A.double().transpose(1, 2)) @ (B.double().transpose(1, 2) if bkc else B.double())
    ref = ref.permute(1, 0, 2).reshape(M, Z * N) + beta * C.double()
    ws = torch.empty(16 << 20, device="cuda")
    k.gemm(A, B, C, M=M, N=N, K=K, a_kc=akc, b_kc=bkc, lda=K if akc else M, ldb=K if bkc else N, ldc=Z * N,
           beta=beta, batch=Z, sA=M * K, sB=N * K, sC=N, workspace=ws)
    torch.cuda.synchronize()
    err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
    assert err <= 1e-5, err


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(768, 768, 16384), (2304, 768, 8192), (300, 200, 9000)])
def test_gemm_wgrad_splitk(dt, M, N, K):
    """Split-K path (under-filled grid, long contraction): fixed-order fp32 slab reduction + beta."""
    k = _k()
    torch.manual_seed(6)
    dy = torch.randn(K, M, device="cuda").to(dt)
    x = torch.randn(K, N, device="cuda").to(dt)
    dw = torch.randn(M, N, device="cuda")
    ref = dw.double() * 0.5 + dy.double().t() @ x.double()
    ws = torch.empty(64 << 20, device="cuda")
    k.gemm(dy, x, dw, M=M, N=N, K=K, a_kc=0, b_kc=0, lda=M, ldb=N, ldc=N, beta=0.5, workspace=ws)
    torch.cuda.synchronize()
    # long fp32 contraction: error relative to the output scale (sqrt(K) growth of fp32 rounding)
    err = ((dw.double() - ref).abs().max() / ref.abs().max()).item()
    assert err <= (1e-5 if dt == torch.float32 else 2e-2), err
    dw2 = torch.empty(M, N, device="cuda")
    k.gemm(dy, x, dw2, M=M, N=N, K=K, a_kc=0, b_kc=0, lda=M, ldb=N, ldc=N, workspace=ws)
    dw3 = torch.empty(M, N, device="cuda")
    k.gemm(dy, x, dw3, M=M, N=N, K=K, a_kc=0, b_kc=0, lda=M, ldb=N, ldc=N, workspace=ws)
    torch.cuda.synchronize()
    assert torch.equal(dw2, dw3)          # deterministic


@pytest.mark.parametrize("epi", ["none", "bias", "bias_gelu", "bias_relu", "bias_tanh", "bias_gelu_d", "gelu_noaux"])
@pytest.mark.parametrize("M,N,K", [(4352, 808, 768), (2048, 2304, 256)])
def test_gemm_big_fwd(epi, M, N, K):
    """256x256 glds-pipelined bf16 kernel (M >= 2048), including M/N edge tiles."""
    k = _k()
    torch.manual_seed(7)
    x = (torch.randn(M, K, device="cuda") * 0.3).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.3).to(torch.bfloat16)
    b = torch.randn(N, device="cuda") if epi != "none" else None
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if epi in ("bias_gelu", "bias_gelu_d") else None
    if epi == "gelu_noaux":      # BIAS_GELU without the pre-activation output (forward-only passes)
        epi = "bias_gelu"
        out = k.linear(x, w, b, epi=epi, aux=None)
        torch.cuda.synchronize()
        _check(out, _ref_epi(x.double() @ w.double().t(), epi, b, None, 1.0)[0], torch.bfloat16)
        return
    out = k.linear(x, w, b, epi=epi, aux=aux)
    torch.cuda.synchronize()
    ref, pre = _ref_epi(x.double() @ w.double().t(), epi, b, None, 1.0)
    _check(out, ref, torch.bfloat16)
    if pre is not None:
        _check(aux, pre, torch.bfloat16)


@pytest.mark.parametrize("epi", ["none", "dgelu", "drelu", "dtanh", "mul_aux"])
@pytest.mark.parametrize("M,N,K", [(4352, 808, 768), (2048, 3072, 320)])
def test_gemm_big_dgrad(epi, M, N, K):
    k = _k()
    torch.manual_seed(8)
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)          # [M, N_out=K]
    w = (torch.randn(K, N, device="cuda") * 0.2).to(torch.bfloat16)   # weight [N_out, N_in]
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi != "none" else None
    if epi == "dtanh":
        aux = torch.tanh(aux.float()).to(torch.bfloat16)
    out = k.linear_dgrad(dy, w, epi=epi, aux=aux, epi_scale=1.25)
    torch.cuda.synchronize()
    ref, _ = _ref_epi(dy.double() @ w.double(), epi, None, aux, 1.25)
    _check(out, ref, torch.bfloat16)


@pytest.mark.parametrize("epi", ["bias", "bias_gelu", "bias_relu", "bias_tanh", "dgelu", "drelu", "dtanh", "none",
                                 "bias_gelu_d", "mul_aux"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("K", [2304, 768])
def test_gemm_small_m_splitk_epilogues(dt, epi, K):
    """Batch-row GEMMs (M = B) take split-K with the epilogue applied in the slab reduction."""
    k = _k()
    torch.manual_seed(10)
    M, N = 256, 768
    ws = torch.empty(8 << 20, device="cuda")
    x = (torch.randn(M, K, device="cuda") * 0.2).to(dt)
    if epi.startswith("bias") or epi == "none":
        w = (torch.randn(N, K, device="cuda") * 0.2).to(dt)
        b = torch.randn(N, device="cuda")
        aux = torch.empty(M, N, device="cuda", dtype=dt) if epi in ("bias_gelu", "bias_gelu_d") else None
        out = torch.empty(M, N, device="cuda", dtype=dt)
        k.gemm(x, w, out, M=M, N=N, K=K, a_kc=1, b_kc=1, lda=K, ldb=K, ldc=N, epi=epi, bias=b if epi != "none" else None,
               aux=aux, ldaux=N, workspace=ws)
        torch.cuda.synchronize()
        ref, pre = _ref_epi(x.double() @ w.double().t(), epi, b, None, 1.0)
        _check(out, ref, dt)
        if pre is not None:
            _check(aux, pre, dt)
    else:
        w = (torch.randn(K, N, device="cuda") * 0.2).to(dt)
        aux = torch.randn(M, N, device="cuda").to(dt)
        if epi == "dtanh":
            aux = torch.tanh(aux.float()).to(dt)
        out = torch.empty(M, N, device="cuda", dtype=dt)
        k.gemm(x, w, out, M=M, N=N, K=K, a_kc=1, b_kc=0, lda=K, ldb=N, ldc=N, epi=epi, aux=aux, ldaux=N,
               epi_scale=1.25, workspace=ws)
        torch.cuda.synchronize()
        ref, _ = _ref_epi(x.double() @ w.double(), epi, None, aux, 1.25)
        _check(out, ref, dt)


@pytest.mark.parametrize("M,N,K", [(2304, 768, 65536), (768, 3072, 16384), (768, 768, 8192)])
def test_gemm_big_wgrad_splitk(M, N, K):
    """Weight gradients on the 256x256 kernel (k-major A and B), split-K slabs, beta accumulate."""
    k = _k()
    torch.manual_seed(11)
    dy = torch.randn(K, M, device="cuda").to(torch.bfloat16)
    x = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    dw = torch.randn(M, N, device="cuda")
    ref = dw.double() + dy.double().t() @ x.double()
    ws = torch.empty(24 << 20, device="cuda")
    k.gemm(dy, x, dw, M=M, N=N, K=K, a_kc=0, b_kc=0, lda=M, ldb=N, ldc=N, beta=1.0, workspace=ws)
    torch.cuda.synchronize()
    err = ((dw.double() - ref).abs().max() / ref.abs().max()).item()
    assert err <= 2e-3, err


@pytest.mark.parametrize("M,N,K", [(4096, 768, 3072), (4096, 2304, 768)])
def test_gemm_big_dgrad_beta(M, N, K):
    """Input gradient accumulated onto the residual gradient (beta = 1) on the 256x256 kernel."""
    k = _k()
    torch.manual_seed(12)
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
    c = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    ref = c.double() + dy.double() @ w.double()
    k.linear_dgrad(dy, w, out=c, beta=1.0)
    torch.cuda.synchronize()
    _check(c, ref, torch.bfloat16)


def _tune(key, value):
    from eegfusion import _lib
    lib = _lib.lib()
    lib.eegf_tune.argtypes = [_lib.i32, _lib.i32]
    return lib.eegf_tune(key, value)


# (M, N, K): 768 tiles, 260 ragged tiles with a ragged N, a short K (2 K-tiles), an odd K-tile count
ROUTE_SHAPES = [(16384, 3072, 768), (16640, 808, 320), (16384, 1024, 128), (8192, 2304, 192)]


@pytest.mark.parametrize("epi", ["bias", "bias_gelu", "bias_gelu_d", "gelu_noaux", "none_beta"])
@pytest.mark.parametrize("M,N,K", ROUTE_SHAPES)
def test_gemm_big_routed_fwd(epi, M, N, K):
    """Forward GEMMs with every bf16 epilogue through the default routing (the persistent kernels on full
    tiles, the 4-wave gemm4w on ragged ones) against a float64 reference."""
    k = _k()
    torch.manual_seed(21)
    x = (torch.randn(M, K, device="cuda") * 0.3).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.3).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    if epi == "none_beta":
        c = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        ref = c.double() + 0.5 * (x.double() @ w.double().t())
        k.gemm(x, w, c, M=M, N=N, K=K, a_kc=1, b_kc=1, lda=K, ldb=K, ldc=N, alpha=0.5, beta=1.0)
        torch.cuda.synchronize()
        _check(c, ref, torch.bfloat16)
        return
    e = "bias_gelu" if epi == "gelu_noaux" else epi
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if epi in ("bias_gelu", "bias_gelu_d") else None
    out = k.linear(x, w, b, epi=e, aux=aux)
    torch.cuda.synchronize()
    ref, pre = _ref_epi(x.double() @ w.double().t(), e, b, None, 1.0)
    _check(out, ref, torch.bfloat16)
    if aux is not None:
        _check(aux, pre, torch.bfloat16)


@pytest.mark.parametrize("epi", ["none", "mul_aux", "dgelu"])
@pytest.mark.parametrize("M,N,K", ROUTE_SHAPES)
def test_gemm_big_routed_dgrad(epi, M, N, K):
    """Input-gradient GEMMs through the default routing against a float64 reference, and bit for bit
    against the non-persistent gemm4w (eegf_tune key 11 = 0: the same MFMA K order and epilogue math)."""
    k = _k()
    torch.manual_seed(22)
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi != "none" else None
    outs = []
    for key in (1, 0):
        old = _tune(11, key)
        try:
            outs.append(k.linear_dgrad(dy, w, epi=epi, aux=aux))
            torch.cuda.synchronize()
        finally:
            _tune(11, old)
    ref, _ = _ref_epi(dy.double() @ w.double(), epi, None, aux, 1.0)
    _check(outs[0], ref, torch.bfloat16)
    if K >= 256:
        assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("epi", ["none", "bias", "bias_gelu", "bias_gelu_d", "gelu_noaux", "none_beta"])
@pytest.mark.parametrize("M,N,K", [(4352, 808, 768), (2048, 2304, 96), (8192, 3072, 32), (16384, 768, 3072)])
def test_gemm_big_4wave_fwd(epi, M, N, K):
    """The 4-wave 256x256 kernel gemm4w (128x128 per wave, AGPR accumulators, BK = 32 ring) on the forward
    layout, every shape on it with eegf_tune(11, 0): edge tiles, K = one K-tile, odd K-tile counts."""
    k = _k()
    old = _tune(11, 0)
    try:
        torch.manual_seed(23)
        x = (torch.randn(M, K, device="cuda") * 0.3).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.3).to(torch.bfloat16)
        b = torch.randn(N, device="cuda")
        if epi in ("none", "none_beta"):
            c = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            beta = 1.0 if epi == "none_beta" else 0.0
            ref = beta * c.double() + 0.5 * (x.double() @ w.double().t())
            k.gemm(x, w, c, M=M, N=N, K=K, a_kc=1, b_kc=1, lda=K, ldb=K, ldc=N, alpha=0.5, beta=beta)
            torch.cuda.synchronize()
            _check(c, ref, torch.bfloat16)
            return
        e = "bias_gelu" if epi == "gelu_noaux" else epi
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if epi in ("bias_gelu", "bias_gelu_d") else None
        out = k.linear(x, w, b, epi=e, aux=aux)
        torch.cuda.synchronize()
        ref, pre = _ref_epi(x.double() @ w.double().t(), e, b, None, 1.0)
        _check(out, ref, torch.bfloat16)
        if aux is not None:
            _check(aux, pre, torch.bfloat16)
    finally:
        _tune(11, old)


@pytest.mark.parametrize("epi", ["none", "mul_aux", "dgelu"])
@pytest.mark.parametrize("M,N,K", [(4352, 808, 768), (2048, 3072, 96), (8192, 768, 2304)])
def test_gemm_big_4wave_dgrad(epi, M, N, K):
    """gemm4w with a k-major B (input gradient, ds_read_b64_tr_b16 fragments)."""
    k = _k()
    old = _tune(11, 0)
    try:
        torch.manual_seed(24)
        dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
        aux = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi != "none" else None
        out = k.linear_dgrad(dy, w, epi=epi, aux=aux)
        torch.cuda.synchronize()
        ref, _ = _ref_epi(dy.double() @ w.double(), epi, None, aux, 1.0)
        _check(out, ref, torch.bfloat16)
    finally:
        _tune(11, old)


@pytest.mark.parametrize("M,N,K", [(2304, 768, 65536), (768, 3072, 16384), (808, 264, 8192)])
def test_gemm_big_4wave_wgrad(M, N, K):
    """gemm4w with k-major A and B (weight gradient), fp32 split-K slabs, beta accumulate, ragged M / N."""
    k = _k()
    torch.manual_seed(25)
    dy = torch.randn(K, M, device="cuda").to(torch.bfloat16)
    x = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    dw = torch.randn(M, N, device="cuda")
    ref = dw.double() + dy.double().t() @ x.double()
    ws = torch.empty(24 << 20, device="cuda")
    k.gemm(dy, x, dw, M=M, N=N, K=K, a_kc=0, b_kc=0, lda=M, ldb=N, ldc=N, beta=1.0, workspace=ws)
    torch.cuda.synchronize()
    err = ((dw.double() - ref).abs().max() / ref.abs().max()).item()
    assert err <= 2e-3, err


@pytest.mark.parametrize("M,N,K,ws_mb", [(2304, 768, 65536, 96), (3072, 768, 65536, 96), (768, 3072, 65536, 96),
                                         (768, 768, 4096, 96), (2312, 776, 8192, 96), (768, 768, 8192, 2)])
def test_gemm_wgrad_bias(M, N, K, ws_mb):
    """eegf_gemm_wgrad_bias: weight gradient dY^T X (+ dW, beta 1) with the bias gradient dY.sum(0)
    summed by the same kernel (ones-operand MFMAs in tile column 0), split-K slabs (ws 96 MB) and one
    slice (ws 2 MB), ragged M / N, fixed-order reductions (bitwise repeatable)."""
    from eegfusion import _lib
    torch.manual_seed(5)
    dy = torch.randn(K, M, device="cuda").to(torch.bfloat16)           # [tokens, out features]
    x = torch.randn(K, N, device="cuda").to(torch.bfloat16)            # [tokens, in features]
    dw0 = torch.randn(M, N, device="cuda")
    db0 = torch.randn(M, device="cuda")
    ws = torch.empty(ws_mb << 18, device="cuda")
    outs = []
    for _ in range(2):
        dw, db = dw0.clone(), db0.clone()
        _lib.call("eegf_gemm_wgrad_bias", _lib.BF16, M, N, K, dy.data_ptr(), M, x.data_ptr(), N, dw.data_ptr(), N,
                  1.0, db.data_ptr(), ws.data_ptr(), ws.numel() * 4, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append((dw, db))
    ref = dy.double().t() @ x.double() + dw0.double()
    err_w = ((outs[0][0].double() - ref).abs().max() / ref.abs().max()).item()
    assert err_w < 2e-5, err_w                        # fp32 accumulation of exact bf16 products
    bref = dy.double().sum(0) + db0.double()
    err_b = ((outs[0][1].double() - bref).abs().max() / bref.abs().max()).item()
    assert err_b < 2e-5, err_b
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_gemm_wgrad_bias_ineligible():
    """shapes off the 4-wave path return EEGF_ERR_ARG without launching (the engine then runs the
    plain GEMM and a column reduction)."""
    from eegfusion import _lib
    dy = torch.zeros(2048, 768, device="cuda", dtype=torch.bfloat16)
    x = torch.zeros(2048, 768, device="cuda", dtype=torch.bfloat16)
    dw = torch.zeros(768, 768, device="cuda")
    db = torch.zeros(768, device="cuda")
    ws = torch.empty(1 << 20, device="cuda")
    st = _lib.lib().eegf_gemm_wgrad_bias(_lib.BF16, 768, 768, 2048, dy.data_ptr(), 768, x.data_ptr(), 768,
                                         dw.data_ptr(), 768, 1.0, db.data_ptr(), ws.data_ptr(), ws.numel() * 4,
                                         torch.cuda.current_stream().cuda_stream)
    assert st == _lib.ERR_ARG                           # K = 2048 tokens < 4096
    st = _lib.lib().eegf_gemm_wgrad_bias(_lib.F32, 768, 768, 8192, dy.data_ptr(), 768, x.data_ptr(), 768,
                                         dw.data_ptr(), 768, 1.0, db.data_ptr(), ws.data_ptr(), ws.numel() * 4,
                                         torch.cuda.current_stream().cuda_stream)
    assert st == _lib.ERR_ARG


# the persistent kernel (eegf_tune key 11): full tiles only; production-sized grids loop several rounds,
# K below the ring depth (3 and 1 K-tiles) prefetches fewer K-tiles, a 24-tile grid runs one round
# nk = K / 32 K-tiles: 24, 24, 3, 1, 96, and the ring-edge cases 5..7 (a full 5-slot ring, no cross-tile
# staging) and 8 (the first cross-staged shape: the next tile's K-tiles 0..4 landed before it starts),
# each with three rounds per CU on a 256-CU grid (768 tiles)
# K = 128 / 320: gemm4r with 2 / 5 K-tile pairs per tile (its 3 + 2 operand slots advance np mod 3 /
# mod 2 per tile), several tiles per CU
P_SHAPES = [(65536, 2304, 768), (4096, 768, 768), (8192, 3072, 96), (2048, 1024, 32), (16384, 768, 3072),
            (16384, 3072, 160), (16384, 3072, 192), (16384, 3072, 224), (16384, 3072, 256), (16384, 3072, 128),
            (16384, 3072, 320)]


@pytest.mark.parametrize("epi", ["bias", "bias_gelu", "bias_gelu_d", "gelu_noaux", "none"])
@pytest.mark.parametrize("M,N,K", P_SHAPES)
def test_gemm_persistent_fwd(epi, M, N, K):
    """The persistent kernels (next tile's K-tiles staged under the epilogue, direct stores) on the
    forward layout against a float64 reference, gemm4r bit for bit against gemm4p, and both against the
    non-persistent gemm4w (the same MFMA K-order and the same epilogue arithmetic)."""
    k = _k()
    torch.manual_seed(26)
    x = (torch.randn(M, K, device="cuda") * 0.3).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.3).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    e = "bias_gelu" if epi == "gelu_noaux" else epi
    outs = []
    # (key 11, key 14): persistent gemm4r (default; gemm4p where K % 64 != 0), gemm4w, persistent gemm4p
    for k11, k14 in ((1, 1), (0, 1), (1, 0)):
        old, old14 = _tune(11, k11), _tune(14, k14)
        try:
            aux = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16) \
                if epi in ("bias_gelu", "bias_gelu_d") else None
            out = k.linear(x, w, None if epi == "none" else b, epi=e, aux=aux)
            torch.cuda.synchronize()
            outs.append((out, aux))
        finally:
            _tune(11, old)
            _tune(14, old14)
    # gemm4r and gemm4p: the same MFMA K order and epilogue, bit for bit
    assert torch.equal(outs[0][0], outs[2][0])
    if outs[0][1] is not None:
        assert torch.equal(outs[0][1], outs[2][1])
    out, aux = outs[0]
    ref, pre = _ref_epi(x.double() @ w.double().t(), e, None if epi == "none" else b, None, 1.0)
    _check(out, ref, torch.bfloat16)
    if aux is not None:
        _check(aux, pre, torch.bfloat16)
    if K >= 256:      # the default routing's kernels share the K order from here on (BK 32 / 64 alike)
        assert torch.equal(out, outs[1][0])
        if aux is not None:
            assert torch.equal(aux, outs[1][1])


@pytest.mark.parametrize("epi", ["none", "mul_aux", "none_beta"])
@pytest.mark.parametrize("M,N,K", P_SHAPES)
def test_gemm_persistent_dgrad(epi, M, N, K):
    """The persistent kernels with a k-major B (input gradient), with the input-tile epilogues (aux product,
    beta = 1 residual accumulate: the tile read in the widened store layout and swapped back), against a
    float64 reference, gemm4r against gemm4p and both against gemm4w (key 11 = 0), bit for bit."""
    k = _k()
    torch.manual_seed(27)
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "mul_aux" else None
    c0 = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    outs = []
    # (key 11, key 14): gemm4r (default), gemm4w, gemm4p
    for k11, k14 in ((1, 1), (0, 1), (1, 0)):
        old, old14 = _tune(11, k11), _tune(14, k14)
        try:
            if epi == "none_beta":
                out = c0.clone()
                k.linear_dgrad(dy, w, out=out, beta=1.0)
            else:
                out = k.linear_dgrad(dy, w, epi=epi, aux=aux)
            torch.cuda.synchronize()
            outs.append(out)
        finally:
            _tune(11, old)
            _tune(14, old14)
    assert torch.equal(outs[0], outs[2])          # gemm4r with a k-major B == gemm4p bit for bit
    if epi == "none_beta":
        ref = c0.double() + dy.double() @ w.double()
    else:
        ref, _ = _ref_epi(dy.double() @ w.double(), epi, None, aux, 1.0)
    _check(outs[0], ref, torch.bfloat16)
    if K >= 256:
        assert torch.equal(outs[0], outs[1])


def test_gemm_persistent_falls_back_on_ragged_shapes():
    """N % 256 != 0: the persistent kernels leave the shape to gemm4w whatever key 11 says (same results)."""
    k = _k()
    torch.manual_seed(28)
    M, N, K = 4352, 808, 768
    x = (torch.randn(M, K, device="cuda") * 0.3).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.3).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    outs = []
    for key in (1, 0):
        old = _tune(11, key)
        try:
            outs.append(k.linear(x, w, b, epi="bias"))
            torch.cuda.synchronize()
        finally:
            _tune(11, old)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M,N,K", P_SHAPES)
@pytest.mark.parametrize("epi", ["bias", "none", "mul_aux", "none_beta", "bias_gelu_d"])
def test_gemm_persistent_ring_variants(epi, M, N, K):
    """eegf_tune key 14: gemm4p (0: 64-B half-line K-tiles, five-slot ring) and gemm4r (1, default: whole-
    line K-tile pairs, rolling A fragments in a 3 + 2 slot ring, two barriers per pair) give the same bits on
    every persistent shape and epilogue (pair counts np = K / 64 of 2..48; the cross-tile staging of both
    rings)."""
    k = _k()
    torch.manual_seed(29)
    fwd = epi in ("bias", "bias_gelu_d")      # the others on the input-gradient layout (k-major B)
    x = (torch.randn(M, K, device="cuda") * 0.3).to(torch.bfloat16)
    wf = (torch.randn(N, K, device="cuda") * 0.3).to(torch.bfloat16)
    wd = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "mul_aux" else None
    c0 = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    outs = []
    for key in (0, 1):
        old = _tune(14, key)
        try:
            if epi == "none_beta":
                out = c0.clone()
                k.linear_dgrad(x, wd, out=out, beta=1.0)
                out = (out,)
            elif not fwd:
                out = (k.linear_dgrad(x, wd, epi=epi, aux=aux),)
            else:
                a2 = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16) \
                    if epi == "bias_gelu_d" else None
                out = (k.linear(x, wf, None if epi == "none" else b, epi=epi, aux=a2), a2)
            torch.cuda.synchronize()
            outs.append(out)
        finally:
            _tune(14, old)
    for o in outs[1:]:
        for a, r in zip(o, outs[0]):
            if r is not None:
                assert torch.equal(a, r)
