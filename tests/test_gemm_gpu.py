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
def test_gemm_small_m_splitk_epilogues(dt, epi):
    """Batch-row GEMMs (M = B) take split-K with the epilogue applied in the slab reduction."""
    k = _k()
    torch.manual_seed(10)
    M, N, K = 256, 768, 2304
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


@pytest.mark.parametrize("epi", ["none", "dgelu"])
@pytest.mark.parametrize("M,N,K,beta", [(4352, 808, 768, 0.0), (2056, 768, 3072, 1.0), (4096, 768, 2304, 1.0),
                                        (16648, 808, 2304, 0.0), (4104, 3072, 3072, 1.0)])
def test_gemm_acs_fused_bias_grad(epi, M, N, K, beta):
    if epi == "dgelu":
        beta = 0.0          # activation-derivative epilogues read aux in place of C (beta must be 0)
    """eegf_gemm_acs: the input-gradient GEMM plus per-256-row-tile column sums of dY (the fused
    bias gradient); ragged M (tiles past M excluded), beta accumulate, epilogue."""
    from eegfusion import _lib
    torch.manual_seed(13)
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)          # [M, N_out=K]
    w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)   # [N_out, N_in]
    c = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "dgelu" else None
    c0 = c.double().clone()
    tiles = _lib.lib().eegf_gemm_colsum_tiles(1, 1, 1, M, N, K)
    assert tiles == (M + 255) // 256
    part = torch.full((tiles, K), float("nan"), device="cuda")
    _lib.call("eegf_gemm_acs", 1, 1, 1, 0, _lib.EPI_DGELU if epi == "dgelu" else _lib.EPI_NONE, M, N, K,
              dy.data_ptr(), K, w.data_ptr(), N, c.data_ptr(), N, None,
              aux.data_ptr() if aux is not None else None, N if aux is not None else 0, 1.0, beta, 1.0,
              part.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref, _ = _ref_epi(dy.double() @ w.double(), epi, None, aux, 1.0)
    _check(c, ref + beta * c0, torch.bfloat16)
    pref = torch.nn.functional.pad(dy.double(), (0, 0, 0, tiles * 256 - M)).view(tiles, 256, K).sum(1)
    assert ((part.double() - pref).abs().max() / pref.abs().max()).item() < 1e-5
    assert _lib.lib().eegf_gemm_colsum_tiles(0, 0, 1, M, N, K) == 0      # fp32: not fused


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
    """Forward GEMMs with every bf16 epilogue through the default routing (8-phase 256x256 kernel for
    wide N, 256x128 two-workgroup kernel for N <= 768) against a float64 reference."""
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
def test_gemm_big_routed_dgrad_colsum(epi, M, N, K):
    """Input-gradient GEMM with fused dY column sums (per-tile sums of the column-0 tiles, 8-phase
    kernel) and without the sums (default routing), same result bit for bit."""
    from eegfusion import _lib
    torch.manual_seed(22)
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi != "none" else None
    code = {"none": _lib.EPI_NONE, "mul_aux": _lib.EPI_MUL_AUX, "dgelu": _lib.EPI_DGELU}[epi]
    tiles = (M + 255) // 256
    part = torch.full((tiles, K), float("nan"), device="cuda")
    _lib.call("eegf_gemm_acs", 1, 1, 1, 0, code, M, N, K, dy.data_ptr(), K, w.data_ptr(), N, c.data_ptr(), N,
              None, aux.data_ptr() if aux is not None else None, N if aux is not None else 0, 1.0, 0.0, 1.0,
              part.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref, _ = _ref_epi(dy.double() @ w.double(), epi, None, aux, 1.0)
    _check(c, ref, torch.bfloat16)
    pref = torch.nn.functional.pad(dy.double(), (0, 0, 0, tiles * 256 - M)).view(tiles, 256, K).sum(1)
    assert ((part.double() - pref).abs().max() / pref.abs().max()).item() < 1e-5
    k_out = _k().linear_dgrad(dy, w, epi=epi, aux=aux)
    torch.cuda.synchronize()
    assert torch.equal(k_out, c)


@pytest.mark.parametrize("epi", ["none", "bias", "bias_gelu", "bias_gelu_d", "gelu_noaux", "none_beta"])
@pytest.mark.parametrize("M,N,K", [(4352, 808, 768), (2048, 2304, 96), (8192, 3072, 32), (16384, 768, 3072)])
def test_gemm_big_4wave_fwd(epi, M, N, K):
    """The 4-wave 256x256 kernel (128x128 per wave, AGPR accumulators, BK = 32 ring) on the forward
    layout, selected with eegf_tune(1, 6): edge tiles, K = one K-tile, odd K-tile counts."""
    k = _k()
    old = _tune(1, 6)
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
        _tune(1, old)


@pytest.mark.parametrize("epi", ["none", "mul_aux", "dgelu"])
@pytest.mark.parametrize("M,N,K", [(4352, 808, 768), (2048, 3072, 96), (8192, 768, 2304)])
def test_gemm_big_4wave_dgrad(epi, M, N, K):
    """4-wave kernel with a k-major B (input gradient, ds_read_b64_tr_b16 fragments)."""
    k = _k()
    old = _tune(1, 6)
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
        _tune(1, old)


@pytest.mark.parametrize("M,N,K", [(2304, 768, 65536), (768, 3072, 16384), (808, 264, 8192)])
def test_gemm_big_4wave_wgrad(M, N, K):
    """4-wave kernel with k-major A and B (weight gradient), fp32 split-K slabs, beta accumulate."""
    k = _k()
    old = _tune(1, 6)
    try:
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
    finally:
        _tune(1, old)


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


@pytest.mark.parametrize("epi", ["none", "bias", "bias_gelu", "bias_gelu_d", "gelu_noaux", "bias_relu", "bias_tanh",
                                 "none_beta"])
@pytest.mark.parametrize("M,N,K", [(4352, 808, 768), (2048, 2304, 96), (8192, 3072, 32), (65536, 3072, 768)])
def test_gemm_4h_fwd(epi, M, N, K):
    """The 256x128 two-workgroups-per-CU kernel (eegf_tune key 8) on the forward layout: N / M edge
    tiles, K = one K-tile, the bench's FFN1 shape with every epilogue."""
    k = _k()
    old = _tune(8, 1)
    try:
        torch.manual_seed(31)
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
        _tune(8, old)


@pytest.mark.parametrize("epi", ["none", "mul_aux", "dgelu", "drelu", "dtanh"])
@pytest.mark.parametrize("M,N,K", [(4352, 808, 768), (2048, 3072, 96), (65536, 3072, 768), (65536, 768, 768)])
def test_gemm_4h_dgrad(epi, M, N, K):
    """256x128 kernel with a k-major B (input gradient, transpose-read fragments of a 128-column image)."""
    k = _k()
    old = _tune(8, 1)
    try:
        torch.manual_seed(32)
        dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
        aux = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi != "none" else None
        if epi == "dtanh":
            aux = torch.tanh(aux.float()).to(torch.bfloat16)
        out = k.linear_dgrad(dy, w, epi=epi, aux=aux, epi_scale=1.25)
        torch.cuda.synchronize()
        ref, _ = _ref_epi(dy.double() @ w.double(), epi, None, aux, 1.25)
        _check(out, ref, torch.bfloat16)
    finally:
        _tune(8, old)



# the persistent kernel (eegf_tune key 11): full tiles only; production-sized grids loop several rounds,
# K below the ring depth (3 and 1 K-tiles) prefetches fewer K-tiles, a 24-tile grid runs one round
# nk = K / 32 K-tiles: 24, 24, 3, 1, 96, and the ring-edge cases 5..7 (a full 5-slot ring, no cross-tile
# staging) and 8 (the first cross-staged shape: the next tile's K-tiles 0..4 landed before it starts),
# each with three rounds per CU on a 256-CU grid (768 tiles)
# K = 128 / 320: gemm4q with 2 / 5 K-tile pairs per tile (its five operand slots advance 2 np mod 5 per
# tile: 4 and 0), several tiles per CU
P_SHAPES = [(65536, 2304, 768), (4096, 768, 768), (8192, 3072, 96), (2048, 1024, 32), (16384, 768, 3072),
            (16384, 3072, 160), (16384, 3072, 192), (16384, 3072, 224), (16384, 3072, 256), (16384, 3072, 128),
            (16384, 3072, 320)]


@pytest.mark.parametrize("epi", ["bias", "bias_gelu", "bias_gelu_d", "gelu_noaux", "none"])
@pytest.mark.parametrize("M,N,K", P_SHAPES)
def test_gemm_persistent_fwd(epi, M, N, K):
    """gemm4p_kernel (persistent, next tile's K-tiles staged under the epilogue, direct stores) on the
    forward layout against a float64 reference, and bit for bit against the default routing (the same
    MFMA K-order and the same epilogue arithmetic)."""
    k = _k()
    torch.manual_seed(26)
    x = (torch.randn(M, K, device="cuda") * 0.3).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.3).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    e = "bias_gelu" if epi == "gelu_noaux" else epi
    outs = []
    # (key 11, key 14): persistent with whole-line staging (gemm4q), non-persistent, persistent gemm4p
    for k11, k14 in ((1, 2), (0, 2), (1, 0)):
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
    # gemm4q and gemm4p: the same MFMA K order and epilogue, bit for bit
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
    """gemm4p_kernel with a k-major B (input gradient), with the input-tile epilogues (aux product, beta = 1
    residual accumulate: the tile read in the widened store layout and swapped back), against a float64
    reference and bit for bit against the default routing (key 11 = 0)."""
    k = _k()
    torch.manual_seed(27)
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "mul_aux" else None
    c0 = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    outs = []
    # (key 11, key 14): forward-only gemm4q (so gemm4p here), non-persistent, gemm4p, gemm4q (default)
    for k11, k14 in ((1, 1), (0, 1), (1, 0), (1, 2)):
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
    assert torch.equal(outs[0], outs[2])          # gemm4p (key 14 = 1) == gemm4p (key 14 = 0)
    assert torch.equal(outs[0], outs[3])          # gemm4q with a k-major B == gemm4p bit for bit
    if epi == "none_beta":
        ref = c0.double() + dy.double() @ w.double()
    else:
        ref, _ = _ref_epi(dy.double() @ w.double(), epi, None, aux, 1.0)
    _check(outs[0], ref, torch.bfloat16)
    if K >= 256:
        assert torch.equal(outs[0], outs[1])


def test_gemm_persistent_falls_back_on_ragged_shapes():
    """N % 256 != 0 / beta != 0: key 11 leaves those shapes on the other kernels (same results)."""
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
    """eegf_tune key 18: gemm4q (0) and gemm4r (1, default: rolling A fragments in a 3 + 2 slot ring, two
    barriers per K-tile pair) give the same bits on every persistent shape and epilogue (pair counts
    np = K / 64 of 2..48; the cross-tile staging of both rings)."""
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
        old = _tune(18, key)
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
            _tune(18, old)
    for o in outs[1:]:
        for a, r in zip(o, outs[0]):
            if r is not None:
                assert torch.equal(a, r)
