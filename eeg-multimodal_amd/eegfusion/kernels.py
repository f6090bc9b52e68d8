"""Thin, checked host wrappers over the C-ABI (one per kernel family).

Each wrapper validates device/dtype/shape/contiguity on the host, converts tensors to raw
pointers and enqueues on ``torch.cuda.current_stream()``.  PyTorch is plumbing here (device
memory and streams); every FLOP runs in ``libeegfusion.so``.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import BF16, F32, call

EPI = dict(none=_lib.EPI_NONE, bias=_lib.EPI_BIAS, bias_gelu=_lib.EPI_BIAS_GELU,
           bias_relu=_lib.EPI_BIAS_RELU, bias_tanh=_lib.EPI_BIAS_TANH, dgelu=_lib.EPI_DGELU,
           drelu=_lib.EPI_DRELU, dtanh=_lib.EPI_DTANH, bias_gelu_d=_lib.EPI_BIAS_GELU_D,
           mul_aux=_lib.EPI_MUL_AUX)


def code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise RuntimeError(f"unsupported dtype {t.dtype}")


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("eegfusion kernels take device tensors only (no CPU fallback)")
    return t.data_ptr()


def _req(cond: bool, msg: str) -> None:
    if not cond:
        raise RuntimeError(msg)


# ----------------------------------------------------------------------------------- GEMM
def gemm(A, B, C, *, M, N, K, a_kc, b_kc, lda, ldb, ldc, epi="none", bias=None, aux=None,
         ldaux=0, alpha=1.0, beta=0.0, epi_scale=1.0, batch=1, sA=0, sB=0, sC=0, sAux=0, sBias=0,
         workspace=None):
    """Raw strided/batched GEMM (see include/eegfusion.h: eegf_gemm)."""
    _req(A.dtype == B.dtype, "A and B must share a dtype")
    _req(bias is None or bias.dtype == torch.float32, "bias must be fp32")
    call("eegf_gemm", code(A), code(C), int(a_kc), int(b_kc), EPI[epi], M, N, K, batch,
         ptr(A), lda, sA, ptr(B), ldb, sB, ptr(C), ldc, sC,
         ptr(bias), sBias, ptr(aux), ldaux, sAux, float(alpha), float(beta), float(epi_scale),
         ptr(workspace), (workspace.numel() * workspace.element_size() if workspace is not None else 0), stream())
    return C


def linear(x, w, bias=None, *, epi=None, out=None, aux=None):
    """out[M,N] = epi(x[M,K] @ w[N,K]^T + bias): nn.Linear forward."""
    _req(x.dim() == 2 and w.dim() == 2 and x.shape[1] == w.shape[1], "linear: shape mismatch")
    _req(x.stride(1) == 1 and w.is_contiguous(), "linear: x rows / w must be contiguous")
    M, K = x.shape
    N = w.shape[0]
    if epi is None:
        epi = "bias" if bias is not None else "none"
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    _req(out.stride(1) == 1, "linear: out rows must be contiguous")
    return gemm(x, w, out, M=M, N=N, K=K, a_kc=1, b_kc=1, lda=x.stride(0), ldb=K, ldc=out.stride(0),
                epi=epi, bias=bias, aux=aux, ldaux=(aux.stride(0) if aux is not None else 0))


def linear_dgrad(dy, w, *, out=None, epi="none", aux=None, epi_scale=1.0, beta=0.0):
    """out[M,K] = (dy[M,N] @ w[N,K]) (* activation' from aux): input gradient of nn.Linear."""
    M, N = dy.shape
    K = w.shape[1]
    _req(w.shape[0] == N and dy.stride(1) == 1 and w.is_contiguous(), "linear_dgrad: shape")
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=dy.dtype)
    return gemm(dy, w, out, M=M, N=K, K=N, a_kc=1, b_kc=0, lda=dy.stride(0), ldb=K, ldc=out.stride(0),
                epi=epi, aux=aux, ldaux=(aux.stride(0) if aux is not None else 0), epi_scale=epi_scale,
                beta=beta)


def linear_wgrad(dy, x, dw, *, beta=0.0):
    """dw[N,K] (fp32) = dy[M,N]^T @ x[M,K] (+ beta*dw): weight gradient of nn.Linear."""
    M, N = dy.shape
    K = x.shape[1]
    _req(x.shape[0] == M and dw.shape == (N, K) and dw.dtype == torch.float32, "linear_wgrad: shape")
    _req(dy.stride(1) == 1 and x.stride(1) == 1 and dw.is_contiguous(), "linear_wgrad: layout")
    return gemm(dy, x, dw, M=N, N=K, K=M, a_kc=0, b_kc=0, lda=dy.stride(0), ldb=x.stride(0), ldc=K,
                beta=beta)
