"""FusionEngine — the MI355X forward/backward of the whole fusion path over a ParamArena.

Every FLOP is a libeegfusion.so launch on torch's current stream; this module only sequences the
launches, owns activation buffers and routes gradients into the arena.  The op sequence restates
ConcatModel.forward (model.py:34-64, past_acc.py:108-139, main_0430.py:108-123) with the BERT
encoder (transformers modeling_bert.py) and the 3-layer post-norm TransformerDecoder
(torch transformer.py) expanded into fused kernels:

  EEG  : window->tokens | eeg_encoder GEMM | +pos+type, LN (+drop)           (contract W)
         word gather     | +pos+type, LN (+drop)                               (contract T)
         12 x [QKV GEMM | flash attention | out GEMM | drop+res+LN | FFN1 GEMM+GELU | FFN2 GEMM | drop+res+LN]
         pooler GEMM+tanh (CLS row read in place, lda = L*768)
  act  : visual_encoder GEMM
  dec  : 3 x [v GEMM | out GEMM | drop+res+LN1 | q GEMM | q' = Wk^T q/8 (batched GEMM) |
              memory softmax/context (eegf_xattn_fwd) | Wv c + bv (batched GEMM) | out GEMM |
              drop+res+LN2 | linear1+ReLU | linear2 | drop+res+LN3]
  fuse : concat + min-max + PriGumbel gate / PriConcat mechanism (one kernel)
  head : fc0+ReLU | fc2+tanh | classifier
Backward runs the same list in reverse with dgrad/wgrad GEMMs, fused epilogues for the activation
derivatives, LN backward with deterministic partial sums and column reductions for biases.
"""
from __future__ import annotations

import math
import os
import struct
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import BF16, F32, call
from .arena import ParamArena

HID, NH, DH, FFN, NL = 768, 12, 64, 3072, 12
DEC_FF, DEC_L = 2048, 3
FUSED = 3 * HID
MODALS = ("ti", "it", "ii", "tt", "tisc")   # TICA / ITCA / IICA / TTCA / TISC (custom_models/models.py:28-272)
EPS_MODES = ("newfrac", "new")    # past_acc.py:132 1/ln((e^eps-w)/(1-w)) | model.py:57 ln(...)
SPLITK_WS = 24 << 20          # fp32 elements of split-K slab workspace (96 MB)
VARIANTS = {"concat": _lib.FUSE_CONCAT, "priconcat": _lib.FUSE_PRICONCAT,
            "priconcat_lap": _lib.FUSE_PRICONCAT_LAP, "prigumbel": _lib.FUSE_PRIGUMBEL,
            # PriGumbel-v1 (train_val.py:125-158): plain concat into fc1+ReLU, fc2, the v1 gate on 768
            "prigumbel_v1": _lib.FUSE_PRICONCAT}


def P(t):
    return None if t is None else t.data_ptr()


@dataclass
class EngineConfig:
    contract: str = "W"            # "W" window / "T" token ids
    variant: str = "prigumbel"     # concat | priconcat | priconcat_lap | prigumbel
    dtype: torch.dtype = torch.bfloat16
    eps: float = 1.0
    eps_mode: str = "newfrac"
    hidden_dropout: float = 0.1    # BertConfig.hidden_dropout_prob
    attn_dropout: float = 0.1      # BertConfig.attention_probs_dropout_prob (fused into eegf_attn_*)
    dec_dropout: float = 0.1       # TransformerDecoderLayer(dropout=0.1)
    eeg_channels: int = 64
    act_dim: int = 32
    seed: int = 980616
    tau: float = 1.0               # PriGumbel-v1 gumbel_softmax temperature (train_val.py:95)
    varlen: bool = True            # contract T: BERT over the packed real tokens (pad skipping, 8(f)#2)
    modal: str = "ti"              # custom_models/models.py variant: ti | it | ii | tt | tisc (MODALS)
    # attention dropout mask exported by the forward and read by the backward (default False: the
    # backward regenerates it; exporting costs the forward 30 us and the reading backward is 18 us
    # slower than the regenerating one per layer at B = 256, profiles/r4s_attn_bits_ab.log)
    attn_bits: bool = field(default_factory=lambda: os.environ.get("EEGF_ATTN_BITS", "0") == "1")


@dataclass
class Saved:
    B: int = 0
    Bb: int = 0                    # BERT batch (2B for TTCA: both token batches in one pass)
    L: int = 0                     # padded sequence length (decoder memory / pooler rows: B * L)
    R: int = 0                     # BERT rows: B * L, or the packed token count rounded up (varlen)
    vl: dict | None = None         # varlen plan (cu_seqlens, packed / total rows) or None
    hard: bool = False
    training: bool = True
    rng: int = 0
    t: dict = field(default_factory=dict)


class Workspace:
    """Reusable scratch buffers keyed by name (grown on demand)."""

    def __init__(self, device):
        self.device = device
        self.bufs: dict[str, torch.Tensor] = {}

    def get(self, name, numel, dtype):
        b = self.bufs.get(name)
        if b is None or b.numel() < numel or b.dtype != dtype:
            b = torch.empty(max(numel, 1), dtype=dtype, device=self.device)
            self.bufs[name] = b
            self._ptrs = None
        return b[:numel]

    def ptrs(self) -> set:
        if getattr(self, "_ptrs", None) is None:
            self._ptrs = {b.untyped_storage().data_ptr() for b in self.bufs.values()}
        return self._ptrs


class FusionEngine:
    def __init__(self, arena: ParamArena, cfg: EngineConfig):
        self.a = arena
        self.cfg = cfg
        self.dt = cfg.dtype
        self.code = F32 if cfg.dtype == torch.float32 else BF16
        if cfg.variant not in VARIANTS:
            raise ValueError(f"eegfusion: unknown variant {cfg.variant!r} (one of {sorted(VARIANTS)})")
        if cfg.modal not in MODALS:
            raise ValueError(f"eegfusion: modal must be one of {MODALS}, got {cfg.modal!r}")
        if cfg.modal != "ti" and cfg.contract != "T":
            raise ValueError("eegfusion: the modality variants take token ids / CLIP vectors (contract T)")
        if cfg.eps_mode not in EPS_MODES:
            raise ValueError(f"eegfusion: eps_mode must be one of {EPS_MODES}, got {cfg.eps_mode!r}")
        self.variant = VARIANTS[cfg.variant]
        self.v1 = cfg.variant == "prigumbel_v1"
        self.ws = Workspace(arena.device)
        self.rng_counter = 0
        self.injected = None        # parity hook: dict(noise=..., gumbels=..., row_noise=...)
        self.needs_grad: set[str] | None = None
        # grad_ready(names): called during the backward, on the host, once the listed parameters'
        # gradients are final in stream order (the DDP reducer starts their all-reduce there)
        self.grad_ready = None
        self.probe: dict | None = None   # tag -> [(start_event, end_event)] (bench.py live timing)
        # column sums deferred during a backward pass (bias / LayerNorm gradients): they feed only the
        # optimizer, so one batched launch at the end replaces ~140 pairs of small launches
        self.defer: list | None = None
        self._defer_k = 0
        self._parts: set[int] = set()
        # DP-SGD norm pass (eegfusion/dpsgd.py): when set to {"out": fp32 [B], "B": B, "T": L}, every
        # gradient site of a needed parameter adds the squared per-sample norms of its gradient to out
        # instead of accumulating the gradient (dpsgd.hip; opacus GradSampleModule semantics)
        self.psn: dict | None = None

    # ------------------------------------------------------------------ parameter access
    def _refresh_shadow(self):
        a = self.a
        if self.dt == torch.float32:
            return
        v = a.master._version
        if a.shadow is None:
            a.shadow = torch.empty(a.numel, dtype=torch.bfloat16, device=a.device)
            a.shadow_version = -1
        if a.shadow_version != v:
            call("eegf_cast_f32_bf16", a.numel, P(a.master), P(a.shadow), _stream())
            a.shadow_version = v

    def W(self, name):
        """weight in compute dtype"""
        return self.a.view(name, self.a.shadow if self.dt != torch.float32 else None)

    def Wspan(self, first, n):
        return self.a.span(first, n, self.a.shadow if self.dt != torch.float32 else None)

    def F(self, name):
        """fp32 master (biases, LN params, tables, DP; decoder/head weights)"""
        return self.a.view(name)

    def eh(self, *shape):
        """fp32 buffer for the decoder / fusion / head section (always fp32)"""
        return torch.empty(*shape, dtype=torch.float32, device=self.a.device)

    def G(self, name):
        return self.a.gview(name)

    def need(self, name):
        return self.needs_grad is None or name in self.needs_grad

    # --------------------------------------------------------------------- primitives
    def empty(self, *shape, dtype=None):
        return torch.empty(*shape, dtype=dtype or self.dt, device=self.a.device)

    def gemm(self, A, B, C, M, N, K, a_kc, b_kc, lda, ldb, ldc, epi=_lib.EPI_NONE, bias=None, aux=None, ldaux=0,
             alpha=1.0, beta=0.0, scale=1.0, batch=1, sA=0, sB=0, sC=0, sAux=0, sBias=0):
        # batched plain GEMMs split K too (eegf_gemm: the decoder's per-head products on under-filled grids)
        ws = self.ws.get("splitk", SPLITK_WS, torch.float32) if batch == 1 or epi == _lib.EPI_NONE else None
        call("eegf_gemm", _code(A), _code(C), a_kc, b_kc, epi, M, N, K, batch,
             P(A), lda, sA, P(B), ldb, sB, P(C), ldc, sC, P(bias), sBias, P(aux), ldaux, sAux,
             float(alpha), float(beta), float(scale), P(ws), (ws.numel() * 4 if ws is not None else 0), _stream())
        return C

    def linear(self, x, w, b, out, M, lda=None, epi=None, aux=None, tag=None):
        N, K = w.shape
        if epi is None:
            epi = _lib.EPI_BIAS if b is not None else _lib.EPI_NONE
        ev = self._ev_start(tag)
        self.gemm(x, w, out, M, N, K, 1, 1, lda or K, K, out.shape[-1], epi=epi, bias=b, aux=aux,
                  ldaux=(aux.shape[-1] if aux is not None else 0))
        self._ev_end(tag, ev, 2.0 * M * N * K)
        return out

    def _ev_start(self, tag):
        if self.probe is None or tag not in self.probe:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def _ev_end(self, tag, ev, flops=0.0, nbytes=0.0):
        """probe[tag] gets (start, end, algorithmic FLOPs, algorithmic HBM bytes) of the launch just
        enqueued: HIP events on the launch stream (torch's current stream, where every eegf_* call is
        enqueued)"""
        if ev is not None:
            e2 = torch.cuda.Event(enable_timing=True)
            e2.record()
            self.probe[tag].append((ev, e2, flops, nbytes))

    def dgrad(self, dy, w, out, M, ldd=None, ldo=None, epi=_lib.EPI_NONE, aux=None, scale=1.0, beta=0.0,
              bias_grad=None, tag=None):
        """out = dy W (* act'(aux)) (+ beta out).  bias_grad: fp32 tensor that receives += dy.sum(0)
        (a column reduction of dy)."""
        N, K = w.shape
        ldaux = aux.shape[-1] if aux is not None else 0
        if bias_grad is not None and self.psn is not None:
            self._psn_mark(bias_grad, "a fused bias gradient")
            self._psn_bias(dy, M, N, ldd or N)
            bias_grad = None
        if bias_grad is not None:
            self.colsum(dy, ldd or N, M, N, bias_grad)
        ev = self._ev_start(tag)
        self.gemm(dy, w, out, M, K, N, 1, 0, ldd or N, K, ldo or K, epi=epi, aux=aux, ldaux=ldaux, scale=scale,
                  beta=beta)
        self._ev_end(tag, ev, 2.0 * M * N * K)
        return out

    def gbias(self, name):
        """gradient view to accumulate a bias gradient into, or None when not needed"""
        return self.G(name) if self.need(name) else None

    def wgrad(self, dy, x, name, M, ldd=None, ldx=None, bias=None, gw=None, gb=None):
        """weight gradient g[N, K] += dy^T x over M rows; with `bias` (a parameter name) or `gb` (its
        gradient view) the bias gradient dy.sum(0) is produced too — on the weight-gradient kernel
        itself (eegf_gemm_wgrad_bias: row sums of the k-major dy by the MFMA) when the shape takes it,
        else by a column reduction."""
        if gb is None and bias is not None:
            gb = self.gbias(bias)
        if gw is None and not self.need(name):
            if gb is not None:
                self.bgrad(dy, bias, M, width=gb.numel(), ld=ldd, out=gb)
            return
        g = gw if gw is not None else self.G(name)
        N, K = g.shape
        if self.psn is not None:
            self._psn_mark(g, name)
            self._psn_linear(dy, x, M, N, K, ldd or N, ldx or K)
            if gb is not None:
                self._psn_mark(gb, bias or name + " (bias)")
                self._psn_bias(dy, M, N, ldd or N)
            return
        ev = self._ev_start("wgrad" if M >= 4096 else None)
        if gb is not None and _code(dy) == BF16 and _code(x) == BF16:
            ws = self.ws.get("splitk", SPLITK_WS, torch.float32)
            st = _lib.lib().eegf_gemm_wgrad_bias(BF16, N, K, M, P(dy), ldd or N, P(x), ldx or K, P(g), K, 1.0,
                                                 P(gb), P(ws), ws.numel() * 4, _stream())
            if st != 0 and st != _lib.ERR_ARG:
                raise RuntimeError(f"eegf_gemm_wgrad_bias failed with status {st} (hipError)")
            if st == 0:
                self._ev_end("wgrad" if M >= 4096 else None, ev, 2.0 * M * N * K)
                return
        self.gemm(dy, x, g, N, K, M, 0, 0, ldd or N, ldx or K, K, beta=1.0)
        self._ev_end("wgrad" if M >= 4096 else None, ev, 2.0 * M * N * K)
        if gb is not None:
            self.colsum(dy, ldd or N, M, N, gb)

    def bgrad(self, dy, name, rows, width=None, ld=None, period=1, out=None):
        if out is None and not self.need(name):
            return
        o = out if out is not None else self.G(name)
        width = width or o.shape[-1]
        if self.psn is not None:
            if period != 1:
                raise NotImplementedError(f"eegfusion DP-SGD: per-sample norms of {name} (periodic sum)")
            self._psn_mark(o, name)
            self._psn_bias(dy, rows, width, ld or width)
            return
        self.colsum(dy, ld or width, rows, width, o, period)

    # ---------------------------------------------------- DP-SGD per-sample gradient norms (dpsgd.hip)
    def _psn_mark(self, dst, name):
        """The norm pass adds each gradient site's own squared per-sample norm, which is the
        parameter's per-sample norm only when the site is the parameter's sole contribution
        (sum_k ||g_k||^2 != ||sum_k g_k||^2).  Disjoint slices of one parameter (the decoder's in_proj
        Q / K|V blocks) are distinct destinations; a destination reached twice (e.g. a shared
        visual_encoder in IICA / TISC) is refused instead of under-clipping silently."""
        seen = self.psn.setdefault("seen", set())
        key = (dst.data_ptr(), dst.numel())
        if key in seen:
            raise NotImplementedError(f"eegfusion DP-SGD: {name} receives gradient from two sites of the graph; "
                                      "per-sample norms of a shared parameter are not implemented")
        seen.add(key)

    def _psn_rows(self, M):
        """rows per sample of a gradient site with M rows: 1 (head / pooler / decoder) or T (BERT)"""
        ps = self.psn
        if M == ps["B"]:
            return 1
        if M == ps["B"] * ps["T"]:
            return ps["T"]
        raise RuntimeError(f"eegfusion DP-SGD: a gradient site with {M} rows (batch {ps['B']}, T {ps['T']})")

    def _psn_linear(self, dy, x, M, N, K, ldd, ldx):
        """squared per-sample norms of the weight gradient dy^T x (dy [M, N], x [M, K])"""
        ps, T = self.psn, self._psn_rows(M)
        if _code(dy) != _code(x):
            raise RuntimeError("eegfusion DP-SGD: mixed operand dtypes at a weight-gradient site")
        if T == 1:
            call("eegf_row_sqnorm", _code(dy), ps["B"], N, P(dy), ldd, K, P(x), ldx, P(ps["out"]), _stream())
            return
        n = _lib.lib().eegf_ghost_norm_workspace(ps["B"], T)
        ws = self.ws.get("ghost", n, torch.float32)
        call("eegf_ghost_norm", _code(dy), ps["B"], T, K, N, P(x), ldx, P(dy), ldd, P(ws), n, 1.0, P(ps["out"]),
             _stream())

    def _psn_bias(self, dy, M, W, ld, ln=None, bias_term=True):
        """squared per-sample norms of a bias gradient dy.sum(0) (dy [M, W]); ln = (s, mean, rstd) adds
        the LayerNorm gamma term sum_t dy_t * xhat_t; bias_term=False leaves out the dy.sum(0) term
        (LayerNorm beta frozen)"""
        ps, T = self.psn, self._psn_rows(M)
        xs, mean, rstd = ln if ln is not None else (None, None, None)
        call("eegf_seg_sqnorm", _code(dy), ps["B"], T, W, P(dy), ld, P(xs), W, P(mean), P(rstd), int(bias_term), 1.0,
             P(ps["out"]), _stream())

    def colsum(self, src, ld, rows, width, dst, period=1):
        """dst += column sums of src (rows x width, row stride ld); deferred to the end of the backward
        pass (eegf_colsum_batch) when small, else a two-stage eegf_colsum now."""
        # one deferred entry per destination: the batched kernel's blocks add into dst[c] without
        # ordering between entries (a second sum into the same bias runs now, in stream order)
        if (self.defer is not None and period == 1 and rows <= 8192 and self._stable(src)
                and all(P(e[5]) != P(dst) for e in self.defer)):
            self.defer.append((src, int(ld), int(rows), int(width), _code(src), dst))
            return
        ws = self.ws.get("colsum", 1 << 24, torch.float32)
        call("eegf_colsum", _code(src), P(src), ld, rows, width, period, P(ws), ws.numel(), P(dst), 1.0, _stream())

    def _part(self, name, numel):
        """fp32 partial-sum buffer; one per call site while column sums are deferred"""
        if self.defer is not None:
            self._defer_k += 1
            name = f"{name}{self._defer_k}"
            b = self.ws.get(name, numel, torch.float32)
            self._parts.add(b.untyped_storage().data_ptr())
            return b
        return self.ws.get(name, numel, torch.float32)

    def _stable(self, src):
        """src is not overwritten before the flush: a per-site partial buffer or a tensor of its own
        (shared workspace buffers are reused by later layers)"""
        ptr = src.untyped_storage().data_ptr()
        return ptr in self._parts or ptr not in self.ws.ptrs()

    def _flush_colsums(self):
        d, self.defer = self.defer, None
        if not d:
            return
        beta = struct.unpack("<i", struct.pack("<f", 1.0))[0]
        rows, blk = [], 0
        for src, ld, r, w, code, dst in d:
            rows.append([P(src), P(dst), ld, r, w | (code << 32), beta | (blk << 32)])
            blk += (w + 63) // 64
        host = torch.tensor(rows, dtype=torch.int64).pin_memory()
        dev = host.to(self.a.device, non_blocking=True)
        call("eegf_colsum_batch", len(rows), P(dev), blk, _stream())
        self._colsum_keep = (d, host, dev)      # sources and descriptors live until the next flush

    def dropout(self, x, group, p, rng):
        if p > 0:
            call("eegf_dropout", _code(x), x.numel(), group, float(p), self.cfg.seed, rng, P(x), _stream())

    def ln_fwd(self, x, r, pre, rows, out, s, mean, rstd, eps, p=0.0, mode=0, rng=0, table=None, period=1,
               table2=None):
        call("eegf_ln_fwd", _code(x), rows, HID, P(x), P(r), P(table), period, P(table2), P(self.F(pre + ".weight")),
             P(self.F(pre + ".bias")), float(eps), float(p), int(mode if p > 0 else 0), self.cfg.seed, rng, P(out),
             P(s), P(mean), P(rstd), _stream())

    def _ln_bytes(self, rows, save):
        """algorithmic bytes of a BERT-layer LayerNorm forward (dropout + residual + LN): the sublayer
        output and the residual in, the normalised row out, and when saving for the backward the pre-LN
        sum and the row mean / rstd; gamma / beta once"""
        e = torch.empty((), dtype=self.dt).element_size()
        return rows * HID * e * (3 + (1 if save else 0)) + (rows * 8 if save else 0) + 2 * HID * 4

    def ln_bwd(self, dy, s, mean, rstd, pre, rows, dx, dr, p=0.0, mode=0, rng=0):
        rpb = _lib.lib().eegf_ln_bwd_partial_rows(rows)
        nb = (rows + rpb - 1) // rpb
        part = self._part("ln_part", 2 * nb * HID)
        call("eegf_ln_bwd", _code(dy), rows, HID, P(dy), P(s), P(mean), P(rstd), P(self.F(pre + ".weight")), float(p),
             int(mode if p > 0 else 0), self.cfg.seed, rng, P(dx), P(dr), P(part), P(part[nb * HID:]), _stream())
        if self.psn is not None:
            gamma, beta = self.need(pre + ".weight"), self.need(pre + ".bias")
            if gamma or beta:
                if mode == 2 and p > 0:
                    raise NotImplementedError("eegfusion DP-SGD: per-sample norms of a post-LN-dropout LayerNorm")
                if gamma:
                    self._psn_mark(self.G(pre + ".weight"), pre + ".weight")
                if beta:
                    self._psn_mark(self.G(pre + ".bias"), pre + ".bias")
                self._psn_bias(dy, rows, HID, HID, ln=(s, mean, rstd) if gamma else None, bias_term=beta)
            return
        self.bgrad(part[: nb * HID], pre + ".weight", nb, HID)
        self.bgrad(part[nb * HID:], pre + ".bias", nb, HID)

    def _uniform_plan(self, B, L, kbias):
        """every row a full-length sequence (cu[b] = b*L) with the key mask: the varlen attention
        kernels on the padded layout, for lengths the dense kernels do not take (L % 256)."""
        key = ("uniform", B, L)
        cu = self._plans.get(key) if hasattr(self, "_plans") else None
        if cu is None:
            self._plans = getattr(self, "_plans", {})
            cu = torch.arange(0, (B + 1) * L, L, dtype=torch.int32).to(self.a.device)
            self._plans[key] = cu
        return dict(cu=cu, T=B * L, rows=B * L, max_len=L, kbias=kbias, uniform=True)

    def _attn_any_fwd(self, qkv, ctx, lse, B, L, kbias, p, rng):
        """BertSelfAttention-form attention over the padded layout at any L (dense kernels for
        L % 256 == 0, else the varlen ones with uniform lengths)."""
        if L % 256 == 0:
            call("eegf_attn_fwd", self.code, B, NH, L, P(qkv), 3 * HID, P(kbias), DH ** -0.5, float(p), self.cfg.seed,
                 rng, P(ctx), HID, P(lse), None, _stream())
        else:
            vl = self._uniform_plan(B, L, kbias)
            call("eegf_attn_varlen_fwd", self.code, B, NH, L, P(vl["cu"]), B * L, B * L, P(qkv), 3 * HID, P(kbias),
                 DH ** -0.5, float(p), self.cfg.seed, rng, P(ctx), HID, P(lse), _stream())

    def _attn_any_bwd(self, qkv, ctx, dctx, lse, dqkv, B, L, kbias, p, rng):
        if L % 256 == 0:
            n = _lib.lib().eegf_attn_bwd_workspace(B, L)
            ws = self.ws.get("b_dqws", n, torch.float32) if n > 0 else None
            call("eegf_attn_bwd", self.code, B, NH, L, P(qkv), 3 * HID, P(kbias), DH ** -0.5, float(p), self.cfg.seed,
                 rng, P(ctx), P(dctx), HID, P(lse), None, P(dqkv), P(ws), _stream())
        else:
            vl = self._uniform_plan(B, L, kbias)
            n = _lib.lib().eegf_attn_varlen_bwd_workspace(B * L, L)
            ws = self.ws.get("b_dqws", n, torch.float32) if n > 0 else None
            call("eegf_attn_varlen_bwd", self.code, B, NH, L, P(vl["cu"]), B * L, B * L, P(qkv), 3 * HID, P(kbias),
                 DH ** -0.5, float(p), self.cfg.seed, rng, P(ctx), P(dctx), HID, P(lse), P(dqkv), P(ws), _stream())

    # ------------------------------------------------------- TTCA sequence decoder (models.py:84-129)
    def _seqdec_fwd(self, t, tgt, mem, B, L, ddrop, rng):
        """multi_head_decoder(tgt=act sequence, memory=eeg sequence) with no masks, then
        .permute(1,0,2).mean(dim=1) (models.py:107-109): post-norm TransformerDecoderLayer x3 over
        [B*L, 768] rows in the encoder dtype; -> cross [B, 768] fp32."""
        R = B * L
        x = tgt
        st = []
        for d in range(DEC_L):
            pre = f"multi_head_decoder.layers.{d}."
            r0 = rng + 400 + 16 * d
            qkv = self.empty(R, 3 * HID)
            self.linear(x, self.W(pre + "self_attn.in_proj_weight"), self.F(pre + "self_attn.in_proj_bias"), qkv, R)
            ctx, lse = self.empty(R, HID), self._f32(B, NH, L)
            self._attn_any_fwd(qkv, ctx, lse, B, L, None, ddrop, r0)
            sa = self.empty(R, HID)
            self.linear(ctx, self.W(pre + "self_attn.out_proj.weight"), self.F(pre + "self_attn.out_proj.bias"), sa, R)
            x1, ln1 = self.empty(R, HID), (self.empty(R, HID), self._f32(R), self._f32(R))
            self.ln_fwd(sa, x, pre + "norm1", R, x1, *ln1, 1e-5, ddrop, 1, r0 + 1)
            cw, cb = self.W(pre + "multihead_attn.in_proj_weight"), self.F(pre + "multihead_attn.in_proj_bias")
            qkv2 = self.empty(R, 3 * HID)          # [q(x1) | k(mem) v(mem)] in the fused QKV layout
            self.gemm(x1, cw[:HID], qkv2, R, HID, HID, 1, 1, HID, HID, 3 * HID, epi=_lib.EPI_BIAS, bias=cb[:HID])
            self.gemm(mem, cw[HID:], qkv2[:, HID:], R, 2 * HID, HID, 1, 1, HID, HID, 3 * HID, epi=_lib.EPI_BIAS,
                      bias=cb[HID:])
            ctx2, lse2 = self.empty(R, HID), self._f32(B, NH, L)
            self._attn_any_fwd(qkv2, ctx2, lse2, B, L, None, ddrop, r0 + 2)
            ca = self.empty(R, HID)
            self.linear(ctx2, self.W(pre + "multihead_attn.out_proj.weight"),
                        self.F(pre + "multihead_attn.out_proj.bias"), ca, R)
            x2, ln2 = self.empty(R, HID), (self.empty(R, HID), self._f32(R), self._f32(R))
            self.ln_fwd(ca, x1, pre + "norm2", R, x2, *ln2, 1e-5, ddrop, 1, r0 + 3)
            f1 = self.empty(R, DEC_FF)
            self.linear(x2, self.W(pre + "linear1.weight"), self.F(pre + "linear1.bias"), f1, R, epi=_lib.EPI_BIAS_RELU)
            self.dropout(f1, 1, ddrop, r0 + 4)
            f2 = self.empty(R, HID)
            self.linear(f1, self.W(pre + "linear2.weight"), self.F(pre + "linear2.bias"), f2, R)
            x3, ln3 = self.empty(R, HID), (self.empty(R, HID), self._f32(R), self._f32(R))
            self.ln_fwd(f2, x2, pre + "norm3", R, x3, *ln3, 1e-5, ddrop, 1, r0 + 5)
            st.append(dict(x=x, qkv=qkv, ctx=ctx, lse=lse, ln1=ln1, x1=x1, qkv2=qkv2, ctx2=ctx2, lse2=lse2, ln2=ln2,
                           x2=x2, f1=f1, ln3=ln3))
            x = x3
        t["sdec"] = dict(layers=st, mem=mem)
        cross = self._f32(B, HID)
        call("eegf_seq_mean", self.code, B, L, HID, P(x), HID, P(cross), HID, _stream())
        return cross

    def _seqdec_bwd(self, t, dcross, dtgt, dmem, B, L, ddrop, rng):
        """backward of _seqdec_fwd: dtgt / dmem [B*L, 768] (encoder dtype) overwritten."""
        R = B * L
        sd = t["sdec"]
        mem = sd["mem"]
        dx3 = self.empty(R, HID)
        call("eegf_seq_mean_bwd", self.code, B, L, HID, P(dcross), HID, P(dx3), HID, 0.0, _stream())
        pscale = 1.0 / (1.0 - ddrop) if ddrop > 0 else 1.0
        for d in reversed(range(DEC_L)):
            pre = f"multi_head_decoder.layers.{d}."
            s = sd["layers"][d]
            r0 = rng + 400 + 16 * d
            df2, dx2 = self.empty(R, HID), self.empty(R, HID)
            self.ln_bwd(dx3, *s["ln3"], pre + "norm3", R, df2, dx2, ddrop, 1, r0 + 5)
            self.wgrad(df2, s["f1"], pre + "linear2.weight", R, bias=pre + "linear2.bias")
            df1 = self.empty(R, DEC_FF)
            self.dgrad(df2, self.W(pre + "linear2.weight"), df1, R, epi=_lib.EPI_DRELU, aux=s["f1"], scale=pscale)
            self.wgrad(df1, s["x2"], pre + "linear1.weight", R, bias=pre + "linear1.bias")
            self.dgrad(df1, self.W(pre + "linear1.weight"), dx2, R, beta=1.0)
            dca, dx1 = self.empty(R, HID), self.empty(R, HID)
            self.ln_bwd(dx2, *s["ln2"], pre + "norm2", R, dca, dx1, ddrop, 1, r0 + 3)
            self.wgrad(dca, s["ctx2"], pre + "multihead_attn.out_proj.weight", R,
                       bias=pre + "multihead_attn.out_proj.bias")
            dctx2 = self.empty(R, HID)
            self.dgrad(dca, self.W(pre + "multihead_attn.out_proj.weight"), dctx2, R)
            dqkv2 = self.empty(R, 3 * HID)
            self._attn_any_bwd(s["qkv2"], s["ctx2"], dctx2, s["lse2"], dqkv2, B, L, None, ddrop, r0 + 2)
            wn, bn = pre + "multihead_attn.in_proj_weight", pre + "multihead_attn.in_proj_bias"
            cw = self.W(wn)
            gw = self.G(wn) if self.need(wn) else None
            gb = self.G(bn) if self.need(bn) else None
            self.wgrad(dqkv2, s["x1"], wn, R, ldd=3 * HID, gw=None if gw is None else gw[:HID],
                       gb=None if gb is None else gb[:HID])
            self.wgrad(dqkv2[:, HID:], mem, wn, R, ldd=3 * HID, gw=None if gw is None else gw[HID:],
                       gb=None if gb is None else gb[HID:])
            self.dgrad(dqkv2, cw[:HID], dx1, R, ldd=3 * HID, beta=1.0)
            self.dgrad(dqkv2[:, HID:], cw[HID:], dmem, R, ldd=3 * HID, beta=0.0 if d == DEC_L - 1 else 1.0)
            dsa, dx = self.empty(R, HID), (dtgt if d == 0 else self.empty(R, HID))
            self.ln_bwd(dx1, *s["ln1"], pre + "norm1", R, dsa, dx, ddrop, 1, r0 + 1)
            self.wgrad(dsa, s["ctx"], pre + "self_attn.out_proj.weight", R, bias=pre + "self_attn.out_proj.bias")
            dctx = self.empty(R, HID)
            self.dgrad(dsa, self.W(pre + "self_attn.out_proj.weight"), dctx, R)
            dqkv = self.empty(R, 3 * HID)
            self._attn_any_bwd(s["qkv"], s["ctx"], dctx, s["lse"], dqkv, B, L, None, ddrop, r0)
            self.wgrad(dqkv, s["x"], pre + "self_attn.in_proj_weight", R, bias=pre + "self_attn.in_proj_bias")
            self.dgrad(dqkv, self.W(pre + "self_attn.in_proj_weight"), dx, R, beta=1.0)
            dx3 = dx

    # --------------------------------------------------------- TISC 2-token encoder (models.py:215-272)
    def _enc2_fwd(self, t, X, B, ddrop, rng):
        """multi_head_encoder over the two tokens [mean(EEG seq), action] of each sample, then
        .mean(dim=0) (models.py:251-253): post-norm TransformerEncoderLayer x3 (ReLU, 2048, LN 1e-5),
        fp32 like the single-query decoder; X [2B, 768] fp32 (row 2b, 2b+1 = sample b's tokens)."""
        R = 2 * B
        st = []
        for e in range(DEC_L):
            pre = f"multi_head_encoder.layers.{e}."
            r0 = rng + 500 + 16 * e
            qkv = self.eh(R, 3 * HID)
            self.linear(X, self.F(pre + "self_attn.in_proj_weight"), self.F(pre + "self_attn.in_proj_bias"), qkv, R)
            ctx, probs = self.eh(R, HID), self._f32(B, NH, 2, 2)
            call("eegf_attn_small_fwd", F32, B, 2, P(qkv), 3 * HID, DH ** -0.5, float(ddrop), self.cfg.seed, r0,
                 P(ctx), HID, P(probs), _stream())
            sa = self.eh(R, HID)
            self.linear(ctx, self.F(pre + "self_attn.out_proj.weight"), self.F(pre + "self_attn.out_proj.bias"), sa, R)
            x1, ln1 = self.eh(R, HID), (self.eh(R, HID), self._f32(R), self._f32(R))
            self.ln_fwd(sa, X, pre + "norm1", R, x1, *ln1, 1e-5, ddrop, 1, r0 + 1)
            f1 = self.eh(R, DEC_FF)
            self.linear(x1, self.F(pre + "linear1.weight"), self.F(pre + "linear1.bias"), f1, R, epi=_lib.EPI_BIAS_RELU)
            self.dropout(f1, 1, ddrop, r0 + 2)
            f2 = self.eh(R, HID)
            self.linear(f1, self.F(pre + "linear2.weight"), self.F(pre + "linear2.bias"), f2, R)
            x2, ln2 = self.eh(R, HID), (self.eh(R, HID), self._f32(R), self._f32(R))
            self.ln_fwd(f2, x1, pre + "norm2", R, x2, *ln2, 1e-5, ddrop, 1, r0 + 3)
            st.append(dict(x=X, qkv=qkv, ctx=ctx, probs=probs, ln1=ln1, x1=x1, f1=f1, ln2=ln2))
            X = x2
        t["enc"] = st
        enc = self._f32(B, HID)
        call("eegf_seq_mean", F32, B, 2, HID, P(X), HID, P(enc), HID, _stream())
        return enc

    def _enc2_bwd(self, t, dX, B, ddrop, rng):
        """backward of _enc2_fwd: dX [2B, 768] fp32, the gradient at the encoder output on entry and
        at its input on return (updated in place)."""
        R = 2 * B
        pscale = 1.0 / (1.0 - ddrop) if ddrop > 0 else 1.0
        for e in reversed(range(DEC_L)):
            pre = f"multi_head_encoder.layers.{e}."
            s = t["enc"][e]
            r0 = rng + 500 + 16 * e
            df2, dx1 = self.eh(R, HID), self.eh(R, HID)
            self.ln_bwd(dX, *s["ln2"], pre + "norm2", R, df2, dx1, ddrop, 1, r0 + 3)
            self.wgrad(df2, s["f1"], pre + "linear2.weight", R, bias=pre + "linear2.bias")
            df1 = self.eh(R, DEC_FF)
            self.dgrad(df2, self.F(pre + "linear2.weight"), df1, R, epi=_lib.EPI_DRELU, aux=s["f1"], scale=pscale)
            self.wgrad(df1, s["x1"], pre + "linear1.weight", R, bias=pre + "linear1.bias")
            self.dgrad(df1, self.F(pre + "linear1.weight"), dx1, R, beta=1.0)
            dsa = self.eh(R, HID)
            self.ln_bwd(dx1, *s["ln1"], pre + "norm1", R, dsa, dX, ddrop, 1, r0 + 1)
            self.wgrad(dsa, s["ctx"], pre + "self_attn.out_proj.weight", R, bias=pre + "self_attn.out_proj.bias")
            dctx = self.eh(R, HID)
            self.dgrad(dsa, self.F(pre + "self_attn.out_proj.weight"), dctx, R)
            dqkv = self.eh(R, 3 * HID)
            call("eegf_attn_small_bwd", F32, B, 2, P(s["qkv"]), 3 * HID, P(s["probs"]), P(dctx), HID, DH ** -0.5,
                 float(ddrop), self.cfg.seed, r0, P(dqkv), 3 * HID, _stream())
            self.wgrad(dqkv, s["x"], pre + "self_attn.in_proj_weight", R, bias=pre + "self_attn.in_proj_bias")
            self.dgrad(dqkv, self.F(pre + "self_attn.in_proj_weight"), dX, R, beta=1.0)

    def _varlen_plan(self, mask, B, L):
        """Contract T pad skipping: per-row token counts of the attention mask (one device pass, one
        small D2H copy), cu_seqlens, and the packed row count rounded up to the 256-row GEMM tile.
        None (the padded path) when a mask row is not right-padded or has no token."""
        dev = self.a.device
        mask = mask.contiguous()
        buf = torch.empty(B + 1, dtype=torch.int32, device=dev)
        call("eegf_seq_lengths", B, L, P(mask), P(buf), P(buf[B:]), _stream())
        host = buf.cpu().numpy()
        lens = host[:B].astype(np.int64)
        if host[B] != 0 or lens.min() <= 0:
            return None
        cu = np.zeros(B + 1, dtype=np.int32)
        cu[1:] = np.cumsum(lens)
        T = int(cu[-1])
        return dict(cu=torch.from_numpy(cu).to(dev), T=T, rows=(T + 255) // 256 * 256, max_len=int(lens.max()))

    # =================================================================== forward
    def forward(self, batch: dict, hard: bool, training: bool, save: bool = True):
        """batch (device tensors): contract W: eeg [B,C,T] f32, act [B,A] f32;
        contract T: title_input [B,L] i64, text_mask [B,L] i64, frame_input [B,1,512] f32 (the modality
        variants add title_input2 / text_mask2 (TTCA) or frame_input2 (IICA), MODALS)."""
        cfg = self.cfg
        self._refresh_shadow()
        sv = Saved(hard=hard, training=training)
        t = sv.t
        sv.rng = self.rng_counter
        self.rng_counter += 1 << 12
        ddrop = cfg.dec_dropout if training else 0.0
        modal = cfg.modal
        if modal == "ii":
            # IICA (models.py:176-214): no BERT; the decoder's memory is the action image token
            ve, va = self._visual_fwd(batch["frame_input"], t, "act"), self._visual_fwd(batch["frame_input2"], t, "act2")
            B = ve.shape[0]
            sv.B = sv.Bb = B
            sv.L = 1
            cross = self._dec1_fwd(t, ve, va, 1, None, ddrop, sv.rng)
            feats = (ve, va, cross)
        else:
            bb = batch
            if modal == "tt":
                # TTCA (models.py:84-129): one BERT pass over both token batches (shared weights)
                bb = {"title_input": torch.cat((batch["title_input"], batch["title_input2"])).contiguous(),
                      "text_mask": torch.cat((batch["text_mask"], batch["text_mask2"])).contiguous()}
            h, pooled = self._bert_fwd(bb, sv, save, training)
            B, L = sv.B, sv.L
            if modal == "tt":
                B = B // 2
                sv.B = B
                cross = self._seqdec_fwd(t, h[B * L:], h[:B * L], B, L, ddrop, sv.rng)
                feats = (pooled[:B], pooled[B:], cross)
            elif modal == "tisc":
                # TISC (models.py:215-272): tokens [mean(EEG seq), action image] -> 3-layer encoder -> mean
                X = self.eh(2 * B, HID)
                call("eegf_seq_mean", self.code, B, L, HID, P(h), HID, P(X), 2 * HID, _stream())
                vis = self._visual_fwd(batch["frame_input"], t, "act", out=X[1::2])
                enc = self._enc2_fwd(t, X, B, ddrop, sv.rng)
                feats = (pooled, vis, enc)
            else:
                act = batch["act"] if cfg.contract == "W" else batch["frame_input"]
                vis = self._visual_fwd(act, t, "act")
                cross = self._dec1_fwd(t, vis, h, L, t["kbias"], ddrop, sv.rng)
                feats = (vis, pooled, cross) if modal == "it" else (pooled, vis, cross)
        t["vis"] = feats

        # ---------------- fusion + privacy stage + head (fp32)
        logits, fh = self.fuse_head_fwd(*feats, hard, sv.rng)
        t.update(fh)
        return logits, sv

    def _visual_fwd(self, x, t, key, out=None):
        """visual_encoder on [B,1,in] / [B,in] fp32 (model.py:18,36): out [B,768] fp32 (or a strided
        row view)"""
        B = x.shape[0]
        act = x.reshape(B, -1).contiguous().float()
        vis = out if out is not None else self.eh(B, HID)
        self.gemm(act, self.F("visual_encoder.weight"), vis, B, HID, act.shape[1], 1, 1, act.shape[1], act.shape[1],
                  vis.stride(0), epi=_lib.EPI_BIAS, bias=self.F("visual_encoder.bias"))
        t[key] = act
        return vis

    def _bert_fwd(self, batch, sv, save, training):
        """EEG front-end + BertModel (model.py:37-39): -> (sequence output [B*L, 768] in the compute
        dtype, padded layout; pooled [B, 768] fp32)."""
        cfg = self.cfg
        t = sv.t
        pdrop = cfg.hidden_dropout if training else 0.0
        adrop = cfg.attn_dropout if training else 0.0
        # ---------------- EEG front-end + BERT embeddings
        if cfg.contract == "W":
            eeg = batch["eeg"]
            B, C, L = eeg.shape
            tok = self.empty(B * L, C)
            call("eegf_window_tokens", self.code, B, C, L, P(eeg), P(tok), _stream())
            x = self.empty(B * L, HID)
            self.linear(tok, self.W("eeg_encoder.weight"), self.F("eeg_encoder.bias"), x, B * L)
            kbias = None
            t["tok"] = tok
        else:
            ids = batch["title_input"]
            B, L = ids.shape
            mask = batch["text_mask"]
            kbias = torch.empty(B, L, dtype=torch.float32, device=self.a.device)
            call("eegf_key_bias", B * L, P(mask), P(kbias), _stream())
            # DP-SGD's per-sample norms index sites by B x L rows: it keeps the padded layout; TTCA /
            # TISC consume the padded positions' outputs (unmasked decoder memory, plain sequence mean)
            packable = cfg.varlen and self.psn is None and cfg.modal in ("ti", "it")
            vl = self._varlen_plan(mask, B, L) if packable else None
            if vl is None and (L % 256 or L % 128):
                # dense lengths the dense attention kernels do not take: the varlen kernels with one
                # full-length sequence per row and the key mask
                vl = self._uniform_plan(B, L, kbias)
            if vl is None or vl.get("uniform"):
                x = self.empty(B * L, HID)
                call("eegf_embed_gather", self.code, B * L, HID, P(ids),
                     P(self.F("bert.embeddings.word_embeddings.weight")), P(x), _stream())
                t["ids"] = ids
            else:
                x = self.empty(vl["rows"], HID)
                ids_p = torch.empty(vl["rows"], dtype=torch.int64, device=self.a.device)
                call("eegf_varlen_embed", self.code, B, L, HID, P(vl["cu"]), vl["T"], vl["rows"], P(ids),
                     P(self.F("bert.embeddings.word_embeddings.weight")),
                     P(self.F("bert.embeddings.position_embeddings.weight")), P(x), P(ids_p), _stream())
                t["ids"] = ids_p
            sv.vl = vl
        sv.B, sv.Bb, sv.L = B, B, L
        vl = sv.vl
        if vl is None:
            if save and L % 256:
                # eegf_attn_bwd handles L % 256 == 0 only: refuse before any gradient is written
                raise ValueError(f"eegfusion: sequence length {L} is not a multiple of 256 (backward unsupported)")
            if L % 128:
                raise ValueError(f"eegfusion: sequence length {L} is not a multiple of 128")
        R = B * L if vl is None else vl["rows"]
        sv.R = R
        t["kbias"] = kbias
        e = "bert.embeddings."
        h = self.empty(R, HID)
        # without save (the PriGumbel DP pass: no full backward) the LN residual sums / statistics and
        # the FFN pre-activations are not stored
        s0, m0, r0 = (self.empty(R, HID), self._f32(R), self._f32(R)) if save else (None, None, None)
        # position rows: the LN table add (dense) or already in the packed gather (varlen)
        packed = vl is not None and not vl.get("uniform")
        self.ln_fwd(x, None, e + "LayerNorm", R, h, s0, m0, r0, 1e-12, pdrop, 2, sv.rng + 1,
                    table=None if packed else self.F(e + "position_embeddings.weight"),
                    period=1 if packed else L, table2=self.F(e + "token_type_embeddings.weight"))
        t["emb"] = (s0, m0, r0)
        scale = DH ** -0.5

        # ---------------- BERT encoder
        layers = []
        for i in range(NL):
            pre = f"bert.encoder.layer.{i}."
            qkv = self.empty(R, 3 * HID)
            self.linear(h, self.Wspan(pre + "attention.self.query.weight", 3).view(3 * HID, HID),
                        self.a.span(pre + "attention.self.query.bias", 3), qkv, R, tag="qkv_fwd")
            ctx = self.empty(R, HID)
            lse = torch.empty(B, NH, L, dtype=torch.float32, device=self.a.device)
            # dropout keep bits (1 bit per probability, 25 MB per layer at B = 256) only with
            # cfg.attn_bits: by default the backward regenerates the Philox stream
            bits = (torch.empty(B * NH * L * L // 32, dtype=torch.int32, device=self.a.device)
                    if save and adrop > 0 and vl is None and self.cfg.attn_bits else None)
            ev = self._ev_start("attn_fwd")
            if vl is None:
                call("eegf_attn_fwd", self.code, B, NH, L, P(qkv), 3 * HID, P(kbias), scale, float(adrop),
                     self.cfg.seed, sv.rng + 12 + 3 * i, P(ctx), HID, P(lse), P(bits), _stream())
            else:
                call("eegf_attn_varlen_fwd", self.code, B, NH, L, P(vl["cu"]), vl["T"], R, P(qkv), 3 * HID,
                     P(vl.get("kbias")), scale, float(adrop), self.cfg.seed, sv.rng + 12 + 3 * i, P(ctx), HID, P(lse),
                     _stream())
            self._ev_end("attn_fwd", ev, 4.0 * B * NH * L * L * DH)
            ao = self.ws.get("ao", R * HID, self.dt).view(R, HID)
            self.linear(ctx, self.W(pre + "attention.output.dense.weight"), self.F(pre + "attention.output.dense.bias"),
                        ao, R, tag="ao_fwd")
            a1 = self.empty(R, HID)
            s1, m1, r1 = (self.empty(R, HID), self._f32(R), self._f32(R)) if save else (None, None, None)
            ev = self._ev_start("ln_fwd768")
            self.ln_fwd(ao, h, pre + "attention.output.LayerNorm", R, a1, s1, m1, r1, 1e-12, pdrop, 1,
                        sv.rng + 10 + 3 * i)
            self._ev_end("ln_fwd768", ev, 0.0, self._ln_bytes(R, save))
            # saved for the backward: gelu'(pre) (the DGELU epilogue becomes a multiply)
            ffgd = self.empty(R, FFN) if save else None
            ffact = self.empty(R, FFN) if save else self.ws.get("ffact", R * FFN, self.dt).view(R, FFN)
            self.linear(a1, self.W(pre + "intermediate.dense.weight"), self.F(pre + "intermediate.dense.bias"), ffact,
                        R, epi=_lib.EPI_BIAS_GELU_D if save else _lib.EPI_BIAS_GELU, aux=ffgd,
                        tag="ffn1_fwd_gd" if save else "ffn1_fwd")
            fo = self.ws.get("fo", R * HID, self.dt).view(R, HID)
            self.linear(ffact, self.W(pre + "output.dense.weight"), self.F(pre + "output.dense.bias"), fo, R,
                        tag="ffn2_fwd")
            h2 = self.empty(R, HID)
            s2, m2, r2 = (self.empty(R, HID), self._f32(R), self._f32(R)) if save else (None, None, None)
            ev = self._ev_start("ln_fwd768")
            self.ln_fwd(fo, a1, pre + "output.LayerNorm", R, h2, s2, m2, r2, 1e-12, pdrop, 1, sv.rng + 11 + 3 * i)
            self._ev_end("ln_fwd768", ev, 0.0, self._ln_bytes(R, save))
            if save:
                layers.append(dict(h=h, qkv=qkv, ctx=ctx, lse=lse, bits=bits, a1=a1, ln1=(s1, m1, r1), ffgd=ffgd, ffact=ffact,
                                   ln2=(s2, m2, r2)))
            h = h2
        t["layers"] = layers
        if packed:                # decoder memory / pooler input: the padded [B, L] layout, zero pad rows
            hp = self.empty(B * L, HID)
            call("eegf_varlen_rows", self.code, B, L, HID, P(vl["cu"]), vl["T"], R, P(h), HID, P(hp), HID, 1,
                 _stream())
            h = hp
        t["mem"] = h
        pooled = self.eh(B, HID)                 # fp32 out of the bf16 pooler GEMM (+ tanh)
        self.linear(h, self.W("bert.pooler.dense.weight"), self.F("bert.pooler.dense.bias"), pooled, B, lda=L * HID,
                    epi=_lib.EPI_BIAS_TANH)
        t["pooled"] = pooled
        return h, pooled

    def _dec1_fwd(self, t, vis, h, L, kbias, ddrop, rng):
        """multi_head_decoder with one query token per sample (model.py:40-44) over the memory h
        [B*L, 768] (encoder dtype, or fp32 for IICA's single-token memory), memory key bias [B, L]
        (nullable); fp32, single-query rewrite.  -> cross [B, 768] fp32."""
        B = vis.shape[0]
        scale = DH ** -0.5
        t["dmem_src"] = (h, L, kbias)
        x = vis
        dl = []
        for d in range(DEC_L):
            pre = f"multi_head_decoder.layers.{d}."
            in_w, in_b = self.F(pre + "self_attn.in_proj_weight"), self.F(pre + "self_attn.in_proj_bias")
            v = self.eh(B, HID)
            self.linear(x, in_w[2 * HID:], in_b[2 * HID:], v, B)
            # one query, one key: the attention weight is 1, so dropout of it is a per-(row, head) mask on v
            self.dropout(v, 64, ddrop, rng + 103 + 8 * d)
            sa = self.eh(B, HID)
            self.linear(v, self.F(pre + "self_attn.out_proj.weight"), self.F(pre + "self_attn.out_proj.bias"), sa, B)
            x1, ln1 = self.eh(B, HID), (self.eh(B, HID), self._f32(B), self._f32(B))
            self.ln_fwd(sa, x, pre + "norm1", B, x1, *ln1, 1e-5, ddrop, 1, rng + 100 + 8 * d)
            cw, cb = self.F(pre + "multihead_attn.in_proj_weight"), self.F(pre + "multihead_attn.in_proj_bias")
            q = self.eh(B, HID)
            self.linear(x1, cw[:HID], cb[:HID], q, B)
            qp = self.eh(B, NH, HID)
            # qp[b,h,:] = Wk_h^T q_h / 8   (batched over heads)
            self.gemm(q, cw[HID:2 * HID], qp, B, HID, DH, 1, 0, HID, HID, NH * HID, alpha=scale, batch=NH, sA=DH,
                      sB=DH * HID, sC=HID)
            probs = self._f32(B, NH, L)
            psum = self._f32(B, NH) if ddrop > 0 else None
            cc = self.eh(B, NH, HID)
            xws = self.ws.get("xattn", B * NH * L, torch.float32)
            call("eegf_xattn_fwd", _code(h), F32, B, L, P(h), P(qp), P(kbias), float(ddrop), self.cfg.seed,
                 rng + 104 + 8 * d, P(xws), P(probs), P(psum), P(cc), _stream())
            ctxd = self.eh(B, HID)
            # ctx[b, h*64+n] = sum_c cc[b,h,c] Wv[h*64+n, c] + s[b,h] bv[h*64+n]   (s = sum_j p~_j; 1 w/o dropout)
            self.gemm(cc, cw[2 * HID:], ctxd, B, DH, HID, 1, 1, NH * HID, HID, HID,
                      epi=_lib.EPI_BIAS if psum is None else _lib.EPI_NONE,
                      bias=cb[2 * HID:] if psum is None else None, batch=NH, sA=HID, sB=DH * HID, sC=DH, sBias=DH)
            if psum is not None:
                call("eegf_head_bias_fwd", B, HID, DH, P(ctxd), P(cb[2 * HID:]), P(psum), _stream())
            ca = self.eh(B, HID)
            self.linear(ctxd, self.F(pre + "multihead_attn.out_proj.weight"),
                        self.F(pre + "multihead_attn.out_proj.bias"), ca, B)
            x2, ln2 = self.eh(B, HID), (self.eh(B, HID), self._f32(B), self._f32(B))
            self.ln_fwd(ca, x1, pre + "norm2", B, x2, *ln2, 1e-5, ddrop, 1, rng + 101 + 8 * d)
            f1 = self.eh(B, DEC_FF)
            self.linear(x2, self.F(pre + "linear1.weight"), self.F(pre + "linear1.bias"), f1, B, epi=_lib.EPI_BIAS_RELU)
            self.dropout(f1, 1, ddrop, rng + 105 + 8 * d)      # _ff_block's inner dropout
            f2 = self.eh(B, HID)
            self.linear(f1, self.F(pre + "linear2.weight"), self.F(pre + "linear2.bias"), f2, B)
            x3, ln3 = self.eh(B, HID), (self.eh(B, HID), self._f32(B), self._f32(B))
            self.ln_fwd(f2, x2, pre + "norm3", B, x3, *ln3, 1e-5, ddrop, 1, rng + 102 + 8 * d)
            dl.append(dict(x=x, v=v, x1=x1, ln1=ln1, q=q, qp=qp, probs=probs, psum=psum, cc=cc, ctx=ctxd, x2=x2,
                           ln2=ln2, f1=f1, ln3=ln3))
            x = x3
        t["dec"] = dl
        return x

    def fuse_head_fwd(self, pooled, vis, cross, hard: bool, rng: int):
        """concat + min-max + privacy stage (one kernel) and the fc head over the three encoder
        outputs [B, 768] fp32 (model.py:46-63, past_acc.py:119-138, main_0430.py:116-122).
        Returns logits [B, 2] and the state the backward needs."""
        cfg = self.cfg
        B = pooled.shape[0]
        if self.v1:
            return self._v1_head_fwd(pooled, vis, cross, hard, rng)
        g = self.eh(B, FUSED)
        xn = self._f32(B, FUSED)
        amin = torch.empty(B, dtype=torch.int32, device=self.a.device)
        amax = torch.empty_like(amin)
        rng_ = self._f32(B)
        inj = self.injected or {}
        eps_a = math.exp(cfg.eps)
        ev = self._ev_start("fusion_fwd")
        call("eegf_fusion_fwd", F32, B, self.variant, P(pooled), pooled.stride(0), P(vis), vis.stride(0), P(cross),
             cross.stride(0),
             P(self.F("DP")) if "DP" in self.a.offsets else None, P(inj.get("noise")), P(inj.get("gumbels")),
             P(inj.get("row_noise")), int(hard), EPS_MODES.index(cfg.eps_mode), eps_a, 1.0 / cfg.eps,
             self.cfg.seed, rng + 200, P(g), P(xn), P(amin), P(amax), P(rng_), _stream())
        # algorithmic bytes: the three fp32 feature rows in; xn and the gated row out; arg-min / max / range
        self._ev_end("fusion_fwd", ev, 0.0, B * (3 * FUSED * 4 + 12) + FUSED * 4)
        z1 = self.eh(B, FUSED)
        self.linear(g, self.F("fc_layers.0.weight"), self.F("fc_layers.0.bias"), z1, B, epi=_lib.EPI_BIAS_RELU)
        z2 = self.eh(B, HID)
        self.linear(z1, self.F("fc_layers.2.weight"), self.F("fc_layers.2.bias"), z2, B, epi=_lib.EPI_BIAS_TANH)
        logits = self.eh(B, 2)
        self.linear(z2, self.F("classifier.weight"), self.F("classifier.bias"), logits, B)
        return logits, dict(fuse=dict(g=g, xn=xn, amin=amin, amax=amax, range=rng_, inj=inj),
                            head=dict(z1=z1, z2=z2))

    def _f32(self, *shape):
        return torch.empty(*shape, dtype=torch.float32, device=self.a.device)

    # =================================================================== backward
    def backward(self, sv: Saved, dlogits: torch.Tensor, head_only: bool = False):
        self.defer, self._defer_k = [], 0
        try:
            self._backward(sv, dlogits, head_only)
        finally:
            self._flush_colsums()

    def _backward(self, sv: Saved, dlogits: torch.Tensor, head_only: bool = False):
        """Accumulate parameter gradients into the arena grad buffer (beta = 1 everywhere; the
        caller zeroes the ranges it overwrites).  head_only: stop after the privacy stage
        (DP gradient only — the PriGumbel DP pass)."""
        cfg = self.cfg
        t = sv.t
        ddrop = cfg.dec_dropout if sv.training else 0.0
        d1, d2, d3 = self.fuse_head_bwd(t, dlogits, sv.hard, sv.rng)
        if head_only:
            return
        modal, B = cfg.modal, sv.B
        if modal == "ii":
            dva = self.eh(B, HID)                                   # decoder memory (action token) grad
            dx = self._dec1_bwd(t, d3, dva, ddrop, sv.rng)
            call("eegf_axpby", F32, B * HID, 1.0, P(dx), 1.0, P(d1), _stream())
            call("eegf_axpby", F32, B * HID, 1.0, P(d2), 1.0, P(dva), _stream())
            self._visual_bwd(d1, t["act"])
            self._visual_bwd(dva, t["act2"])
            self._ready(lambda n: True)
            return
        L = sv.L
        if modal == "tt":
            dmem = self.empty(2 * B * L, HID)                       # [eeg rows | act rows]
            self._seqdec_bwd(t, d3, dmem[B * L:], dmem[:B * L], B, L, ddrop, sv.rng)
            dpool = self.eh(2 * B, HID)
            call("eegf_axpby", F32, B * HID, 1.0, P(d1), 0.0, P(dpool[:B]), _stream())
            call("eegf_axpby", F32, B * HID, 1.0, P(d2), 0.0, P(dpool[B:]), _stream())
            self._bert_bwd(sv, dmem, dpool)
            return
        if modal == "tisc":
            dX = self.eh(2 * B, HID)
            call("eegf_seq_mean_bwd", F32, B, 2, HID, P(d3), HID, P(dX), HID, 0.0, _stream())
            self._enc2_bwd(t, dX, B, ddrop, sv.rng)                 # dX <- d(encoder input)
            dmem = self.empty(B * L, HID)
            call("eegf_seq_mean_bwd", self.code, B, L, HID, P(dX), 2 * HID, P(dmem), HID, 0.0, _stream())
            self._visual_bwd(d2, t["act"])
            self._visual_bwd(dX[1::2], t["act"], ldd=2 * HID)
            self._bert_bwd(sv, dmem, d1)
            return
        dpooled, dvis = (d2, d1) if modal == "it" else (d1, d2)
        dmem = self.empty(B * L, HID)
        dx = self._dec1_bwd(t, d3, dmem, ddrop, sv.rng)
        # vis receives the fusion path + the decoder path
        call("eegf_axpby", F32, B * HID, 1.0, P(dx), 1.0, P(dvis), _stream())
        self._visual_bwd(dvis, t["act"])
        self._bert_bwd(sv, dmem, dpooled)

    def _visual_bwd(self, dvis, act, ldd=None):
        B = act.shape[0]
        self.wgrad(dvis, act, "visual_encoder.weight", B, ldd=ldd)
        self.bgrad(dvis, "visual_encoder.bias", B, ld=ldd)

    def _dec1_bwd(self, t, dcross, dmem, ddrop, rng):
        """backward of _dec1_fwd: writes the memory gradient into dmem (overwritten) and returns the
        query-token (tgt) gradient [B, 768] fp32."""
        mem, L, _ = t["dmem_src"]
        B = dcross.shape[0]
        dx3 = dcross
        scale = DH ** -0.5
        for d in reversed(range(DEC_L)):
            pre = f"multi_head_decoder.layers.{d}."
            s = t["dec"][d]
            df2, dx2 = self.eh(B, HID), self.eh(B, HID)
            self.ln_bwd(dx3, *s["ln3"], pre + "norm3", B, df2, dx2, ddrop, 1, rng + 102 + 8 * d)
            self.wgrad(df2, s["f1"], pre + "linear2.weight", B)
            self.bgrad(df2, pre + "linear2.bias", B)
            df1 = self.eh(B, DEC_FF)
            # f1 holds dropout(relu(.)): f1 > 0 exactly where both the mask and the ReLU pass
            self.dgrad(df2, self.F(pre + "linear2.weight"), df1, B, epi=_lib.EPI_DRELU, aux=s["f1"],
                       scale=1.0 / (1.0 - ddrop))
            self.wgrad(df1, s["x2"], pre + "linear1.weight", B)
            self.bgrad(df1, pre + "linear1.bias", B)
            self.dgrad(df1, self.F(pre + "linear1.weight"), dx2, B, beta=1.0)
            dca, dx1 = self.eh(B, HID), self.eh(B, HID)
            self.ln_bwd(dx2, *s["ln2"], pre + "norm2", B, dca, dx1, ddrop, 1, rng + 101 + 8 * d)
            self.wgrad(dca, s["ctx"], pre + "multihead_attn.out_proj.weight", B)
            self.bgrad(dca, pre + "multihead_attn.out_proj.bias", B)
            dctx = self.eh(B, HID)
            self.dgrad(dca, self.F(pre + "multihead_attn.out_proj.weight"), dctx, B)
            cw = self.F(pre + "multihead_attn.in_proj_weight")
            gname = pre + "multihead_attn.in_proj_weight"
            bname = pre + "multihead_attn.in_proj_bias"
            if self.need(gname):
                gw = self.G(gname)
                # dWv_h[n, c] = sum_b dctx[b, h*64+n] cc[b,h,c]
                self.gemm(dctx, s["cc"], gw[2 * HID:], DH, HID, B, 0, 0, HID, NH * HID, HID, beta=1.0, batch=NH,
                          sA=DH, sB=HID, sC=DH * HID)
            dpsum = None
            if s["psum"] is not None:
                dpsum = self._f32(B, NH)
                call("eegf_head_bias_bwd", B, HID, DH, P(dctx), P(self.F(bname)[2 * HID:]), P(s["psum"]), P(dpsum),
                     P(self.G(bname)[2 * HID:]) if self.need(bname) else None, 1.0, _stream())
            elif self.need(bname):
                self.bgrad(dctx, bname, B, out=self.G(bname)[2 * HID:])
            dcc = self.eh(B, NH, HID)
            # dcc[b,h,c] = sum_n dctx[b, h*64+n] Wv[h*64+n, c]
            self.gemm(dctx, cw[2 * HID:], dcc, B, HID, DH, 1, 0, HID, HID, NH * HID, batch=NH, sA=DH, sB=DH * HID,
                      sC=HID)
            dqp = self.eh(B, NH, HID)
            xws = self.ws.get("xattn", B * NH * L, torch.float32)
            call("eegf_xattn_bwd", _code(mem), F32, B, L, P(mem), P(s["qp"]), P(s["probs"]), P(dpsum), P(dcc),
                 float(ddrop), self.cfg.seed, rng + 104 + 8 * d, P(xws), P(dmem), 0.0 if d == DEC_L - 1 else 1.0,
                 P(dqp), _stream())
            dq = self.eh(B, HID)
            # dq[b, h*64+i] = sum_c dqp[b,h,c] Wk[h*64+i, c] / 8
            self.gemm(dqp, cw[HID:2 * HID], dq, B, DH, HID, 1, 1, NH * HID, HID, HID, alpha=scale, batch=NH, sA=HID,
                      sB=DH * HID, sC=DH)
            if self.need(gname):
                # dWk_h[i, c] = sum_b q[b, h*64+i] dqp[b,h,c] / 8
                self.gemm(s["q"], dqp, gw[HID:2 * HID], DH, HID, B, 0, 0, HID, NH * HID, HID, alpha=scale, beta=1.0,
                          batch=NH, sA=DH, sB=HID, sC=DH * HID)
                self.gemm(dq, s["x1"], gw[:HID], HID, HID, B, 0, 0, HID, HID, HID, beta=1.0)
            if self.need(bname):
                self.bgrad(dq, bname, B, out=self.G(bname)[:HID])
            self.dgrad(dq, cw[:HID], dx1, B, beta=1.0)
            dsa, dx = self.eh(B, HID), self.eh(B, HID)
            self.ln_bwd(dx1, *s["ln1"], pre + "norm1", B, dsa, dx, ddrop, 1, rng + 100 + 8 * d)
            self.wgrad(dsa, s["v"], pre + "self_attn.out_proj.weight", B)
            self.bgrad(dsa, pre + "self_attn.out_proj.bias", B)
            dv = self.eh(B, HID)
            self.dgrad(dsa, self.F(pre + "self_attn.out_proj.weight"), dv, B)
            self.dropout(dv, 64, ddrop, rng + 103 + 8 * d)
            sw = self.F(pre + "self_attn.in_proj_weight")
            if self.need(pre + "self_attn.in_proj_weight"):
                self.gemm(dv, s["x"], self.G(pre + "self_attn.in_proj_weight")[2 * HID:], HID, HID, B, 0, 0, HID, HID,
                          HID, beta=1.0)
            if self.need(pre + "self_attn.in_proj_bias"):
                self.bgrad(dv, pre + "self_attn.in_proj_bias", B, out=self.G(pre + "self_attn.in_proj_bias")[2 * HID:])
            self.dgrad(dv, sw[2 * HID:], dx, B, beta=1.0)
            dx3 = dx
        return dx3

    def _bert_bwd(self, sv, dmem, dpooled):
        """pooler + BertModel + EEG front-end backward from the sequence-output gradient dmem
        [B*L, 768] (padded layout, encoder dtype; the pooler's part is added here) and dpooled fp32."""
        cfg = self.cfg
        t = sv.t
        B, L = sv.Bb, sv.L
        R, vl = sv.R or B * L, sv.vl
        packed = vl is not None and not vl.get("uniform")
        pdrop = cfg.hidden_dropout if sv.training else 0.0
        adrop = cfg.attn_dropout if sv.training else 0.0
        mem = t["mem"]
        scale = DH ** -0.5
        # ---------------- pooler (fp32 tanh derivative, encoder-dtype GEMMs)
        pooled = t["pooled"]
        dpp32 = self.eh(B, HID)
        call("eegf_tanh_bwd", F32, B * HID, P(dpooled), P(pooled), P(dpp32), _stream())
        self.bgrad(dpp32, "bert.pooler.dense.bias", B)
        if self.dt == torch.float32:
            dpp = dpp32
        else:
            dpp = self.empty(B, HID)
            call("eegf_cast_f32_bf16", B * HID, P(dpp32), P(dpp), _stream())
        self.wgrad(dpp, mem, "bert.pooler.dense.weight", B, ldx=L * HID)
        self.dgrad(dpp, self.W("bert.pooler.dense.weight"), dmem, B, ldo=L * HID, beta=1.0)

        # decoder / head / pooler / visual weight matrices are final here
        self._ready(lambda n: not n.startswith(("bert.encoder.", "bert.embeddings.", "eeg_encoder.")))

        # ---------------- BERT encoder backward
        dh = dmem
        if packed:                # padded memory gradient -> the packed rows (zeros past the tokens)
            dh = self.empty(R, HID)
            call("eegf_varlen_rows", self.code, B, L, HID, P(vl["cu"]), vl["T"], R, P(dmem), HID, P(dh), HID, 0,
                 _stream())
        dfo = self.ws.get("b_dfo", R * HID, self.dt).view(R, HID)
        da = self.ws.get("b_da", R * HID, self.dt).view(R, HID)
        dffp = self.ws.get("b_dffp", R * FFN, self.dt).view(R, FFN)
        dao = self.ws.get("b_dao", R * HID, self.dt).view(R, HID)
        dctx = self.ws.get("b_dctx", R * HID, self.dt).view(R, HID)
        dqkv = self.ws.get("b_dqkv", R * 3 * HID, self.dt).view(R, 3 * HID)
        dq_ws_n = (_lib.lib().eegf_attn_bwd_workspace(B, L) if vl is None
                   else _lib.lib().eegf_attn_varlen_bwd_workspace(R, L))
        dq_ws = self.ws.get("b_dqws", dq_ws_n, torch.float32) if dq_ws_n > 0 else None
        lowest = self._lowest_needed_layer()
        for i in reversed(range(NL)):
            if i < lowest:
                break
            pre = f"bert.encoder.layer.{i}."
            s = t["layers"][i]
            dhn = self.ws.get(f"b_dh{i % 2}", R * HID, self.dt).view(R, HID)
            self.ln_bwd(dh, *s["ln2"], pre + "output.LayerNorm", R, dfo, da, pdrop, 1, sv.rng + 11 + 3 * i)
            # bias gradients ride on the weight-gradient GEMMs (eegf_gemm_wgrad_bias)
            self.wgrad(dfo, s["ffact"], pre + "output.dense.weight", R, bias=pre + "output.dense.bias")
            self.dgrad(dfo, self.W(pre + "output.dense.weight"), dffp, R, epi=_lib.EPI_MUL_AUX, aux=s["ffgd"],
                       tag="dgrad_ffn2")
            self.wgrad(dffp, s["a1"], pre + "intermediate.dense.weight", R, bias=pre + "intermediate.dense.bias")
            self.dgrad(dffp, self.W(pre + "intermediate.dense.weight"), da, R, beta=1.0, tag="dgrad_ffn1")
            self.ln_bwd(da, *s["ln1"], pre + "attention.output.LayerNorm", R, dao, dhn, pdrop, 1, sv.rng + 10 + 3 * i)
            self.wgrad(dao, s["ctx"], pre + "attention.output.dense.weight", R,
                       bias=pre + "attention.output.dense.bias")
            self.dgrad(dao, self.W(pre + "attention.output.dense.weight"), dctx, R, tag="dgrad_out")
            ev = self._ev_start("attn_bwd")
            if vl is None:
                call("eegf_attn_bwd", self.code, B, NH, L, P(s["qkv"]), 3 * HID, P(t["kbias"]), scale, float(adrop),
                     self.cfg.seed, sv.rng + 12 + 3 * i, P(s["ctx"]), P(dctx), HID, P(s["lse"]), P(s["bits"]),
                     P(dqkv), P(dq_ws), _stream())
            else:
                call("eegf_attn_varlen_bwd", self.code, B, NH, L, P(vl["cu"]), vl["T"], R, P(s["qkv"]), 3 * HID,
                     P(vl.get("kbias")), scale, float(adrop), self.cfg.seed, sv.rng + 12 + 3 * i, P(s["ctx"]), P(dctx),
                     HID, P(s["lse"]), P(dqkv), P(dq_ws), _stream())
            self._ev_end("attn_bwd", ev, 2.5 * 4.0 * B * NH * L * L * DH)
            qn = pre + "attention.self.query.weight"
            bn = pre + "attention.self.query.bias"
            gb = self.a.span(bn, 3, self.a.grad) if self.need(bn) else None
            if self.need(qn):
                gq = self.a.span(qn, 3, self.a.grad).view(3 * HID, HID)
                self.wgrad(dqkv, s["h"], qn, R, ldd=3 * HID, gw=gq, gb=gb)
            elif gb is not None:
                self.bgrad(dqkv, bn, R, width=3 * HID, out=gb)
            if i > lowest or lowest == 0:
                self.dgrad(dqkv, self.Wspan(qn, 3).view(3 * HID, HID), dhn, R, beta=1.0, tag="dgrad_qkv")
            self._ready(lambda n, pre=pre: n.startswith(pre))
            dh = dhn
        if lowest > 0:
            return
        # ---------------- embeddings
        e = "bert.embeddings."
        demb = self.ws.get("b_demb", R * HID, self.dt).view(R, HID)
        self.ln_bwd(dh, *t["emb"], e + "LayerNorm", R, demb, None, pdrop, 2, sv.rng + 1)
        if self.need(e + "position_embeddings.weight"):
            dpos = demb
            if packed:            # position j of every sequence: the padded layout's period-L column sums
                dpos = self.empty(B * L, HID)
                call("eegf_varlen_rows", self.code, B, L, HID, P(vl["cu"]), vl["T"], R, P(demb), HID, P(dpos), HID,
                     1, _stream())
            self.bgrad(dpos, e + "position_embeddings.weight", B * L, width=HID, period=L,
                       out=self.G(e + "position_embeddings.weight")[:L])
        if self.need(e + "token_type_embeddings.weight"):
            self.bgrad(demb, e + "token_type_embeddings.weight", R, width=HID,
                       out=self.G(e + "token_type_embeddings.weight")[0])
        if cfg.contract == "W":
            self.wgrad(demb, t["tok"], "eeg_encoder.weight", R)
            self.bgrad(demb, "eeg_encoder.bias", R)
        elif self.need(e + "word_embeddings.weight"):
            call("eegf_embed_scatter_add", self.code, R, HID, P(t["ids"]), P(demb),
                 P(self.G(e + "word_embeddings.weight")), _stream())

    def fuse_head_bwd(self, t: dict, dlogits: torch.Tensor, hard: bool, rng: int):
        """Backward of fuse_head_fwd: head weight / bias gradients and the DP gradient (PriGumbel)
        into the arena; returns dL/d(pooled, vis, cross) [B, 768] fp32."""
        cfg = self.cfg
        dlogits = dlogits.float().contiguous()
        B = dlogits.shape[0]
        if self.v1:
            return self._v1_head_bwd(t, dlogits, hard, rng)
        hd = t["head"]
        fz = t["fuse"]
        g = fz["g"]
        self.wgrad(dlogits, hd["z2"], "classifier.weight", B)
        self.bgrad(dlogits, "classifier.bias", B)
        dz2 = self.eh(B, HID)
        self.dgrad(dlogits, self.F("classifier.weight"), dz2, B, epi=_lib.EPI_DTANH, aux=hd["z2"])
        self.wgrad(dz2, hd["z1"], "fc_layers.2.weight", B)
        self.bgrad(dz2, "fc_layers.2.bias", B)
        dz1 = self.eh(B, FUSED)
        self.dgrad(dz2, self.F("fc_layers.2.weight"), dz1, B, epi=_lib.EPI_DRELU, aux=hd["z1"])
        self.wgrad(dz1, g, "fc_layers.0.weight", B)
        self.bgrad(dz1, "fc_layers.0.bias", B)
        dg = self.eh(B, FUSED)
        self.dgrad(dz1, self.F("fc_layers.0.weight"), dg, B)
        dpooled, dvis, dcross = self.eh(B, HID), self.eh(B, HID), self.eh(B, HID)
        has_dp = "DP" in self.a.offsets and self.variant == _lib.FUSE_PRIGUMBEL and self.need("DP")
        ddp = self._f32(B, FUSED) if has_dp else None
        inj = fz["inj"]
        ev = self._ev_start("fusion_bwd")
        call("eegf_fusion_bwd", F32, B, self.variant, P(dg), P(fz["xn"]), P(fz["amin"]), P(fz["amax"]),
             P(fz["range"]), P(self.F("DP")) if "DP" in self.a.offsets else None, P(inj.get("noise")),
             P(inj.get("gumbels")), int(hard), EPS_MODES.index(cfg.eps_mode), math.exp(cfg.eps),
             self.cfg.seed, rng + 200, P(dpooled), HID, P(dvis), HID, P(dcross), HID, P(ddp), _stream())
        # dout and xn in, the three input-gradient rows out (+ the per-row DP gradient rows in pass 1)
        self._ev_end("fusion_bwd", ev, 0.0, B * ((3 + (1 if has_dp else 0)) * FUSED * 4 + 12) + FUSED * 4)
        if has_dp:
            self.bgrad(ddp, "DP", B, FUSED)
        return dpooled, dvis, dcross

    # ------------------------------------------------------------- PriGumbel-v1 head
    def _v1_head_fwd(self, pooled, vis, cross, hard, rng):
        """train_val.py:152-157: feature_concat -> relu(fc1) -> fc2 -> gumbel_dropout(w, tau) ->
        Lap_noise (row min-max + Laplace(0, 1/eps)) -> classifier (768 -> 2)."""
        cfg = self.cfg
        B = pooled.shape[0]
        inj = self.injected or {}
        g = self.eh(B, FUSED)
        call("eegf_fusion_fwd", F32, B, _lib.FUSE_PRICONCAT, P(pooled), pooled.stride(0), P(vis), vis.stride(0),
             P(cross), cross.stride(0), None, None,
             None, None, 0, 0, math.exp(cfg.eps), 1.0 / cfg.eps, self.cfg.seed, rng + 200, P(g), None, None, None,
             None, _stream())
        z1 = self.eh(B, FUSED)
        self.linear(g, self.F("fc1.weight"), self.F("fc1.bias"), z1, B, epi=_lib.EPI_BIAS_RELU)
        x = self.eh(B, HID)
        self.linear(z1, self.F("fc2.weight"), self.F("fc2.bias"), x, B)
        out, xn = self.eh(B, HID), self._f32(B, HID)
        amin = torch.empty(B, dtype=torch.int32, device=self.a.device)
        amax = torch.empty_like(amin)
        rg = self._f32(B)
        call("eegf_v1_gate_fwd", B, P(x), HID, P(self.F("w")), P(inj.get("v1_gumbels")), P(inj.get("row_noise")),
             float(cfg.tau), int(hard), 1.0 / cfg.eps, self.cfg.seed, rng + 200, P(out), P(xn), P(amin), P(amax),
             P(rg), _stream())
        logits = self.eh(B, 2)
        self.linear(out, self.F("classifier.weight"), self.F("classifier.bias"), logits, B)
        return logits, dict(fuse=dict(g=g, xn=xn, amin=amin, amax=amax, range=rg, inj=inj),
                            head=dict(z1=z1, x=x, out=out))

    def _v1_head_bwd(self, t, dlogits, hard, rng):
        cfg = self.cfg
        B = dlogits.shape[0]
        hd, fz = t["head"], t["fuse"]
        self.wgrad(dlogits, hd["out"], "classifier.weight", B)
        self.bgrad(dlogits, "classifier.bias", B)
        dout = self.eh(B, HID)
        self.dgrad(dlogits, self.F("classifier.weight"), dout, B)
        dx = self.eh(B, HID)
        dw = self._f32(B, HID) if self.need("w") else None
        call("eegf_v1_gate_bwd", B, P(dout), P(hd["x"]), HID, P(self.F("w")), P(fz["inj"].get("v1_gumbels")),
             P(fz["xn"]), P(fz["amin"]), P(fz["amax"]), P(fz["range"]), float(cfg.tau), int(hard), self.cfg.seed,
             rng + 200, P(dx), P(dw), _stream())
        if dw is not None:
            self.bgrad(dw, "w", B, HID)
        self.wgrad(dx, hd["z1"], "fc2.weight", B)
        self.bgrad(dx, "fc2.bias", B)
        dz1 = self.eh(B, FUSED)
        self.dgrad(dx, self.F("fc2.weight"), dz1, B, epi=_lib.EPI_DRELU, aux=hd["z1"])
        self.wgrad(dz1, fz["g"], "fc1.weight", B)
        self.bgrad(dz1, "fc1.bias", B)
        dg = self.eh(B, FUSED)
        self.dgrad(dz1, self.F("fc1.weight"), dg, B)
        dpooled, dvis, dcross = self.eh(B, HID), self.eh(B, HID), self.eh(B, HID)
        call("eegf_fusion_bwd", F32, B, _lib.FUSE_PRICONCAT, P(dg), None, None, None, None, None, None, None, 0, 0,
             math.exp(cfg.eps), self.cfg.seed, rng + 200, P(dpooled), HID, P(dvis), HID, P(dcross), HID, None,
             _stream())
        return dpooled, dvis, dcross

    def v1_wloss(self, dscale: float, loss: torch.Tensor | None = None):
        """loss_function's max_j((1 - w_j) e^eps + w_j) term (train_val.py:88-90): value into `loss`
        (nullable) and dscale * d/dw into the arena gradient of w."""
        call("eegf_v1_wloss", HID, P(self.F("w")), math.exp(self.cfg.eps), float(dscale), P(loss),
             P(self.G("w")) if self.need("w") else None, _stream())

    def _ready(self, pred):
        """Report weight matrices matching pred as final.  Vectors (biases, LayerNorm, embeddings,
        DP) are left out: their column sums are deferred to the end of the backward."""
        if self.grad_ready is None:
            return
        gp = self.graph_params()
        names = [n for n, (_, shp) in self.a.offsets.items()
                 if n in gp and self.need(n) and pred(n) and len(shp) == 2 and n != "DP"
                 and "norm" not in n.lower() and "embeddings" not in n]
        if names:
            self.grad_ready(names)

    def _lowest_needed_layer(self) -> int:
        if self.needs_grad is None:
            return 0
        emb = any(n.startswith(("bert.embeddings", "eeg_encoder")) for n in self.needs_grad)
        if emb:
            return 0
        for i in range(NL):
            if any(n.startswith(f"bert.encoder.layer.{i}.") for n in self.needs_grad):
                return i
        return NL

    # ------------------------------------------------------------- graph membership
    def graph_params(self) -> set[str]:
        """Parameters that take part in the forward graph (others keep grad None, as in torch)."""
        out = set()
        for n in self.a.offsets:
            if n.startswith(("multi_head_decoderlayer.", "multi_head_encoderlayer.")):
                continue                                  # unused template layer (model.py:20, models.py:227)
            if n == "bert.embeddings.word_embeddings.weight" and self.cfg.contract == "W":
                continue
            if n == "DP" and self.variant != _lib.FUSE_PRIGUMBEL:
                continue
            out.add(n)
        return out


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _code(t):
    return F32 if t.dtype == torch.float32 else BF16
