"""Drop-in nn.Module mirrors of the reference model classes, backed by the HIP engine.

The module tree reproduces the reference's attribute names and state_dict keys exactly
(`bert.embeddings.*`, `bert.encoder.layer.{i}.*`, `bert.pooler.dense.*`, `visual_encoder.*`,
`multi_head_decoderlayer.*` (unused template, model.py:20), `multi_head_decoder.layers.{0,1,2}.*`,
`fc_layers.{0,2}.*`, `classifier.*`, `DP`), so `load_state_dict` of a reference checkpoint works and
callers that touch `.bert.encoder.layer[-1]`, `.fc_layers`, `.classifier`, `.DP`, `.eps`
(train.py:139, main_0430.py:144-151) keep working.  The submodules are parameter holders only:
every parameter is a view into the engine's ParamArena and, for a model on the GPU, every FLOP runs
in libeegfusion.so.  A model left in host memory (configs[0]'s no-GPU plumbing run) computes with
plain torch ops (eegfusion/cpu_path.py, the "ti" models); a device model never falls back to it.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn

from .arena import ParamArena
from .engine import DEC_FF, DEC_L, FFN, FUSED, HID, NL, EngineConfig, FusionEngine

# ------------------------------------------------------------------- name-holding modules


class _Holder(nn.Module):
    def forward(self, *a, **k):  # pragma: no cover - never called
        raise RuntimeError("eegfusion submodules are parameter holders; call the top-level model")


def _linear(i, o, bias=True):
    m = nn.Linear(i, o, bias=bias)
    return m


def _bert(vocab=30522, max_pos=512):
    bert = _Holder()
    emb = _Holder()
    emb.word_embeddings = nn.Embedding(vocab, HID, padding_idx=0)
    emb.position_embeddings = nn.Embedding(max_pos, HID)
    emb.token_type_embeddings = nn.Embedding(2, HID)
    emb.LayerNorm = nn.LayerNorm(HID, eps=1e-12)
    bert.embeddings = emb
    enc = _Holder()
    layers = []
    for _ in range(NL):
        L = _Holder()
        att = _Holder()
        selfa = _Holder()
        selfa.query, selfa.key, selfa.value = _linear(HID, HID), _linear(HID, HID), _linear(HID, HID)
        att.self = selfa
        out = _Holder()
        out.dense = _linear(HID, HID)
        out.LayerNorm = nn.LayerNorm(HID, eps=1e-12)
        att.output = out
        L.attention = att
        inter = _Holder()
        inter.dense = _linear(HID, FFN)
        L.intermediate = inter
        o2 = _Holder()
        o2.dense = _linear(FFN, HID)
        o2.LayerNorm = nn.LayerNorm(HID, eps=1e-12)
        L.output = o2
        layers.append(L)
    enc.layer = nn.ModuleList(layers)
    bert.encoder = enc
    pool = _Holder()
    pool.dense = _linear(HID, HID)
    bert.pooler = pool
    return bert


def _init_bert_(bert: nn.Module, std=0.02):
    """BertPreTrainedModel._init_weights: normal(0, 0.02) Linear/Embedding, zero bias, LN = (1, 0)."""
    for m in bert.modules():
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, std)
            nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, std)
            if m.padding_idx is not None:
                with torch.no_grad():
                    m.weight[m.padding_idx].zero_()
        elif isinstance(m, nn.LayerNorm):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)


_LAYER_MATRICES = ("attention.self.query.weight", "attention.self.key.weight", "attention.self.value.weight",
                   "attention.output.dense.weight", "intermediate.dense.weight", "output.dense.weight")


def _qkv_first_order(named):
    """Arena order: every BERT layer's six weight matrices first, layer after layer with no gap (Q|K|V
    adjacent, so the fused QKV projection reads one [2304, 768] matrix; each layer's block is one
    contiguous gradient range that the DDP reducer all-reduces as soon as that layer's backward is
    done, and the blocks of consecutive layers are adjacent, so a reducer bucket of several layers is
    one contiguous range too), then the remaining parameters in module order with each layer's Q/K/V
    biases adjacent."""
    named = list(named)
    byname = dict(named)
    out, seen = [], set()
    for n, _ in named:
        if n.endswith("attention.self.query.weight"):
            base = n[: -len("attention.self.query.weight")]
            for k in _LAYER_MATRICES:
                out.append((base + k, byname[base + k]))
                seen.add(base + k)
    for n, p in named:
        if n in seen:
            continue
        if n.endswith("attention.self.query.bias"):
            base = n[: -len("attention.self.query.bias")]
            for k in ("attention.self.query.bias", "attention.self.key.bias", "attention.self.value.bias"):
                out.append((base + k, byname[base + k]))
                seen.add(base + k)
        else:
            out.append((n, p))
            seen.add(n)
    return out


class _PathFunction(torch.autograd.Function):
    """One autograd node for the whole path: forward/backward are HIP launch sequences; parameter
    gradients are written straight into the arena and published as `.grad` views."""

    @staticmethod
    def forward(ctx, model, batch_keys, hard, *tensors):
        batch = dict(zip(batch_keys, tensors[: len(batch_keys)]))
        logits, saved = model._engine.forward(batch, hard, model.training, save=True)
        ctx.model, ctx.saved = model, saved
        return logits.float()

    @staticmethod
    def backward(ctx, dlogits):
        ctx.model._backward(ctx.saved, dlogits)
        ctx.saved = None
        return (None, None, None) + (None,) * (len(ctx.needs_input_grad) - 3)


class _EmptyBatch(torch.autograd.Function):
    """logits [0, 2] for an empty batch; its backward sets zero gradients on the trainable params"""

    @staticmethod
    def forward(ctx, model, *params):
        ctx.model = model
        return torch.zeros(0, 2, device=model.arena.device)

    @staticmethod
    def backward(ctx, dlogits):
        m = ctx.model
        for n, p in m.named_parameters():
            if p.requires_grad and p.grad is None:
                g = m.arena.gview(n)
                g.zero_()
                p.grad = g
        return (None,) * (len(ctx.needs_input_grad))


class FusionModel(nn.Module):
    """Common body of ConcatModel / PriConcat / PriGumbel / TICA_LapDropout."""

    def __init__(self, variant: str, contract: str = "T", eps: float = 1.0, eps_mode: str = "newfrac",
                 dtype: torch.dtype = torch.float32, eeg_channels: int = 64, act_dim: int = 32, frame_dim: int = 512,
                 with_dp: bool = True, dp_init: torch.Tensor | None = None, dropout: float = 0.1, seed: int = 980616,
                 tau: float = 1.0, modal: str = "ti", host_path: bool = False):
        super().__init__()
        self._variant, self._contract, self._modal = variant, contract, modal
        # host_path=True: run the torch-op host path (cpu_path) while the model is in host memory even
        # when a GPU is present (e.g. CPU evaluation beside a busy GPU); otherwise that case is refused
        self.host_path = bool(host_path)
        # module sets of the custom_models variants (models.py:28-272): no BERT in IICA, no visual
        # encoder in TTCA, a TransformerEncoder instead of the decoder in TISC
        if modal != "ii":
            self.bert = _bert()
            _init_bert_(self.bert)
        if contract == "W":
            self.eeg_encoder = nn.Linear(eeg_channels, HID)
            self.visual_encoder = nn.Linear(act_dim, HID)
        elif modal != "tt":
            self.visual_encoder = nn.Linear(frame_dim, HID)
        if modal == "tisc":
            self.multi_head_encoderlayer = nn.TransformerEncoderLayer(d_model=HID, nhead=12)
            self.multi_head_encoder = nn.TransformerEncoder(self.multi_head_encoderlayer, num_layers=DEC_L,
                                                            enable_nested_tensor=False)
        else:
            self.multi_head_decoderlayer = nn.TransformerDecoderLayer(d_model=HID, nhead=12)
            self.multi_head_decoder = nn.TransformerDecoder(self.multi_head_decoderlayer, num_layers=DEC_L)
        if variant == "prigumbel_v1":
            # train_val.py:125-142 registration order: classifier (first assigned at :134), w, dropout,
            # fc1, fc2; no fc_layers, no DP
            self.classifier = nn.Linear(HID, 2)
            self.w = nn.Parameter(torch.rand(HID))
            self.dropout = GumbelSoftmaxDropout(tau)
            self.fc1 = nn.Linear(FUSED, FUSED)
            self.fc2 = nn.Linear(FUSED, HID)
            with_dp = False
        else:
            self.dropout = nn.Dropout(0.1)
            self.fc_layers = nn.Sequential(nn.Linear(FUSED, FUSED), nn.ReLU(), nn.Linear(FUSED, HID), nn.Tanh())
            self.classifier = nn.Linear(HID, 2)
        if with_dp:
            self.DP = nn.Parameter(torch.zeros(1, FUSED) if dp_init is None else dp_init.reshape(1, FUSED).float())
        self.noiser = torch.distributions.laplace.Laplace(torch.tensor([0.0]), torch.tensor([1.0]))
        self.eps = torch.tensor(eps)
        self._cfg = EngineConfig(contract=contract, variant=variant, dtype=dtype, eps=float(eps), eps_mode=eps_mode,
                                 hidden_dropout=dropout, attn_dropout=dropout, dec_dropout=dropout,
                                 eeg_channels=eeg_channels, act_dim=act_dim, seed=seed, tau=float(tau), modal=modal)
        self._build_arena(torch.device("cpu"))
        self._dp = None                      # DP-SGD state (eegfusion.dpsgd.GradSampleModule)

    # ------------------------------------------------------------------ arena binding
    def _build_arena(self, device):
        named = _qkv_first_order(self.named_parameters())
        arena = ParamArena([(n, tuple(p.shape)) for n, p in named], device)
        with torch.no_grad():
            for n, p in named:
                arena.view(n).copy_(p.detach().to(device))
                p.data = arena.view(n)
        self._arena = arena
        self._engine = FusionEngine(arena, self._cfg)

    def _apply(self, fn, recurse=True):
        # .cuda()/.to()/.half() would re-allocate each parameter separately; instead move the
        # arena once and re-bind every parameter view (dtype conversions are not supported).
        probe = fn(torch.zeros(1))
        if probe.dtype != torch.float32:
            raise RuntimeError("eegfusion models keep fp32 master weights; use compute_dtype= for bf16")
        if probe.device != self._arena.device:
            self._arena.to(probe.device)
            for n, p in self.named_parameters():
                p.data = self._arena.view(n)
                p.grad = None
            self._engine = FusionEngine(self._arena, self._engine.cfg)
        return self

    def set_compute_dtype(self, dtype: torch.dtype):
        self._cfg.dtype = dtype
        self._engine = FusionEngine(self._arena, self._cfg)
        return self

    @property
    def engine(self) -> FusionEngine:
        return self._engine

    @property
    def arena(self) -> ParamArena:
        return self._arena

    # ------------------------------------------------------------------ forward / backward
    def _check_device(self, *ts):
        if not self._arena.device.type == "cuda":
            raise RuntimeError("eegfusion runs on the GPU only (libeegfusion.so); call model.cuda() first")
        for t in ts:
            if t is not None and not t.is_cuda:
                raise RuntimeError("eegfusion: inputs must be device tensors (no CPU path)")

    def _host(self, *ts) -> bool:
        """True when the model lives in host memory (cpu_path); mixed host/device operands raise"""
        if self._arena.device.type != "cpu":
            return False
        if any(t is not None and t.is_cuda for t in ts):
            raise RuntimeError("eegfusion: the model is in host memory but the inputs are device tensors; "
                               "call model.cuda()")
        # the host path serves machines without a GPU (BASELINE configs[0]); on a GPU machine a model
        # left in host memory is almost always a forgotten .cuda() and would run orders of magnitude
        # slower without a word, so it is refused unless the model asks for it (host_path=True, or the
        # process-wide EEGF_HOST_PATH=1 for scripts that cannot pass the argument)
        if torch.cuda.is_available() and not self.host_path and os.environ.get("EEGF_HOST_PATH") != "1":
            raise RuntimeError("eegfusion: the model is in host memory while a GPU is present; call model.cuda() "
                               "(or construct it with host_path=True to run the torch-op host path on purpose)")
        return True

    def _run(self, batch: dict, hard: bool) -> torch.Tensor:
        if self._host(*batch.values()):
            from .cpu_path import forward as host_forward
            self._engine.cfg.eps = float(self.eps)
            return host_forward(self, batch, bool(hard))
        self._check_device(*batch.values())
        self._engine.cfg.eps = float(self.eps)
        params = [p for p in self.parameters() if p.requires_grad]
        if next(iter(batch.values())).shape[0] == 0:
            # an empty batch (DP-SGD Poisson sampling draws them): no launches; the backward leaves
            # zero gradients so the private step adds noise only (opacus semantics)
            return _EmptyBatch.apply(self, *params)
        if torch.is_grad_enabled() and params:
            keys = tuple(batch)
            return _PathFunction.apply(self, keys, bool(hard), *batch.values(), *params)
        logits, _ = self._engine.forward(batch, bool(hard), self.training, save=False)
        return logits.float()

    def _backward(self, saved, dlogits):
        eng = self._engine
        names = dict(self.named_parameters())
        in_graph = eng.graph_params()
        need = {n for n, p in names.items() if p.requires_grad and n in in_graph}
        a = self._arena
        if self._dp is not None:
            from .dpsgd import private_backward
            private_backward(self, saved, dlogits, need)      # overwrites: sum_b c_b grad_b
            for n in need:
                names[n].grad = a.gview(n)
            return
        eng.needs_grad = need
        # grad routing: overwrite (zero first) params whose .grad is None, accumulate into our views
        for n in need:
            p = names[n]
            gv = a.gview(n)
            if p.grad is None:
                gv.zero_()
            elif p.grad.data_ptr() != gv.data_ptr():
                gv.copy_(p.grad)
        eng.backward(saved, dlogits)
        for n in need:
            p = names[n]
            if p.grad is None or p.grad.data_ptr() != a.gview(n).data_ptr():
                p.grad = a.gview(n)
        eng.needs_grad = None

    def forward_window(self, eeg: torch.Tensor, act: torch.Tensor, hard: bool = True) -> torch.Tensor:
        """Contract W: eeg [B, C, T] (channel x time) fp32, act [B, A] fp32 -> logits [B, 2]."""
        return self._run({"eeg": eeg.contiguous().float(), "act": act.contiguous().float()}, hard)

    def _token_batch(self, frame_input, vedio_mask, title_input, text_mask):
        if self._contract == "W":
            # contract-W models accept the window through the reference's argument slots:
            # title_input <- eeg [B,C,T], frame_input <- act [B,1,A]
            return {"eeg": title_input.contiguous().float(), "act": frame_input.reshape(frame_input.shape[0], -1)
                    .contiguous().float()}
        # token ids / mask arrive as [B, L], or [B, 1, L] when a pickle holds [1, L] per sample
        # (the shape data.py:25's comment names); both mean the same sequence
        B, L = title_input.shape[0], title_input.shape[-1]
        return {"title_input": title_input.reshape(B, L).contiguous().long(),
                "text_mask": text_mask.reshape(B, L).contiguous().long(),
                "frame_input": frame_input.contiguous().float()}

    def extra_repr(self):
        return f"variant={self._variant}, contract={self._contract}, compute={self._cfg.dtype}"


# ============================================================ reference-signature classes
class ConcatModel(FusionModel):
    """model.py:14-64 — ConcatModel(); forward(x, hard=True) with x = (frame_input [B,1,512],
    vedio_mask [B,1], title_input [B,512], text_mask [B,512]); min-max fused feature, no gate."""

    def __init__(self, contract: str = "T", **kw):
        super().__init__("concat", contract=contract, **kw)

    def feature(self, x):
        frame_input, vedio_mask, title_input, text_mask = x
        batch = self._token_batch(frame_input, vedio_mask, title_input, text_mask)
        if self._host(*batch.values()):
            from .cpu_path import forward as host_forward
            with torch.no_grad():
                return host_forward(self, batch, True, return_feature=True)[2]
        self._check_device(*batch.values())
        with torch.no_grad():
            _, sv = self._engine.forward(batch, True, self.training, save=False)
        return sv.t["fuse"]["g"].float()

    def forward(self, x, hard=True):
        frame_input, vedio_mask, title_input, text_mask = x
        return self._run(self._token_batch(frame_input, vedio_mask, title_input, text_mask), hard)


class PriConcatModel(FusionModel):
    """main_0430.py:88-123 — ConcatModel(args, dp_mode=None); forward(frame_input, vedio_mask,
    title_input, text_mask).  DP_guarantee is called with dp_mode=None there (:118), i.e. identity;
    honor_dp_mode=True applies 'feature_all_lap' (min-max + Laplace(0, 1/EPSILON) per row)."""

    def __init__(self, args=None, dp_mode=None, contract: str = "T", honor_dp_mode: bool = False, **kw):
        eps = float(getattr(args, "EPSILON", 1.0)) if args is not None else 1.0
        variant = "priconcat_lap" if (honor_dp_mode and dp_mode == "feature_all_lap") else "priconcat"
        super().__init__(variant, contract=contract, eps=eps, with_dp=False, **kw)
        self.dp_mode = dp_mode
        self.EPSILON = eps

    def forward(self, frame_input, vedio_mask, title_input, text_mask):
        return self._run(self._token_batch(frame_input, vedio_mask, title_input, text_mask), True)


class PriGumbelModel(FusionModel):
    """past_acc.py:79-139 — ConcatModel(epsilon); forward(frame_input, vedio_mask, title_input,
    text_mask, hard): Laplace noise scaled by eps_hat = 1/ln((e^eps - w)/(1 - w)), w = sigmoid(DP),
    then the Gumbel-softmax gate."""

    def __init__(self, epsilon: float = 1.0, contract: str = "T", eps_mode: str = "newfrac", **kw):
        super().__init__("prigumbel", contract=contract, eps=float(epsilon), eps_mode=eps_mode, **kw)

    def forward(self, frame_input, vedio_mask, title_input, text_mask, hard):
        return self._run(self._token_batch(frame_input, vedio_mask, title_input, text_mask), hard)


class TICA_LapDropout(FusionModel):
    """python/src/custom_models/models.py:28-82 — TICA_LapDropout(bert_coef); forward(eeg_txt_input,
    eeg_txt_mask, act_img_input, act_img_mask, epsilon, hard).  `bert_coef` names pretrained BERT
    weights: a local directory/safetensors path is loaded if it exists (no network)."""

    def __init__(self, bert_coef: str = "bert-base-uncased", contract: str = "T", **kw):
        super().__init__("prigumbel", contract=contract, **kw)
        if bert_coef and os.path.exists(str(bert_coef)):
            load_bert_weights(self, bert_coef)

    def forward(self, eeg_txt_input, eeg_txt_mask, act_img_input, act_img_mask, epsilon, hard):
        self.eps = torch.tensor(float(epsilon))
        return self._run(self._token_batch(act_img_input, act_img_mask, eeg_txt_input, eeg_txt_mask), hard)


class TICA_NonPrivate(FusionModel):
    """python/src/custom_models/models.py:309-352 — TICA_NonPrivate(bert_coef); forward(eeg_txt_input,
    eeg_txt_mask, act_img_input, act_img_mask): the TICA encoders, concat + min-max, fc head, no privacy
    stage and no DP parameter (model.py's ConcatModel computation under the TICA signature; base_train's
    'NDP' baseline)."""

    def __init__(self, bert_coef: str = "bert-base-uncased", contract: str = "T", **kw):
        super().__init__("concat", contract=contract, with_dp=False, **kw)
        if bert_coef and os.path.exists(str(bert_coef)):
            load_bert_weights(self, bert_coef)

    def forward(self, eeg_txt_input, eeg_txt_mask, act_img_input, act_img_mask):
        return self._run(self._token_batch(act_img_input, act_img_mask, eeg_txt_input, eeg_txt_mask), True)


def _tokens(x):
    """token ids / masks as [B, L] int64 (a pickle may hold [1, L] per sample: [B, 1, L] batches)"""
    return x.reshape(x.shape[0], x.shape[-1]).contiguous().long()


class _LapDropoutVariant(FusionModel):
    """Common body of the custom_models *_LapDropout variants: the PriGumbel newfrac gate over the
    variant's three fused features, forward(..., epsilon, hard)."""

    def __init__(self, modal: str, bert_coef=None, contract: str = "T", **kw):
        super().__init__("prigumbel", contract=contract, modal=modal, **kw)
        if bert_coef and os.path.exists(str(bert_coef)) and modal != "ii":
            load_bert_weights(self, bert_coef)

    def _go(self, batch, epsilon, hard):
        self.eps = torch.tensor(float(epsilon))
        return self._run(batch, hard)


class TTCA_LapDropout(_LapDropoutVariant):
    """models.py:84-129 — EEG and action both as text: one BERT (shared) over both token batches, the
    decoder with the action sequence as target and the EEG sequence as memory (no masks), mean over the
    target tokens; features BERT(eeg) pooled | BERT(act) pooled | cross."""

    def __init__(self, bert_coef: str = "bert-base-uncased", **kw):
        super().__init__("tt", bert_coef, **kw)

    def forward(self, eeg_txt_input, eeg_txt_mask, act_txt_input, act_txt_mask, epsilon, hard):
        return self._go({"title_input": _tokens(eeg_txt_input), "text_mask": _tokens(eeg_txt_mask),
                         "title_input2": _tokens(act_txt_input), "text_mask2": _tokens(act_txt_mask)}, epsilon, hard)


class ITCA_LapDropout(_LapDropoutVariant):
    """models.py:130-175 — EEG as image (CLIP vector through visual_encoder), action as text (BERT);
    the single-query decoder over the action sequence; features visual(eeg) | BERT(act) pooled | cross."""

    def __init__(self, bert_coef: str = "bert-base-uncased", **kw):
        super().__init__("it", bert_coef, **kw)

    def forward(self, eeg_img_input, eeg_img_mask, act_txt_input, act_txt_mask, epsilon, hard):
        return self._go({"title_input": _tokens(act_txt_input), "text_mask": _tokens(act_txt_mask),
                         "frame_input": eeg_img_input.contiguous().float()}, epsilon, hard)


class IICA_LapDropout(_LapDropoutVariant):
    """models.py:176-214 — both modalities as images: no BERT; visual_encoder (shared) on both CLIP
    vectors; the decoder with the EEG token as target and the action token as memory (length 1)."""

    def __init__(self, **kw):
        super().__init__("ii", None, **kw)

    def forward(self, eeg_img_input, eeg_img_mask, act_img_input, act_img_mask, epsilon, hard):
        return self._go({"frame_input": eeg_img_input.contiguous().float(),
                         "frame_input2": act_img_input.contiguous().float()}, epsilon, hard)


class TISC_LapDropout(_LapDropoutVariant):
    """models.py:215-272 — EEG as text, action as image, 'single attention': a 3-layer
    TransformerEncoder over the two tokens [mean of the BERT sequence output, action image embedding],
    mean over them; features BERT(eeg) pooled | visual(act) | encoder mean."""

    def __init__(self, bert_coef: str = "bert-base-uncased", **kw):
        super().__init__("tisc", bert_coef, **kw)

    def forward(self, eeg_txt_input, eeg_txt_mask, act_img_input, act_img_mask, epsilon, hard):
        return self._go({"title_input": _tokens(eeg_txt_input), "text_mask": _tokens(eeg_txt_mask),
                         "frame_input": act_img_input.contiguous().float()}, epsilon, hard)


class GumbelSoftmaxDropout(nn.Module):
    """train_val.py:103-112 holder (no parameters): tau; soft masks in train mode, hard in eval.  The
    computation is the engine's v1 gate (eegf_v1_gate_fwd / bwd)."""

    def __init__(self, tau):
        super().__init__()
        self.tau = tau

    def forward(self, *a, **k):  # pragma: no cover - never called
        raise RuntimeError("GumbelSoftmaxDropout runs inside the engine; call the top-level model")


class PriGumbelV1Model(FusionModel):
    """train_val.py:125-158 — ConcatModel(tau, epsilon); forward(frame_input, vedio_mask, title_input,
    text_mask): concat -> relu(fc1) -> fc2 -> Gumbel-softmax feature dropout x*m/(1-w) (soft in train
    mode, hard in eval, one draw per feature per forward) -> row min-max + Laplace(0, 1/eps) ->
    classifier."""

    def __init__(self, tau: float = 0.01, epsilon: float = 1.0, contract: str = "T", **kw):
        super().__init__("prigumbel_v1", contract=contract, eps=float(epsilon), tau=float(tau), **kw)
        self.epsilon = epsilon

    def forward(self, frame_input, vedio_mask, title_input, text_mask):
        self._engine.cfg.tau = float(self.dropout.tau)
        return self._run(self._token_batch(frame_input, vedio_mask, title_input, text_mask), not self.training)

    def forward_window(self, eeg, act, hard=None):
        self._engine.cfg.tau = float(self.dropout.tau)
        return super().forward_window(eeg, act, (not self.training) if hard is None else hard)


def load_bert_weights(model: FusionModel, path: str):
    """Load `bert.*` weights from a local safetensors file or HF directory (no network)."""
    from safetensors.torch import load_file
    f = path if path.endswith(".safetensors") else os.path.join(path, "model.safetensors")
    sd = load_file(f)
    sd = {("bert." + k if not k.startswith("bert.") else k): v for k, v in sd.items()}
    missing = model.load_state_dict({k: v for k, v in sd.items() if k in model.state_dict()}, strict=False)
    return missing
