"""PriGumbel / PriConcat training iterations on the engine (no autograd on the hot path).

`PriGumbelTrainer.step` restates one batch of past_acc.main2's loop (past_acc.py:194-212) and of
TrainAndTest.train's 'lapacian_dropout' branch (base_train.py:167-210):

  1. DP_optimizer.zero_grad(); fwd(hard=False); CE(mean); backward; DP_optimizer.step()
  2. model_optimizer.zero_grad(); fwd(hard=True); CE(mean); backward; model_optimizer.step()

Only the DP gradient of pass 1 is ever used (model_optimizer.zero_grad() discards the rest), so
pass 1 runs the encoders forward without saving activations and backpropagates only through the
head and the privacy stage; pass 2's DP gradient is likewise dead (DP_optimizer.zero_grad()
clears it before its next use) and is not computed.  Parameter values after the step are
identical to the reference loop.  With world_size > 1 the gradients are averaged over ranks with
RCCL all-reduce on arena grad ranges before each Adam; pass 2's all-reduces start during the
backward, one BERT layer at a time (GradReducer).

consume_grads (default True): each Adam step zeroes the gradient range it read (eegf_adam_consume) and
the next zero_grad() skips its fill pass, so after step() the arena gradients read as zero instead of
holding the last step's values until the next zero_grad (the reference order); pass False to inspect
gradients after a step.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib
from ._lib import call
from .engine import FusionEngine


def _s():
    return torch.cuda.current_stream().cuda_stream


class FlatAdam:
    """torch.optim.Adam over one contiguous arena range, one fused launch per step (eegf_adam)."""

    def __init__(self, engine: FusionEngine, rng: tuple[int, int], lr=1e-6, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, write_shadow=True, names=None, consume=True):
        self.e = engine
        self.lo, self.hi = rng
        # names: the group's parameters that take part in the graph.  torch.optim.Adam skips a
        # parameter whose .grad is None (never touching its state), so only their coalesced
        # sub-ranges are stepped: the unused template decoder layer and the contract-W word
        # embeddings (31 M elements) are not streamed through Adam.
        self.sub = [(max(lo, self.lo), min(hi, self.hi)) for lo, hi in engine.a.ranges(names)
                    if lo < self.hi and hi > self.lo] if names is not None else [(self.lo, self.hi)]
        a = engine.a
        n = self.hi - self.lo
        self.m = torch.zeros(n, dtype=torch.float32, device=a.device)
        self.v = torch.zeros(n, dtype=torch.float32, device=a.device)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.t = 0
        self.write_shadow = write_shadow
        # consume: the step zeroes the gradient it read (eegf_adam_consume), so the next zero_grad() has
        # nothing to clear.  The gradient range is then zero outside the backward that fills it; the
        # trainers are its only writers (the sub-ranges Adam skips are never written at all).
        self.consume = consume and _lib.has("eegf_adam_consume")   # (absent only in an older A/B build)
        self._clean = False

    def zero_grad(self):
        if not self._clean:
            self.e.a.grad[self.lo:self.hi].zero_()
        self._clean = False

    def step(self, grad_scale: float = 1.0):
        """grad_scale multiplies the gradient as Adam reads it (1/N over an all-reduced sum)."""
        a = self.e.a
        self.t += 1
        sh = None
        if self.write_shadow and self.e.dt == torch.bfloat16:
            self.e._refresh_shadow()
            sh = a.shadow[self.lo:self.hi].data_ptr()
        for lo, hi in self.sub:
            o = lo - self.lo
            ev = self.e._ev_start("adam")
            call("eegf_adam_consume" if self.consume else "eegf_adam", hi - lo, a.master[lo:].data_ptr(), a.grad[lo:].data_ptr(), self.m[o:].data_ptr(),
                 self.v[o:].data_ptr(), None if sh is None else a.shadow[lo:].data_ptr(), float(self.lr),
                 float(self.betas[0]), float(self.betas[1]), float(self.eps), float(self.wd), float(grad_scale),
                 self.t, _s())
            # master, gradient, m, v in; master, m, v (+ the zeroed gradient, + the bf16 shadow) out
            self.e._ev_end("adam", ev, 0.0, (hi - lo) * (28 + (4 if self.consume else 0) + (2 if sh is not None else 0)))
        if self.consume:
            # every written element of [lo, hi) lies in a stepped sub-range (the graph parameters' ranges)
            self._clean = True


class GradReducer:
    """Average gradients over ranks: RCCL all_reduce(SUM) of arena grad ranges, then scale by 1/N.

    Two uses:
      * `reducer(g)`: one contiguous range, reduced now in buckets (the 9 KB DP gradient of pass 1);
      * `begin(arena, names)` / `ready(names)` / `finish(lo, hi)` around a backward: the engine calls
        `ready` (FusionEngine.grad_ready) as soon as a group of weight gradients is final in stream
        order — the decoder/head/pooler matrices before the BERT backward starts, then each BERT
        layer's contiguous six-matrix block (~28 MB) right after that layer — and each group's
        all_reduce is issued at once (async_op) so RCCL runs it on its own stream while the
        remaining layers' backward kernels run; `finish` reduces what is left (biases, LayerNorm,
        embeddings: their column sums are deferred to the end of the backward), makes the compute
        stream wait for every outstanding collective, and scales the range by 1/N — or, with
        scale_in_optimizer=True, leaves the SUM in place and the trainers pass `grad_scale` = 1/N to
        the fused Adam, which applies it as it reads the gradient (no extra pass over the ~0.47 GB
        gradient arena per step; bitwise the same update).
    Only parameters in `names` are reduced: the unused decoder template layer and (contract W) the
    word embeddings (31 M of 148 M elements) never enter a bucket.  The issue order is the same on
    every rank (same backward sequence), as RCCL requires.  With world_size 1 nothing is launched,
    but the ranges are still recorded (`self.log`), so a single-GPU test can check coverage.
    """

    def __init__(self, bucket_elems: int = 32 << 20, scale_in_optimizer: bool = False, coalesce_elems: int = 1 << 20,
                 merge_elems: int = 0):
        self.bucket = int(bucket_elems)
        # ranges shorter than this, issued together, are gathered into one staging buffer and reduced by
        # one collective (the 37 bias / LayerNorm / embedding ranges of the BERT step at finish(), the
        # 23 decoder / head matrices before the encoder backward): one RCCL launch instead of dozens of
        # latency-bound small ones; 0 disables.  At most half a bucket, so two always share one.
        self.coalesce = min(int(coalesce_elems), self.bucket // 2)
        # ready() ranges are held until they add up to merge_elems, then issued together (adjacent
        # ranges merged: consecutive BERT layers' blocks are adjacent in the arena, so a bucket of k
        # layers is one collective); 0 (default) issues every ready() group at once
        self.merge = int(merge_elems)
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.scale_in_optimizer = bool(scale_in_optimizer)
        self.works, self.todo, self.log, self.staged, self.pending = [], set(), [], [], []
        self.n_coalesced = 0            # staged collectives issued since begin()
        self.arena = None

    def __call__(self, g: torch.Tensor):
        if self.world == 1:
            return
        for i in range(0, g.numel(), self.bucket):
            dist.all_reduce(g[i: i + self.bucket], op=dist.ReduceOp.SUM)
        if not self.scale_in_optimizer:
            g.mul_(1.0 / self.world)

    @property
    def grad_scale(self) -> float:
        """the factor Adam must apply to the reduced gradients (1/N when the reducer leaves sums)"""
        return 1.0 / self.world if self.scale_in_optimizer else 1.0

    @staticmethod
    def ranges(arena, names) -> list[tuple[int, int]]:
        return arena.ranges(names)

    def begin(self, arena, names):
        self.arena, self.todo, self.works, self.log, self.staged, self.pending = arena, set(names), [], [], [], []
        self.n_coalesced = 0

    def ready(self, names):
        names = [n for n in names if n in self.todo]
        if not names:
            return
        self.todo.difference_update(names)
        rngs = self.ranges(self.arena, names)
        if self.merge <= 0:
            self._launch(rngs)
            return
        self.pending += rngs
        if sum(hi - lo for lo, hi in self.pending) >= self.merge:
            self._flush()

    def _flush(self):
        if self.pending:
            rngs, self.pending = _merge_adjacent(self.pending), []
            self._launch(rngs)

    def plan(self, rngs) -> list[list[tuple[int, int]]]:
        """The collectives for these ranges, in issue order: each entry is a list of ranges reduced by one
        collective.  Runs of small ranges (< coalesce elements) are gathered into groups of at most one
        bucket (staged through one buffer); a small range that would sit alone is reduced on its own;
        every other range is cut into bucket-sized pieces."""
        rngs = list(rngs)
        small = [r for r in rngs if r[1] - r[0] < self.coalesce]
        groups, cur, n = [], [], 0
        for r in small:
            if cur and n + r[1] - r[0] > self.bucket:
                groups.append(cur)
                cur, n = [], 0
            cur.append(r)
            n += r[1] - r[0]
        if cur:
            groups.append(cur)
        out = [g for g in groups if len(g) > 1]
        alone = {g[0] for g in groups if len(g) == 1}
        for lo, hi in rngs:
            if hi - lo < self.coalesce and (lo, hi) not in alone:
                continue
            out += [[(i, min(hi, i + self.bucket))] for i in range(lo, hi, self.bucket)]
        return out

    def _launch(self, rngs):
        for grp in self.plan(rngs):
            self.log.extend(grp)
            if len(grp) > 1:
                self.n_coalesced += 1
                self._issue_staged(grp)
            else:
                self._issue(*grp[0])

    def _issue(self, lo: int, hi: int):
        """one collective over the arena gradient range [lo, hi)"""
        if self.world > 1:
            self.works.append(dist.all_reduce(self.arena.grad[lo:hi], op=dist.ReduceOp.SUM, async_op=True))

    def _issue_staged(self, grp):
        """one collective over several ranges gathered into a staging buffer (copied back in finish)"""
        if self.world > 1:
            g = self.arena.grad
            buf = torch.cat([g[lo:hi] for lo, hi in grp])
            self.works.append(dist.all_reduce(buf, op=dist.ReduceOp.SUM, async_op=True))
            self.staged.append((grp, buf))

    def finish(self, lo: int, hi: int):
        self._flush()
        if self.todo:
            self._launch(self.ranges(self.arena, self.todo))
            self.todo = set()
        for w in self.works:
            w.wait()                    # compute stream waits for the RCCL stream (no host sync)
        self.works = []
        g = self.arena.grad if self.arena is not None else None
        for grp, buf in self.staged:    # staged small ranges back into the arena (one fused copy)
            torch._foreach_copy_([g[lo:hi] for lo, hi in grp], list(buf.split([hi - lo for lo, hi in grp])))
        self.staged = []
        if self.world > 1 and not self.scale_in_optimizer:
            self.arena.grad[lo:hi].mul_(1.0 / self.world)


def _merge_adjacent(rngs):
    """sorted ranges with touching neighbours joined (consecutive BERT layer blocks become one range)"""
    out = []
    for lo, hi in sorted(rngs):
        if out and lo <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], hi))
        else:
            out.append((lo, hi))
    return out


class PriGumbelTrainer:
    def __init__(self, engine: FusionEngine, lr: float = 1e-6, reducer: GradReducer | None = None,
                 consume_grads: bool = True):
        self.e = engine
        a = engine.a
        gp = engine.graph_params()
        self.model_params = {n for n in gp if n != "DP"}
        self.model_opt = FlatAdam(engine, a.model_range, lr=lr, names=self.model_params, consume=consume_grads)
        self.dp_opt = FlatAdam(engine, a.dp_range, lr=lr, write_shadow=False, consume=consume_grads)
        self.reduce = reducer or GradReducer()
        dev = a.device
        self.loss = torch.zeros(2, dtype=torch.float32, device=dev)
        self.correct = torch.zeros(2, dtype=torch.int32, device=dev)

    def _ce(self, logits, labels, i):
        B = logits.shape[0]
        dl = torch.empty_like(logits)
        ev = self.e._ev_start("cross_entropy")
        call("eegf_cross_entropy", _lib.F32 if logits.dtype == torch.float32 else _lib.BF16, B, 2, logits.data_ptr(), labels.data_ptr(), 0, 1.0,
             self.loss[i:].data_ptr(), self.correct[i:].data_ptr(), dl.data_ptr(), _s())
        # logits and int64 labels in, the logit gradients + loss / correct count out
        self.e._ev_end("cross_entropy", ev, 0.0, 2 * logits.numel() * logits.element_size() + B * 8 + 8)
        return dl

    def step(self, batch: dict, labels: torch.Tensor):
        e = self.e
        # ---- pass 1: DP parameters (hard=False)
        logits, sv = e.forward(batch, hard=False, training=True, save=False)
        dl = self._ce(logits, labels, 0)
        self.dp_opt.zero_grad()
        e.needs_grad = {"DP"}
        e.backward(sv, dl, head_only=True)
        self.reduce(e.a.grad[self.dp_opt.lo:self.dp_opt.hi])
        self.dp_opt.step(self.reduce.grad_scale)
        # ---- pass 2: model parameters (hard=True)
        logits, sv = e.forward(batch, hard=True, training=True, save=True)
        dl = self._ce(logits, labels, 1)
        self.model_opt.zero_grad()
        e.needs_grad = self.model_params
        self.reduce.begin(e.a, self.model_params)
        e.grad_ready = self.reduce.ready
        try:
            e.backward(sv, dl)
        finally:
            e.grad_ready = None
        e.needs_grad = None
        self.reduce.finish(self.model_opt.lo, self.model_opt.hi)
        self.model_opt.step(self.reduce.grad_scale)
        return self.loss, self.correct


class SinglePassTrainer:
    """PriConcat / ConcatModel step: one fwd(hard=True) + bwd + Adam over all graph params
    (main_0430.train finetune loop :177-187; train.py:94-113)."""

    def __init__(self, engine: FusionEngine, lr: float = 1e-6, reducer: GradReducer | None = None,
                 consume_grads: bool = True):
        self.e = engine
        self.params = engine.graph_params()
        self.opt = FlatAdam(engine, (0, engine.a.numel), lr=lr, names=self.params, consume=consume_grads)
        self.reduce = reducer or GradReducer()
        self.loss = torch.zeros(1, dtype=torch.float32, device=engine.a.device)
        self.correct = torch.zeros(1, dtype=torch.int32, device=engine.a.device)

    def step(self, batch, labels):
        e = self.e
        logits, sv = e.forward(batch, hard=True, training=True, save=True)
        dl = torch.empty_like(logits)
        call("eegf_cross_entropy", _lib.F32 if logits.dtype == torch.float32 else _lib.BF16, logits.shape[0], 2, logits.data_ptr(), labels.data_ptr(), 0, 1.0,
             self.loss.data_ptr(), self.correct.data_ptr(), dl.data_ptr(), _s())
        self.opt.zero_grad()
        e.needs_grad = self.params
        self.reduce.begin(e.a, self.params)
        e.grad_ready = self.reduce.ready
        try:
            e.backward(sv, dl)
        finally:
            e.grad_ready = None
        e.needs_grad = None
        self.reduce.finish(0, e.a.numel)
        self.opt.step(self.reduce.grad_scale)
        return self.loss, self.correct


class PriGumbelV1Trainer:
    """PriGumbel-v1 step (train_val.py:204-215): Adam over every parameter in the graph,
    loss = alpha * CE(mean) + max_j((1 - w_j) e^eps + w_j) (loss_function :80-93); the CE gradient
    scaled by alpha in the loss kernel, the privacy term's gradient added by eegf_v1_wloss."""

    def __init__(self, engine: FusionEngine, alpha: float, lr: float = 1e-5, reducer: GradReducer | None = None,
                 consume_grads: bool = True):
        self.e, self.alpha = engine, float(alpha)
        self.params = engine.graph_params()
        self.opt = FlatAdam(engine, (0, engine.a.numel), lr=lr, names=self.params, consume=consume_grads)
        self.reduce = reducer or GradReducer()
        dev = engine.a.device
        self.loss = torch.zeros(2, dtype=torch.float32, device=dev)     # [alpha * CE, privacy term]
        self.correct = torch.zeros(1, dtype=torch.int32, device=dev)

    def step(self, batch, labels, training: bool = True):
        e = self.e
        logits, sv = e.forward(batch, hard=not training, training=training, save=True)
        dl = torch.empty_like(logits)
        call("eegf_cross_entropy", _lib.F32, logits.shape[0], 2, logits.data_ptr(), labels.data_ptr(), 0, self.alpha,
             self.loss.data_ptr(), self.correct.data_ptr(), dl.data_ptr(), _s())
        self.opt.zero_grad()
        e.needs_grad = self.params
        self.reduce.begin(e.a, self.params)
        e.grad_ready = self.reduce.ready
        try:
            e.backward(sv, dl)
        finally:
            e.grad_ready = None
        e.v1_wloss(1.0, self.loss[1:])     # before finish(): w is all-reduced (sum / N) with the vectors
        e.needs_grad = None
        self.reduce.finish(0, e.a.numel)
        self.opt.step(self.reduce.grad_scale)
        self.loss[:1].mul_(self.alpha)
        return self.loss, self.correct
