"""DP-SGD on the engine: the drop-in for opacus's
`PrivacyEngine.make_private_with_epsilon` as main_0430.py:143-162 (PriConcat pretrain: trainable
bert.encoder.layer[-1], fc_layers, classifier; max_grad_norm = args.MAX_GRAD_NORM) and
base_train.py:322-348 (TICA DPSGD baseline, max_grad_norm 0.1) call it.

opacus semantics restated (opacus is absent; no version is pinned by the reference):
  * data: Poisson sampling — every step draws each training sample independently with probability
    q = 1 / len(data_loader), len(data_loader) steps per epoch (DPDataLoader /
    UniformWithReplacementSampler); empty batches are legal;
  * per-sample gradients of the per-sample loss: with loss_reduction="mean" the backward's
    output gradient is multiplied by the batch size n (GradSampleModule);
  * per-sample norm over ALL trainable parameters, clip factor c_b = min(1, C / (norm_b + 1e-6)),
    summed_grad = sum_b c_b grad_b (DPOptimizer.clip_and_accumulate);
  * p.grad = (summed_grad + N(0, (sigma C)^2)) / expected_batch_size, expected_batch_size =
    int(len(dataset) * q) (add_noise, scale_grad); then the wrapped optimizer's step;
  * noise multiplier sigma from the accountant's search (eegfusion.privacy; RDP accountant);
  * the returned module is a GradSampleModule-style wrapper, so its state_dict keys carry the
    `_module.` prefix exactly as opacus's do (main_0430.py:218 saves them that way, and the finetune's
    load_state_dict(strict=False) at :139 then matches none of them — a reference quirk kept as is).
How (MI355X): per-sample gradients are never formed.  The backward runs twice over the trainable
region: a norm pass in which every gradient site adds its per-sample squared norms
(FusionEngine.psn: ghost norms on the MFMA for the BERT layer's token-sequence Linears, per-sample
column sums for biases / LayerNorm, row norms for the head), then — since each per-sample gradient
is linear in that sample's logit gradient — an ordinary backward with the logit-gradient rows
scaled by c_b (eegf_dp_clip_rows) accumulates exactly sum_b c_b grad_b.  eegf_dp_noise adds the
Gaussian noise and the 1/expected-batch scale in one pass per parameter.
"""
from __future__ import annotations

import logging
import math

import torch
import torch.nn as nn
from torch.utils.data import DataLoader, Sampler

from . import _lib
from ._lib import call
from .privacy import create_accountant, get_noise_multiplier

log = logging.getLogger(__name__)

_UNSUPPORTED = ("multi_head_decoder.", "multi_head_decoderlayer.", "bert.embeddings.", "eeg_encoder.", "DP")


def _s():
    return torch.cuda.current_stream().cuda_stream


# ----------------------------------------------------------------------------- data: Poisson
class UniformWithReplacementSampler(Sampler):
    """opacus UniformWithReplacementSampler: each of `steps` batches takes every index independently
    with probability sample_rate."""

    def __init__(self, *, num_samples: int, sample_rate: float, generator=None, steps: int | None = None):
        if num_samples <= 0 or not (0 < sample_rate <= 1):
            raise ValueError("invalid Poisson sampler parameters")
        self.num_samples, self.sample_rate, self.generator = num_samples, sample_rate, generator
        self.steps = int(1 / sample_rate) if steps is None else steps

    def __len__(self):
        return self.steps

    def __iter__(self):
        for _ in range(self.steps):
            mask = torch.rand(self.num_samples, generator=self.generator) < self.sample_rate
            yield mask.nonzero(as_tuple=False).reshape(-1).tolist()


def _collate_with_empty(collate_fn, sample_shapes):
    def fn(batch):
        if len(batch) > 0:
            return collate_fn(batch)
        return [torch.zeros((0, *shape), dtype=dt) for shape, dt in sample_shapes]
    return fn


class DPDataLoader(DataLoader):
    """opacus DPDataLoader.from_data_loader: same dataset / collate, Poisson batch sampler."""

    @classmethod
    def from_data_loader(cls, data_loader: DataLoader, generator=None):
        ds = data_loader.dataset
        sample_rate = 1 / len(data_loader)
        first = ds[0]
        shapes = [(tuple(torch.as_tensor(x).shape), torch.as_tensor(x).dtype) for x in first]
        from torch.utils.data.dataloader import default_collate
        collate = data_loader.collate_fn or default_collate
        return cls(ds, batch_sampler=UniformWithReplacementSampler(num_samples=len(ds), sample_rate=sample_rate,
                                                                   generator=generator),
                   collate_fn=_collate_with_empty(collate, shapes), num_workers=data_loader.num_workers,
                   pin_memory=data_loader.pin_memory)

    @property
    def sample_rate(self):
        return self.batch_sampler.sample_rate


# --------------------------------------------------------------------------- module wrapper
class GradSampleModule(nn.Module):
    """opacus GradSampleModule stand-in: forwards to the wrapped FusionModel (attribute `_module`,
    so state_dict keys read `_module.*` as opacus's do) whose backward now runs the private
    two-pass schedule (FusionModel._backward -> private_backward)."""

    def __init__(self, m, max_grad_norm: float, loss_reduction: str = "mean"):
        super().__init__()
        self._module = m
        m._dp = dict(max_grad_norm=float(max_grad_norm), loss_reduction=loss_reduction, last_norms=None,
                     last_clip=None)
        # per-sample norms index the BERT gradient sites by B x L rows: keep contract T padded
        m.engine.cfg.varlen = False

    def forward(self, *a, **k):
        return self._module(*a, **k)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self._module, name)


def private_backward(model, saved, dlogits, need: set[str]):
    """The DP-SGD backward of one batch: per-sample norms (pass A), clip factors, clipped sum
    (pass B) into the arena gradients of `need` (overwritten)."""
    bad = sorted(n for n in need if n.startswith(_UNSUPPORTED))
    if bad:
        raise NotImplementedError(f"eegfusion DP-SGD: per-sample norms of {bad[:3]} are not implemented "
                                  "(the reference trains the last BERT layer, pooler, visual encoder and head)")
    dp = model._dp
    eng = model.engine
    B = dlogits.shape[0]
    dl = dlogits.float().contiguous().clone()
    if dp["loss_reduction"] == "mean":
        dl.mul_(B)                                   # GradSampleModule: backprops * n
    psn = torch.zeros(B, dtype=torch.float32, device=dl.device)
    clip = torch.empty(B, dtype=torch.float32, device=dl.device)
    eng.needs_grad = need
    eng.psn = {"out": psn, "B": B, "T": saved.L}
    try:
        eng.backward(saved, dl)
    finally:
        eng.psn = None
    call("eegf_dp_clip_rows", B, dl.shape[1], psn.data_ptr(), dp["max_grad_norm"], dl.data_ptr(), clip.data_ptr(),
         _s())
    for n in need:
        eng.G(n).zero_()
    eng.backward(saved, dl)
    eng.needs_grad = None
    dp["last_norms"], dp["last_clip"] = psn, clip


def _draw_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (), dtype=torch.int64).item())


class DPOptimizer:
    """opacus DPOptimizer over the wrapped optimizer: step() = add N(0, (sigma C)^2) noise to every
    trainable parameter's (clipped-sum) gradient and divide by the expected batch size, count one
    accountant step, then the original step."""

    def __init__(self, optimizer, *, noise_multiplier: float, max_grad_norm: float, expected_batch_size: int,
                 seed: int | None = None, on_step=None):
        self.original_optimizer = optimizer
        self.noise_multiplier, self.max_grad_norm = float(noise_multiplier), float(max_grad_norm)
        self.expected_batch_size = int(expected_batch_size)
        # opacus draws its noise from torch's advancing generator: take the Philox key from the global
        # torch RNG (so set_seed(...) decides it and two optimizers in one process differ); a fixed
        # seed is an explicit test option
        self.seed = _draw_seed() if seed is None else int(seed)
        self.steps, self.on_step = 0, on_step

    @property
    def param_groups(self):
        return self.original_optimizer.param_groups

    @property
    def state(self):
        return self.original_optimizer.state

    def zero_grad(self, set_to_none: bool = True):
        self.original_optimizer.zero_grad(set_to_none=set_to_none)

    def add_noise_and_scale(self):
        std = self.noise_multiplier * self.max_grad_norm
        k = 0
        for group in self.param_groups:
            for p in group["params"]:
                if not p.requires_grad:
                    continue
                if p.grad is None:           # no sample this step (empty Poisson batch): noise only
                    p.grad = torch.zeros_like(p)
                call("eegf_dp_noise", p.numel(), p.grad.data_ptr(), std, 1.0 / self.expected_batch_size, self.seed,
                     (self.steps << 20) + k, _s())
                k += 1

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.add_noise_and_scale()
        self.steps += 1
        if self.on_step is not None:
            self.on_step()
        self.original_optimizer.step()
        return loss

    def state_dict(self):
        return self.original_optimizer.state_dict()

    def load_state_dict(self, sd):
        self.original_optimizer.load_state_dict(sd)


class PrivacyEngine:
    """opacus PrivacyEngine stand-in (make_private / make_private_with_epsilon / get_epsilon)."""

    def __init__(self, *, accountant: str = "rdp", secure_mode: bool = False, seed: int | None = None):
        if secure_mode:
            raise NotImplementedError("secure_mode (cryptographic RNG) is not provided")
        self.accountant = create_accountant(accountant)
        self.seed = seed

    def make_private(self, *, module, optimizer, data_loader, noise_multiplier: float, max_grad_norm: float,
                     poisson_sampling: bool = True, loss_reduction: str = "mean", **_):
        dl = DPDataLoader.from_data_loader(data_loader) if poisson_sampling else data_loader
        sample_rate = 1 / len(data_loader)
        expected = int(len(data_loader.dataset) * sample_rate)
        wrapped = module if isinstance(module, GradSampleModule) else GradSampleModule(module, max_grad_norm,
                                                                                       loss_reduction)
        opt = DPOptimizer(optimizer, noise_multiplier=noise_multiplier, max_grad_norm=max_grad_norm,
                          expected_batch_size=expected, seed=self.seed,
                          on_step=lambda: self.accountant.step(noise_multiplier=noise_multiplier,
                                                               sample_rate=sample_rate))
        return wrapped, opt, dl

    def make_private_with_epsilon(self, *, module, optimizer, data_loader, target_epsilon: float,
                                  target_delta: float, epochs: int, max_grad_norm: float,
                                  epsilon_tolerance: float = 0.01, **kw):
        sample_rate = 1 / len(data_loader)
        sigma = get_noise_multiplier(target_epsilon=target_epsilon, target_delta=target_delta, sample_rate=sample_rate,
                                     epochs=epochs, accountant=self.accountant.mechanism(),
                                     epsilon_tolerance=epsilon_tolerance)
        # opacus >= 1.3 defaults to the PRV accountant; this build implements RDP only, so sigma can
        # differ from such a run: say which one chose it
        log.info("make_private_with_epsilon: noise_multiplier %.6f from the %s accountant (target eps %g, delta %g, "
                 "sample rate %g, %d epochs)", sigma, self.accountant.mechanism(), target_epsilon, target_delta,
                 sample_rate, epochs)
        self.last_noise_multiplier = sigma
        return self.make_private(module=module, optimizer=optimizer, data_loader=data_loader, noise_multiplier=sigma,
                                 max_grad_norm=max_grad_norm, **kw)

    def get_epsilon(self, delta: float) -> float:
        return self.accountant.get_epsilon(delta=delta)
