"""Drop-in `Adam` for the reference harnesses' `torch.optim.Adam(model.parameters(), lr=...)`
(main_0430.py:132, past_acc.py:159-160, train.py:77, base_train.py:170-171): the same update
(Kingma & Ba with bias correction, torch's eps placement and L2 weight decay) as one eegf_adam
launch per parameter with a gradient (parameters whose .grad is None are skipped, as torch does).
Parameters that are views into a ParamArena have their bf16 compute shadow refreshed before the
next forward.  The trainers (eegfusion/trainer.py FlatAdam) step whole arena ranges instead."""
from __future__ import annotations

import torch

from ._lib import call
from .arena import ParamArena


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid Adam hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.grad.dtype == torch.float32
                        and p.is_contiguous() and p.grad.is_contiguous()):
                    raise RuntimeError("eegfusion Adam: fp32 contiguous device parameters and gradients only")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                call("eegf_adam", p.numel(), p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                     st["exp_avg_sq"].data_ptr(), None, float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                     float(group["weight_decay"]), 1.0, st["step"], torch.cuda.current_stream().cuda_stream)
                a = ParamArena.owner(p)
                if a is not None:
                    a.invalidate_shadow()
        return loss
