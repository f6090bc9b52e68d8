"""Shared helpers for golden fixtures (tests only)."""
from __future__ import annotations

import functools
import json
from pathlib import Path

import numpy as np
import torch

from oracle import fusion_oracle as O
from oracle.detweights import det_tensor, sample_positions

GOLDEN = Path(__file__).resolve().parent / "golden"
SEED = 20240501


def load(name: str):
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    cfg = json.loads(str(z["config"]))
    return cfg, {k: z[k] for k in z.files if k != "config"}


@functools.lru_cache(maxsize=8)
def _det_params_np(contract: str, variant: str, seed: int = SEED, modal: str = "ti"):
    shapes = O.param_shapes(contract, variant, modal=modal)
    return {k: det_tensor(seed, k, s) for k, s in shapes.items() if k != "DP"}


def det_params(contract: str, variant: str, dp=None, requires_grad=True, modal: str = "ti") -> dict[str, torch.Tensor]:
    p = {k: torch.from_numpy(v.copy()) for k, v in _det_params_np(contract, variant, modal=modal).items()}
    if "DP" in O.param_shapes(contract, variant, modal=modal):
        p["DP"] = torch.as_tensor(dp if dp is not None else np.zeros((1, O.FUSED), np.float32)).float().clone()
    for t in p.values():
        t.requires_grad_(requires_grad)
    return p


def w_values_dp():
    """logit of the reference's learned gate values w_values.txt (fixture copy of that data file)."""
    return np.load(GOLDEN / "w_values_dp.npz", allow_pickle=False)["DP"]


def rel_err(a, b) -> float:
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def delta_bound(before, tol: float, lr: float):
    """Element-wise bound for |delta/lr - ref| of an fp32 parameter update delta = after - before:
    max(tol, 2 ulp(|p|) / lr).  Both sides of the comparison are differences of fp32 parameters, so
    each is quantised to ulp(p) (at lr 1e-6 one ulp of a parameter in [1/32, 1/16) is 3.7e-3 of
    delta/lr) — a rounding artefact, not a parity difference."""
    b = np.abs(np.asarray(before, dtype=np.float32))
    return np.maximum(tol, 2.0 * np.spacing(b).astype(np.float64) / lr)


def check_grads(grads: dict, fx: dict, tol: float, skip=()):
    """Compare a {name: grad tensor|None} dict with a fixture's grad records.
    Each recorded quantity must agree to `tol` relative to its own max magnitude."""
    bad = []
    names = {k.split(":", 1)[1] for k in fx if k.startswith(("gsum:", "gnone:"))}
    for n in sorted(names):
        if n in skip:
            continue
        g = grads.get(n)
        if f"gnone:{n}" in fx:
            if g is not None and float(g.abs().max()) != 0.0:
                bad.append((n, "expected no grad"))
            continue
        if g is None:
            bad.append((n, "missing grad"))
            continue
        g = g.detach().double().reshape(-1).cpu().numpy()
        gabs = float(fx[f"gabs:{n}"])
        ref = fx[f"gfull:{n}"] if f"gfull:{n}" in fx else fx[f"gval:{n}"]
        if gabs / g.size < 1e-9 and np.abs(ref).max() < 1e-7:
            # mathematically-zero gradient (softmax shift invariance: attention key biases; the
            # decoder's single-key self-attention q/k): reference holds fp residue only.
            if np.abs(g).max() > 1e-6:
                bad.append((n, "expected ~0", np.abs(g).max()))
            continue
        if abs(g.sum() - float(fx[f"gsum:{n}"])) > tol * max(gabs, 1e-30):
            bad.append((n, "sum", g.sum(), float(fx[f"gsum:{n}"]), gabs))
        if f"gfull:{n}" in fx:
            e = rel_err(g, fx[f"gfull:{n}"])
        else:
            e = rel_err(g[fx[f"gpos:{n}"]], fx[f"gval:{n}"]) if np.abs(fx[f"gval:{n}"]).max() > 0 else 0.0
        if e > tol:
            bad.append((n, "values", e))
    assert not bad, bad[:10]


def modal_case(fx: dict, modal: str) -> dict:
    """the arrays of one variant of tests/golden/modal_variants.npz (keys '<modal>:<name>')"""
    pre = modal + ":"
    return {k[len(pre):]: v for k, v in fx.items() if k.startswith(pre)}
