"""Closed-form deterministic parameters for parity tests (TEST INFRASTRUCTURE ONLY).

Pretrained `bert-base-uncased` / CLIP weights are not available offline, so every
parity fixture is generated with parameters that are a pure function of (seed, parameter name,
element index): value = centre + half_width * (2u - 1), u = splitmix64(hash) / 2^64.
The golden generator (tests/golden/make_golden.py, run against the reference in the survey
container) and the tests (against the oracle and the HIP path) regenerate identical tensors, so
the fixtures stay small.
"""
from __future__ import annotations

import hashlib

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _name_key(seed: int, name: str) -> np.uint64:
    h = hashlib.blake2b(f"{seed}:{name}".encode(), digest_size=8).digest()
    return np.uint64(int.from_bytes(h, "little"))


def uniform01(seed: int, name: str, n: int) -> np.ndarray:
    """n float64 values in [0,1) determined by (seed, name)."""
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = _splitmix64(idx * np.uint64(0x632BE59BD9B4E019) + _name_key(seed, name))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def init_rule(name: str, shape: tuple[int, ...]) -> tuple[float, float]:
    """(centre, half_width) for a parameter, by its role (name suffix / rank)."""
    if "LayerNorm" in name or ".norm" in name:
        return (1.0, 0.1) if name.endswith("weight") else (0.0, 0.05)
    if name.endswith("bias"):
        return 0.0, 0.02
    if len(shape) >= 2:
        return 0.0, 1.0 / np.sqrt(shape[-1])
    return 0.0, 0.05


def det_tensor(seed: int, name: str, shape: tuple[int, ...]) -> np.ndarray:
    c, hw = init_rule(name, shape)
    n = int(np.prod(shape)) if len(shape) else 1
    u = uniform01(seed, name, n)
    return (c + hw * (2.0 * u - 1.0)).astype(np.float32).reshape(shape)


def det_state_dict(seed: int, shapes: dict[str, tuple[int, ...]], skip=("DP",)) -> dict[str, np.ndarray]:
    return {k: det_tensor(seed, k, tuple(s)) for k, s in shapes.items() if k not in skip}


def sample_positions(name: str, numel: int, k: int = 16) -> np.ndarray:
    """Fixed element positions at which fixtures record large gradients."""
    u = uniform01(12345, "pos:" + name, k)
    return np.unique((u * numel).astype(np.int64))
