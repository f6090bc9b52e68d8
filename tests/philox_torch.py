"""Philox4x32 on torch int64 tensors (any device) — test infrastructure only: the device form of
tests/philox_ref.py, for replaying the HIP path's dropout masks at full size (B = 256: 2.4 G
attention-probability draws per step, beyond numpy).  Same streams, same keep rules; pinned against
philox_ref by tests/test_philox_cpu.py."""
import torch

_M32 = 0xFFFFFFFF


def philox4x32(c0, c1, c2, c3, k0: int, k1: int, rounds: int = 10):
    """c0..c3: int64 tensors (or ints) holding uint32 values; returns four int64 tensors.  int64
    products of two uint32 values wrap exactly like the uint64 product, so (p >> 32) & M32 and
    p & M32 are its high and low words."""
    ref = next(x for x in (c0, c1, c2, c3) if torch.is_tensor(x))
    c = [x if torch.is_tensor(x) else torch.full_like(ref, int(x)) for x in (c0, c1, c2, c3)]
    c = [x & _M32 for x in c]
    k0, k1 = int(k0) & _M32, int(k1) & _M32
    for _ in range(rounds):
        p0 = c[0] * 0xD2511F53
        p1 = c[2] * 0xCD9E8D57
        hi0, lo0 = (p0 >> 32) & _M32, p0 & _M32
        hi1, lo1 = (p1 >> 32) & _M32, p1 & _M32
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = (k0 + 0x9E3779B9) & _M32
        k1 = (k1 + 0xBB67AE85) & _M32
    return c


def _scale(p: float) -> float:
    import numpy as np
    return float(1.0 / (1.0 - np.float64(np.float32(p))))


def drop_mask(seed: int, offset: int, e: torch.Tensor, p: float) -> torch.Tensor:
    """philox_ref.drop_mask: element e kept iff word (e & 3) of philox10(e >> 2, offset; seed) >=
    float32(p) 2^32; float32 scale-or-zero mask."""
    import numpy as np
    e4 = e >> 2
    w = philox4x32(e4 & _M32, e4 >> 32, offset & _M32, offset >> 32, seed & _M32, seed >> 32)
    word = e & 3
    r = torch.where(word == 0, w[0], torch.where(word == 1, w[1], torch.where(word == 2, w[2], w[3])))
    thr = int(min(float(np.float32(p) * np.float32(4294967296.0)), 4294967295.0))
    return torch.where(r >= thr, _scale(p), 0.0).float()


def _keep16(seed: int, offset: int, call: torch.Tensor, k: torch.Tensor, p: float) -> torch.Tensor:
    import numpy as np
    w = philox4x32(call & _M32, call >> 32, offset & _M32, offset >> 32, seed & _M32, seed >> 32, rounds=7)
    wi = k >> 1
    word = torch.where(wi == 0, w[0], torch.where(wi == 1, w[1], torch.where(wi == 2, w[2], w[3])))
    half = (word >> (16 * (k & 1))) & 0xFFFF
    thr = int(min(float(np.float32(p) * np.float32(65536.0)), 65535.0))
    return torch.where(half >= thr, _scale(p), 0.0).float()


def attn_mask(seed: int, offset: int, e: torch.Tensor, p: float) -> torch.Tensor:
    """philox_ref.attn_mask (the LayerNorm-fused sites' Philox-7 16-bit stream)."""
    return _keep16(seed, offset, e >> 3, e & 7, p)


def attn_probs_mask(seed: int, offset: int, e: torch.Tensor, p: float, L: int) -> torch.Tensor:
    """philox_ref.attn_probs_mask (attention-probability dropout, attention.hip attn_call)."""
    row, key = e // L, e % L
    c, j, u, r = key >> 5, (key >> 4) & 1, (key >> 2) & 3, key & 3
    call = row * (4 * ((L + 31) // 32)) + 4 * c + u
    return _keep16(seed, offset, call, 4 * j + r, p)
