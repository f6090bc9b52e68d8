"""Philox4x32-10 in numpy — test infrastructure only: replays the dropout masks the HIP kernels draw
(csrc/common.h philox4x32 / drop_mask4) so dropout sites are checked element-exactly.

Element e of a dropout site keyed (seed, offset) is kept iff word (e & 3) of
philox(counter = (e >> 2, offset), key = seed) >= float32(p) * 2^32; kept elements scale by 1/(1-p).
"""
import numpy as np

_M32 = np.uint64(0xFFFFFFFF)


def philox4x32(c0, c1, c2, c3, k0, k1, rounds=10):
    c = [np.asarray(x, dtype=np.uint64) & _M32 for x in (c0, c1, c2, c3)]
    c = list(np.broadcast_arrays(*c))
    k0, k1 = np.uint64(k0) & _M32, np.uint64(k1) & _M32
    for _ in range(rounds):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & _M32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _M32
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = (k0 + np.uint64(0x9E3779B9)) & _M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & _M32
    return c


def drop_mask(seed: int, offset: int, elems, p: float) -> np.ndarray:
    """scale-or-zero mask (float64) for the element indices `elems` (any shape)."""
    e = np.asarray(elems, dtype=np.uint64)
    e4 = e >> np.uint64(2)
    w = philox4x32(e4 & _M32, e4 >> np.uint64(32), offset & 0xFFFFFFFF, offset >> 32, seed & 0xFFFFFFFF, seed >> 32)
    word = (e & np.uint64(3)).astype(np.int64)
    r = np.choose(word, w)
    thr = np.uint64(min(float(np.float32(p) * np.float32(4294967296.0)), 4294967295.0))
    return np.where(r >= thr, 1.0 / (1.0 - np.float64(np.float32(p))), 0.0)


def _keep16(seed: int, offset: int, call, k, p: float) -> np.ndarray:
    """halfword k (0..7) of philox7(call, offset; seed) >= uint32(float32(p) * 65536): scale or zero."""
    c = np.asarray(call, dtype=np.uint64)
    w = philox4x32(c & _M32, c >> np.uint64(32), offset & 0xFFFFFFFF, offset >> 32, seed & 0xFFFFFFFF, seed >> 32,
                   rounds=7)
    k = np.asarray(k, dtype=np.int64)
    word = np.choose(k >> 1, w)
    half = (word >> (np.uint64(16) * (k & 1).astype(np.uint64))) & np.uint64(0xFFFF)
    thr = np.uint64(min(float(np.float32(p) * np.float32(65536.0)), 65535.0))
    return np.where(half >= thr, 1.0 / (1.0 - np.float64(np.float32(p))), 0.0)


def attn_mask(seed: int, offset: int, elems, p: float) -> np.ndarray:
    """The Philox-7 16-bit stream of the LayerNorm-fused dropout sites (common.h keep_bits8): eight
    16-bit draws per call; element e kept iff halfword (e & 7) of philox7(e >> 3, offset; seed) >=
    uint32(float32(p) * 65536)."""
    e = np.asarray(elems, dtype=np.uint64)
    return _keep16(seed, offset, e >> np.uint64(3), (e & np.uint64(7)).astype(np.int64), p)


def attn_probs_mask(seed: int, offset: int, elems, p: float, L: int) -> np.ndarray:
    """Attention-probability dropout (csrc/attention.hip attn_call): element e = row * L + key of the
    [B, H, L, L] probabilities (row = (b * H + h) * L + q), key = 32 c + 16 j + 4 u + r, is kept iff
    halfword 4 j + r of philox7(row * 4 * ceil(L / 32) + 4 c + u, offset; seed) >= uint32(float32(p) * 65536)."""
    e = np.asarray(elems, dtype=np.uint64)
    row, key = e // np.uint64(L), e % np.uint64(L)
    c, j, u, r = key >> np.uint64(5), (key >> np.uint64(4)) & np.uint64(1), (key >> np.uint64(2)) & np.uint64(3), \
        key & np.uint64(3)
    call = row * np.uint64(4 * ((L + 31) // 32)) + np.uint64(4) * c + u
    return _keep16(seed, offset, call, (np.uint64(4) * j + r).astype(np.int64), p)
