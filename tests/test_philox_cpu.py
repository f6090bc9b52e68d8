"""Philox4x32 restatement (tests/philox_ref.py, which mirrors csrc/common.h) against the Random123
known-answer vectors (kat_vectors: philox4x32_10), and the dropout-stream conventions."""
import numpy as np

from philox_ref import attn_mask, drop_mask, philox4x32

KAT = [  # (counter, key, expected) — Random123 philox4x32_10 KAT
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox4x32_10_known_answers():
    for ctr, key, want in KAT:
        got = tuple(int(w) for w in philox4x32(*ctr, *key))
        assert got == want, (ctr, [hex(x) for x in got])


def test_dropout_streams_rates():
    e = np.arange(1 << 18)
    for p in (0.1, 0.25):
        for fn in (drop_mask, attn_mask):
            m = fn(7, 3, e, p)
            assert abs((m > 0).mean() - (1 - p)) < 0.005
            assert np.allclose(m[m > 0], 1 / (1 - np.float32(p)))
    # distinct offsets give independent masks
    a, b = drop_mask(7, 3, e, 0.5) > 0, drop_mask(7, 4, e, 0.5) > 0
    assert abs((a == b).mean() - 0.5) < 0.01


def test_attn_probs_numbering_is_a_bijection():
    """attention.hip attn_call: (row, key) -> (call, halfword) is one-to-one for any L (L % 32 != 0
    leaves draws unused), and the kept fraction is 1 - p."""
    import numpy as np
    from philox_ref import attn_probs_mask
    for L in (256, 65):
        rows = 3 * L
        key = np.arange(L, dtype=np.int64)
        c, j, u, r = key >> 5, (key >> 4) & 1, (key >> 2) & 3, key & 3
        call = np.arange(rows, dtype=np.int64)[:, None] * (4 * ((L + 31) // 32)) + 4 * c + u
        draw = call * 8 + 4 * j + r
        assert np.unique(draw).size == rows * L
    m = attn_probs_mask(7, 3, np.arange(64 * 256 * 256, dtype=np.uint64), 0.1, 256)
    assert abs((m > 0).mean() - 0.9) < 2e-3


def test_torch_philox_matches_numpy_replay():
    """tests/philox_torch.py (the device form used at full size) draws exactly philox_ref's masks:
    the known answers, and every dropout stream on 2^16 elements at offsets past 2^32."""
    import torch
    import philox_torch as PT
    from philox_ref import attn_probs_mask
    for ctr, key, want in KAT:
        got = tuple(int(w) for w in PT.philox4x32(*(torch.tensor([c]) for c in ctr), *key))
        assert got == want
    e = np.arange(1 << 16, dtype=np.uint64) + np.uint64(12345)
    et = torch.from_numpy(e.astype(np.int64))
    for seed, off in ((980616, 7), (3, (5 << 32) + 11)):
        assert np.array_equal(PT.drop_mask(seed, off, et, 0.1).numpy(), drop_mask(seed, off, e, 0.1).astype(np.float32))
        assert np.array_equal(PT.attn_mask(seed, off, et, 0.1).numpy(), attn_mask(seed, off, e, 0.1).astype(np.float32))
        assert np.array_equal(PT.attn_probs_mask(seed, off, et, 0.1, 256).numpy(),
                              attn_probs_mask(seed, off, e, 0.1, 256).astype(np.float32))
