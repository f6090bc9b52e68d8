"""feawei DP initialisation: known-answer checks of the oracle restatement of
past_acc.py:98-103 / past_acc_feawei.py:153-163.  The reference holds no feawei fixture (its
feawei.pkl is not shipped), so the hand-computed values below pin the formula."""
import math

import numpy as np
import torch

from oracle import fusion_oracle as O


def _sig(x):
    return 1.0 / (1.0 + math.exp(-x))


def test_feawei_raw_k5_known_answer():
    # 3 columns (one per modality block), 2 rows: column means [0.5, 1.0, 0.0]
    f = np.array([[0.0, 1.0, 0.0], [1.0, 1.0, 0.0]], np.float32)
    dp = O.feawei_dp_init(f, k=5.0, zscore=False)
    want = [0.4 + (1 - _sig(2.5)) - 0.5, 0.5 + (1 - _sig(5.0)) - 0.5, 0.3 + 0.5 - 0.5]
    assert dp.shape == (1, 3) and dp.dtype == torch.float32
    np.testing.assert_allclose(dp[0].numpy(), want, rtol=0, atol=1e-7)


def test_feawei_zscore_known_answer():
    # means [0, 1, 2] -> z = [-1.2247, 0, 1.2247] (population std sqrt(2/3))
    f = np.array([[0.0, 1.0, 2.0]], np.float32)
    dp = O.feawei_dp_init(f, k=1.0, zscore=True)
    z = 1.0 / math.sqrt(2.0 / 3.0)
    want = [0.4 + (1 - _sig(-z)) - 0.5, 0.5 + 0.5 - 0.5, 0.3 + (1 - _sig(z)) - 0.5]
    np.testing.assert_allclose(dp[0].numpy(), want, rtol=0, atol=1e-7)


def test_feawei_block_layout():
    # zero-spread features on 2304 columns, raw mode k=0: DP = base - 0 (w = 0.5)
    f = np.zeros((4, O.FUSED), np.float32)
    dp = O.feawei_dp_init(f, k=0.0, zscore=False)[0].numpy()
    np.testing.assert_allclose(dp[:768], 0.4, atol=1e-7)
    np.testing.assert_allclose(dp[768:1536], 0.5, atol=1e-7)
    np.testing.assert_allclose(dp[1536:], 0.3, atol=1e-7)
