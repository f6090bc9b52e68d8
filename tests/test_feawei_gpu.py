"""feawei DP initialisation on the device (eegf_colsum running sums + eegf_feawei_init) against the
oracle restatement (oracle/fusion_oracle.py feawei_dp_init, past_acc.py:98-103).
Tolerance: DP within 1e-5 absolute (fp32 column sums vs the reference's float64 mean; |DP| < 1)."""
import numpy as np
import pytest
import torch

from goldens import det_params, load
from oracle import fusion_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,zscore", [(1.0, True), (3.0, True), (5.0, False)])
@pytest.mark.parametrize("chunks", [(7,), (256, 256, 3), (1, 1000)])
def test_feawei_kernel_vs_oracle(k, zscore, chunks):
    from eegfusion.feawei import FeatureMean
    g = torch.Generator().manual_seed(sum(chunks) + int(k))
    f = torch.rand(sum(chunks), O.FUSED, generator=g)
    f[:, :768] *= 0.6                                   # distinct per-block means, like real features
    acc = FeatureMean("cuda")
    i = 0
    for c in chunks:
        acc.add(f[i: i + c].cuda())
        i += c
    assert acc.count == sum(chunks)
    got = acc.dp_init(k, zscore).cpu()
    want = O.feawei_dp_init(f.numpy(), k=k, zscore=zscore)
    assert got.shape == (1, O.FUSED)
    assert float((got - want).abs().max()) < 1e-5


def test_feawei_empty_raises():
    from eegfusion.feawei import FeatureMean
    with pytest.raises(RuntimeError):
        FeatureMean("cuda").dp_init()


def test_feawei_model_feature_pass():
    """Feature pass of the PriGumbel model (deterministic weights, dropout 0) over the golden
    window batch, then DP init, against the oracle's normalised feature -> feawei_dp_init."""
    from eegfusion.feawei import init_dp_
    from eegfusion.modules import PriGumbelModel
    cfg, fx = load("full_prigumbel_soft")
    p = det_params("W", "prigumbel", None, requires_grad=False)
    torch.manual_seed(0)
    m = PriGumbelModel(cfg["eps"], contract="W", dropout=0.0)
    m.load_state_dict(p, strict=False)
    m = m.cuda().train()
    eeg, act = torch.from_numpy(fx["eeg"]), torch.from_numpy(fx["act"])
    batches = [{"eeg": eeg[i: i + 1].cuda(), "act": act[i: i + 1].cuda()} for i in range(eeg.shape[0])]
    dp = init_dp_(m, batches, k=1.0, zscore=True).detach().cpu()
    ocfg = O.PathConfig(contract="W", variant="prigumbel", eps=cfg["eps"])
    with torch.no_grad():
        pooled, img, cross = O.encoders(p, {"eeg": eeg, "act": act}, ocfg)
        feat = O.minmax(torch.cat((pooled, img, cross), 1))
    want = O.feawei_dp_init(feat.numpy(), k=1.0, zscore=True)
    assert float((dp - want).abs().max()) < 1e-4
    assert m.DP.data_ptr() == m.arena.view("DP").data_ptr()      # still the arena view
