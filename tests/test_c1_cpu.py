"""configs[0] (ConcatModel, train.py, batch 32, contract T) on the CPU: the oracle against the
c1_batch32 fixture the reference produced (tests/golden/make_golden.py gen_c1_batch32), and the
data.py mirror reading the split the fixture describes exactly as the reference's loader did."""
import numpy as np
import torch

from c1_split import write_c1_split
from goldens import det_params, load, rel_err
from oracle import fusion_oracle as O


def test_oracle_c1_per_sample_logits():
    """samples 0-3 (no op couples samples, so their logits equal the batch-32 rows); logits 2e-5."""
    cfg, fx = load("c1_batch32")
    p = det_params("T", "concat", requires_grad=False)
    sel = slice(0, 4)
    batch = {"title_input": torch.from_numpy(fx["title_input"][sel]), "text_mask": torch.from_numpy(fx["text_mask"][sel]),
             "frame_input": torch.from_numpy(fx["frame_input"][sel]),
             "vedio_mask": torch.ones(4, 1, dtype=torch.long)}
    with torch.no_grad():
        logits = O.forward(p, batch, O.PathConfig(contract="T", variant="concat"))
    assert rel_err(logits, fx["logits_all"][sel]) < 2e-5
    ce = torch.nn.functional.cross_entropy(logits, torch.from_numpy(fx["labels"][sel]), reduction="none")
    assert rel_err(ce, fx["ce_all"][sel]) < 2e-5


def test_loader_reads_c1_split_like_the_reference(tmp_path):
    from data import MultiModalDataset_ti
    fx = write_c1_split(tmp_path, "train")
    ds = MultiModalDataset_ti(tmp_path / "train_EEG.csv", tmp_path / "action" / "train_clip_v2.pickle",
                              tmp_path / "EEG" / "train_bert.pickle")
    assert len(ds) == 64
    (frame, vmask, ids, am), y = torch.utils.data.default_collate([ds[i] for i in range(64)])
    assert torch.equal(y.view(-1), torch.from_numpy(fx["labels"]))         # NaN rows -> 0, as the reference
    assert ids.shape == (64, 512) and torch.equal(ids, torch.from_numpy(fx["title_input"]))
    assert torch.equal(am, torch.from_numpy(fx["text_mask"]))
    assert torch.equal(frame, torch.from_numpy(fx["frame_input"]))
    assert vmask.shape == (64, 1) and int(vmask.sum()) == 64
    lens = fx["text_mask"].sum(1)
    assert lens.min() >= 33 and lens.max() <= 65 and abs(lens.mean() - 51.3) < 3
