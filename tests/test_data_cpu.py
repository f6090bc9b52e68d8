"""data.py mirror: MultiModalDataset_ti over feature files written by this test (same formats as the
reference's feature/ directory: CSV labels, pickled ndarray, pickled list of BatchEncoding)."""
import pickle
import types

import numpy as np
import pandas as pd
import pytest
import torch


def _write_split(tmp_path, n=5, L=512):
    rng = np.random.default_rng(0)
    labels = [1.0, 0.0, float("nan"), 1.0, 0.0][:n]
    pd.DataFrame({"EEG": ["1 2 3"] * n, "label": labels}).to_csv(tmp_path / "x_EEG.csv", index=False)
    (tmp_path / "action").mkdir(exist_ok=True)
    (tmp_path / "EEG").mkdir(exist_ok=True)
    with open(tmp_path / "action" / "x_clip_v2.pickle", "wb") as f:
        pickle.dump(rng.standard_normal((n, 512)).astype(np.float32), f)
    try:
        from transformers import BatchEncoding
        enc = [BatchEncoding({"input_ids": [[101] + [1000 + i] * 5 + [102] + [0] * (L - 7)],
                              "attention_mask": [[1] * 7 + [0] * (L - 7)]}) for i in range(n)]
    except Exception:
        enc = [{"input_ids": [[101] + [1000 + i] * 5 + [102] + [0] * (L - 7)],
                "attention_mask": [[1] * 7 + [0] * (L - 7)]} for i in range(n)]
    with open(tmp_path / "EEG" / "x_bert.pickle", "wb") as f:
        pickle.dump(enc, f)


def test_multimodal_dataset_ti_items(tmp_path):
    from data import MultiModalDataset_ti
    _write_split(tmp_path)
    ds = MultiModalDataset_ti(tmp_path / "x_EEG.csv", tmp_path / "action" / "x_clip_v2.pickle",
                              tmp_path / "EEG" / "x_bert.pickle")
    assert len(ds) == 5
    (frame, mask, ids, am), label = ds[2]
    assert frame.shape == (1, 512) and frame.dtype == torch.float32
    assert mask.tolist() == [1]
    assert ids.shape == (1, 512) and am.shape == (1, 512)
    assert label.tolist() == [0]                      # NaN label -> 0 (data.py:29-32)
    loader = torch.utils.data.DataLoader(ds, batch_size=4)
    (f, m, i, a), y = next(iter(loader))
    assert f.shape == (4, 1, 512) and m.shape == (4, 1) and i.shape == (4, 1, 512) and y.shape == (4, 1)


def test_restricted_unpickler_refuses_code(tmp_path):
    from data import load_feature_pickle
    import os
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    p = tmp_path / "evil.pickle"
    with open(p, "wb") as f:
        pickle.dump(Evil(), f)
    with pytest.raises(pickle.UnpicklingError):
        load_feature_pickle(p)


def test_window_dataset_shards_are_disjoint_and_deterministic():
    from data import WindowDataset
    full = WindowDataset(10)
    a, b = WindowDataset(10, shard=0, num_shards=2), WindowDataset(10, shard=1, num_shards=2)
    assert len(a) + len(b) == 10 and set(a.idx).isdisjoint(b.idx)
    (e0, _), _ = full[3]
    (e1, _), _ = b[1]                                   # global index 3
    assert torch.equal(e0, e1)
    assert e0.shape == (64, 256)


def test_get_data_signature(tmp_path, monkeypatch):
    from data import get_data
    for split in ("train", "test"):
        _write_split(tmp_path)
        (tmp_path / "x_EEG.csv").rename(tmp_path / f"{split}_EEG.csv")
        (tmp_path / "action" / "x_clip_v2.pickle").rename(tmp_path / "action" / f"{split}_clip_v2.pickle")
        (tmp_path / "EEG" / "x_bert.pickle").rename(tmp_path / "EEG" / f"{split}_bert.pickle")
    (tmp_path / "feature").mkdir()
    for p in list(tmp_path.iterdir()):
        if p.name != "feature":
            p.rename(tmp_path / "feature" / p.name)
    monkeypatch.chdir(tmp_path)
    tr, va = get_data(types.SimpleNamespace(batch_size=2, data_name="EEG"))
    assert len(tr.dataset) == 5 and len(va.dataset) == 5


def test_device_batch_loader_matches_dataloader(tmp_path):
    """DeviceBatchLoader (collated once, resident, device-side gathers) serves the batches the
    reference's DataLoader(shuffle=True) serves from the same global seed: same structure, shapes,
    dtypes, values and sample order (RandomSampler's RNG draw), last partial batch included."""
    from data import DeviceBatchLoader, MultiModalDataset_ti
    _write_split(tmp_path, n=5)
    ds = MultiModalDataset_ti(tmp_path / "x_EEG.csv", tmp_path / "action" / "x_clip_v2.pickle",
                              tmp_path / "EEG" / "x_bert.pickle")
    for shuffle in (True, False):
        torch.manual_seed(980616)
        ref = [b for _ in range(2) for b in torch.utils.data.DataLoader(ds, batch_size=2, shuffle=shuffle)]
        torch.manual_seed(980616)
        dl = DeviceBatchLoader(ds, batch_size=2, shuffle=shuffle, device="cpu")
        got = [b for _ in range(2) for b in dl]
        assert len(dl) == 3 and len(got) == len(ref) == 6
        for (xr, yr), (xg, yg) in zip(ref, got):
            assert type(xr) is type(xg) and len(xr) == len(xg) == 4
            for a, b in zip(list(xr) + [yr], list(xg) + [yg]):
                assert a.shape == b.shape and a.dtype == b.dtype and torch.equal(a, b)
