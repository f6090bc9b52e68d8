"""The python/src/custom_models surface on the CPU: the four dataset mirrors (custom_models/dataset.py)
over files in the reference's layout, the not-built baselines raising on construction, and the
reference's own base_train.py importing this build's `dataset` / `models` modules (VERDICT r2
missing #2)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

from custom_split import ACT_COEF, ACT_MODEL, EEG_COEF, EEG_MODEL, _std, write_custom_split

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")


@pytest.mark.parametrize("pair", ["ti", "tt", "it", "ii"])
def test_custom_datasets(tmp_path, pair):
    from custom_models import dataset as D
    write_custom_split(tmp_path, n=5)
    ek, ak = {"ti": ("txt", "img"), "tt": ("txt", "txt"), "it": ("img", "txt"), "ii": ("img", "img")}[pair]
    e = tmp_path / f"data/embedding/EEG/{ek}/{EEG_MODEL}_{_std(EEG_COEF)}/train.pickle"
    a = tmp_path / f"data/embedding/act/{ak}/{ACT_MODEL}_{_std(ACT_COEF)}/train.pickle"
    ds = getattr(D, f"MultiModalDataset_{pair}")(e, a, tmp_path / "data/processed/train_label.csv")
    assert len(ds) == 5
    e_in, e_mask, a_in, a_mask, y = ds[2]
    assert y.tolist() == [0]                                   # NaN -> 0
    if ek == "img":
        assert e_in.shape == (1, 512) and e_mask.tolist() == [1]
    else:
        assert e_in.shape == (128,) and e_in[0] == 101 and e_mask.shape == (128,)
    if ak == "img":
        assert a_in.shape == (1, 512) and a_mask.tolist() == [1]
    elif pair == "tt":
        assert torch.equal(a_in, a_mask)                       # the reference's quirk (dataset.py:62)
    else:
        assert a_in[0] == 101
    batch = torch.utils.data.default_collate([ds[i] for i in range(4)])
    assert len(batch) == 5 and batch[4].shape == (4, 1)


def test_not_built_baselines_raise_on_construction():
    from custom_models import models as M
    for cls in ("TICA_DPSGD", "TISC_LapDropoutEquWeight"):
        with pytest.raises(NotImplementedError, match="comparison baseline"):
            getattr(M, cls)("bert-base-uncased", 0.5) if cls.endswith("Weight") else getattr(M, cls)("x")


@pytest.mark.skipif(not REF.exists(), reason="needs the reference tree (survey container only)")
def test_reference_base_train_imports_this_build():
    """base_train.py:6-7 `from dataset import ...` / `from models import ...` resolve to this build's
    custom_models (first on sys.path); opacus is absent here and is stubbed (its PrivacyEngine is used
    only by the DPSGD branch).  Run in a child process: the reference sets CUDA_VISIBLE_DEVICES at
    import (base_train.py:2)."""
    code = f"""
import sys, types, importlib.util
sys.modules['opacus'] = types.SimpleNamespace(PrivacyEngine=object)
sys.path[:0] = [{str(ROOT / 'eeg-multimodal_amd' / 'custom_models')!r}, {str(ROOT / 'eeg-multimodal_amd')!r}]
spec = importlib.util.spec_from_file_location('ref_base_train', {str(REF / 'python/src/custom_models/base_train.py')!r})
m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
import dataset, models
assert dataset.__file__.startswith({str(ROOT)!r}) and models.__file__.startswith({str(ROOT)!r})
assert m.TICA_LapDropout is models.TICA_LapDropout and m.MultiModalDataset_tt is dataset.MultiModalDataset_tt
t = m.TrainAndTest(batch_size=2, epochs=1)
print('ok', type(t).__name__)
"""
    env = {k: v for k, v in os.environ.items()}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "ok TrainAndTest" in r.stdout, r.stderr[-3000:]
