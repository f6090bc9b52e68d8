"""Feature files in the layout python/src/custom_models/base_train.py reads (tests only):
data/embedding/{EEG,act}/{txt,img}/<model>_<coef>/{train,test}.pickle and
data/processed/{train,test}_label.csv.  txt = pickled list of BERT encodings (1-D lists), img =
pickled ndarray [N, 512] f32."""
from __future__ import annotations

import pickle
from pathlib import Path

import numpy as np
import pandas as pd

EEG_MODEL, EEG_COEF, ACT_MODEL, ACT_COEF = "bert", "bert-base-uncased", "clip", "ViT-B/32"


def _std(c):
    return c.replace("/", "_").replace("-", "_")


def write_custom_split(root: Path, n=5, L=128, seed=0):
    rng = np.random.default_rng(seed)
    try:
        from transformers import BatchEncoding as Enc
    except Exception:
        Enc = dict
    for split in ("train", "test"):
        for side, model, coef in (("EEG", EEG_MODEL, EEG_COEF), ("act", ACT_MODEL, ACT_COEF)):
            for kind in ("txt", "img"):
                d = root / "data" / "embedding" / side / kind / f"{model}_{_std(coef)}"
                d.mkdir(parents=True, exist_ok=True)
                if kind == "img":
                    obj = (rng.standard_normal((n, 512)) * 0.5).astype(np.float32)
                else:
                    obj = []
                    for i in range(n):
                        k = int(rng.integers(20, 60))
                        ids = [101] + rng.integers(1015, 1025, k - 2).tolist() + [102] + [0] * (L - k)
                        obj.append(Enc({"input_ids": ids, "attention_mask": [1] * k + [0] * (L - k)}))
                with open(d / f"{split}.pickle", "wb") as f:
                    pickle.dump(obj, f)
        (root / "data" / "processed").mkdir(parents=True, exist_ok=True)
        labels = [1.0, 0.0, float("nan"), 1.0, 0.0, 1.0, 0.0, 1.0][:n]
        pd.DataFrame({"label": labels}).to_csv(root / "data" / "processed" / f"{split}_label.csv", index=False)
