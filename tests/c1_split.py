"""configs[0] split helper (tests only): writes the c1_batch32 fixture's 64 samples as feature files in
the reference's formats (feature/{prefix}_EEG.csv, action/{prefix}_clip_v2.pickle ndarray [N, 512] f32,
EEG/{prefix}_bert.pickle list of encodings with 1-D input_ids / attention_mask), the same layout
tests/golden/make_golden.py wrote for the reference's own data.MultiModalDataset_ti."""
from __future__ import annotations

import pickle
from pathlib import Path

import numpy as np
import pandas as pd

from goldens import load


def write_c1_split(feature_dir: Path, prefix: str):
    _, fx = load("c1_batch32")
    ids, mask = fx["title_input"], fx["text_mask"]
    (feature_dir / "action").mkdir(parents=True, exist_ok=True)
    (feature_dir / "EEG").mkdir(parents=True, exist_ok=True)
    pd.DataFrame({"EEG": [" ".join(map(str, r[r > 0].tolist())) for r in ids],
                  "label": fx["labels_csv"]}).to_csv(feature_dir / f"{prefix}_EEG.csv", index=False)
    with open(feature_dir / "action" / f"{prefix}_clip_v2.pickle", "wb") as f:
        pickle.dump(np.ascontiguousarray(fx["frame_input"][:, 0]), f)
    try:
        from transformers import BatchEncoding as Enc
    except Exception:                                   # the loader maps BatchEncoding to a dict anyway
        Enc = dict
    enc = [Enc({"input_ids": ids[i].tolist(), "attention_mask": mask[i].tolist()}) for i in range(len(ids))]
    with open(feature_dir / "EEG" / f"{prefix}_bert.pickle", "wb") as f:
        pickle.dump(enc, f)
    return fx
