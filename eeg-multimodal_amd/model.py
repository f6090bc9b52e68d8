"""Drop-in for the reference's model.py (model.py:8-64), backed by the MI355X engine.

`get_model(cfg)` / `ConcatModel()` keep the reference signatures; `forward(x, hard=True)` takes
x = (frame_input [B,1,512] f32, vedio_mask [B,1], title_input [B,512] i64, text_mask [B,512] i64)
and returns logits [B,2].  `BertModel.from_pretrained('bert-base-uncased')` cannot run offline:
BERT starts from the BERT initialiser (normal(0, 0.02)); set EEGF_BERT_WEIGHTS to a local
safetensors file / HF directory to load pretrained weights.  On a machine without a GPU the model
stays in host memory and runs the torch-op host path (eegfusion/cpu_path.py).
"""
import os

import torch

from eegfusion.modules import ConcatModel as _ConcatModel
from eegfusion.modules import load_bert_weights


def get_model(cfg):
    """model.py:8-12.  The reference moves the model to CUDA unconditionally; here it goes to the GPU
    when one is present and stays in host memory otherwise (configs[0]'s no-GPU plumbing run,
    SURVEY §8(f)#1), where it computes with torch ops (eegfusion/cpu_path.py)."""
    if cfg.data_name == 'EEG':
        model = ConcatModel()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    model.eps = torch.tensor(cfg.eps).to(dev)
    return model.to(dev)


class ConcatModel(_ConcatModel):
    """model.py:14-64 (contract T: BERT over token ids + Linear(512,768) over the CLIP vector)."""

    def __init__(self):
        super().__init__(contract="T")
        w = os.environ.get("EEGF_BERT_WEIGHTS")
        if w:
            load_bert_weights(self, w)
