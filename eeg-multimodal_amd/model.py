"""Drop-in for the reference's model.py (model.py:8-64), backed by the MI355X engine.

`get_model(cfg)` / `ConcatModel()` keep the reference signatures; `forward(x, hard=True)` takes
x = (frame_input [B,1,512] f32, vedio_mask [B,1], title_input [B,512] i64, text_mask [B,512] i64)
and returns logits [B,2].  `BertModel.from_pretrained('bert-base-uncased')` cannot run offline:
BERT starts from the BERT initialiser (normal(0, 0.02)); set EEGF_BERT_WEIGHTS to a local
safetensors file / HF directory to load pretrained weights.
"""
import os

import torch

from eegfusion.modules import ConcatModel as _ConcatModel
from eegfusion.modules import load_bert_weights


def get_model(cfg):
    """model.py:8-12"""
    if cfg.data_name == 'EEG':
        model = ConcatModel()
    model.eps = torch.tensor(cfg.eps).cuda()
    return model.cuda()


class ConcatModel(_ConcatModel):
    """model.py:14-64 (contract T: BERT over token ids + Linear(512,768) over the CLIP vector)."""

    def __init__(self):
        super().__init__(contract="T")
        w = os.environ.get("EEGF_BERT_WEIGHTS")
        if w:
            load_bert_weights(self, w)
