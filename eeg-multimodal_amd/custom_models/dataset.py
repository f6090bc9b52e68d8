"""Drop-in for python/src/custom_models/dataset.py (:21-121): the four modality-pairing datasets
TrainAndTest loads (base_train.py:6,74-129).  Each item is the reference's 5-tuple
(eeg_input, eeg_mask, act_input, act_mask, label [1] int64, NaN label -> 0).  "txt" files are pickled
lists of BERT encodings ('input_ids' / 'attention_mask'), "img" files pickled [N, 512] float arrays;
both are read through data.load_feature_pickle (restricted unpickler: no transformers import, no code
from the file).  The reference seeds torch / numpy at import (:19); that is kept."""
import numpy as np
import pandas as pd
import torch
from torch.utils.data import Dataset

from data import load_feature_pickle


def set_seed(seed):
    """dataset.py:7-17"""
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)


set_seed(980616)


def _txt(enc, key):
    return torch.tensor(enc[key])                    # [L] (or [1, L] for [[...]] encodings)


def _img(arr):
    return torch.tensor(arr).unsqueeze(0)            # [1, 512]


def _label(labels, idx):
    y = labels[idx]
    return torch.LongTensor([0 if pd.isnull(y) else y])


class _Pair(Dataset):
    """Two pickled feature files + a label CSV; `kinds` says how each side is read."""
    kinds = ("txt", "img")

    def __init__(self, eeg_path, act_path, label_df_path):
        self.eeg = load_feature_pickle(eeg_path)
        self.act = load_feature_pickle(act_path)
        self.label = pd.read_csv(label_df_path)['label']

    def __len__(self):
        return len(self.label)

    @staticmethod
    def _side(kind, item, mask_as_input=False):
        if kind == "img":
            return _img(item), torch.tensor([1])
        return _txt(item, 'attention_mask' if mask_as_input else 'input_ids'), _txt(item, 'attention_mask')

    def __getitem__(self, idx):
        e_in, e_mask = self._side(self.kinds[0], self.eeg[idx])
        a_in, a_mask = self._side(self.kinds[1], self.act[idx], self.kinds == ("txt", "txt"))
        return e_in, e_mask, a_in, a_mask, _label(self.label, idx)


class MultiModalDataset_ti(_Pair):
    '''treat eeg as txt, act as img; ti means txt + img (dataset.py:21-44)'''
    kinds = ("txt", "img")


class MultiModalDataset_tt(_Pair):
    '''treat eeg as txt, act as txt (dataset.py:46-69).  As in the reference (:62), the action token
    input is read from the encoding's 'attention_mask', not its 'input_ids'.'''
    kinds = ("txt", "txt")


class MultiModalDataset_it(_Pair):
    '''treat eeg as img, act as txt (dataset.py:71-95)'''
    kinds = ("img", "txt")


class MultiModalDataset_ii(_Pair):
    '''treat eeg as img, act as img (dataset.py:97-121)'''
    kinds = ("img", "img")
