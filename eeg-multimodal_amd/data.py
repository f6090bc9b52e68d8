"""Drop-in for the reference's data.py (data.py:7-45): MultiModalDataset_ti and get_data.

Host-side Python, same behaviour: labels from the EEG CSV (NaN -> 0), CLIP action vectors from a
pickled ndarray, BERT token ids/masks from a pickled list of encodings.  The token pickle holds
`transformers.BatchEncoding` objects; a restricted unpickler maps that class (and only the numpy /
builtin reconstructors) to plain containers so no `transformers` import is needed.  Use it on your
own feature files only.
"""
import pickle

import pandas as pd
import torch
from torch.utils.data import Dataset

_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"), ("builtins", "dict"), ("builtins", "list"),
    ("collections", "OrderedDict"), ("_codecs", "encode"),
}


class _Encoding(dict):
    """Stand-in for transformers.BatchEncoding: a dict that accepts the pickled state."""

    def __setstate__(self, state):
        if isinstance(state, dict):
            self.update(state.get("data", state))


class _RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if name in ("BatchEncoding", "Encoding") and module.startswith("transformers"):
            return _Encoding
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name}")


def load_feature_pickle(path):
    with open(path, "rb") as f:
        return _RestrictedUnpickler(f).load()


class MultiModalDataset_ti(Dataset):
    '''
    treat eeg as txt, action as img. ti means txt + img   (data.py:7-34)
    '''

    def __init__(self, eeg_df_path, action_path, eeg_path):
        self.eeg_df = pd.read_csv(eeg_df_path)
        self.label = self.eeg_df['label']
        self.train_clip_feature = load_feature_pickle(action_path)
        self.train_text_embedding = load_feature_pickle(eeg_path)

    def __len__(self):
        return len(self.eeg_df)

    def __getitem__(self, idx):
        video_feature = torch.tensor(self.train_clip_feature[idx]).unsqueeze(0)      # [1, 512]
        mask = torch.tensor([1])
        input_ids = torch.tensor(self.train_text_embedding[idx]['input_ids'])
        attention_mask = torch.tensor(self.train_text_embedding[idx]['attention_mask'])
        label = self.label[idx]
        if pd.isnull(label):
            label = 0
        label = torch.LongTensor([label])
        return (video_feature, mask, input_ids, attention_mask), label


class DeviceBatchLoader:
    """Batched loader for a map-style dataset such as MultiModalDataset_ti.

    The reference collates sample by sample on the host and copies every batch to the device
    (data.py:22-34 + DataLoader default collate, train.py:96-98).  Here the split is collated ONCE
    (the feature files are tens of MB), staged through pinned host memory, and kept resident in HBM;
    each batch is a device-side row gather of the epoch permutation — no per-sample Python and no
    per-step host-to-device copy.  Batches have the structure, shapes and dtypes of
    DataLoader(dataset, batch_size, shuffle) with the default collate, and with shuffle=True the
    sample order is the one RandomSampler draws from the same global torch RNG state (one int64 seed
    draw per epoch after the iterator's base-seed draw, then randperm on a CPU generator), so a seeded
    run sees the reference's batches and leaves the global RNG where DataLoader leaves it."""

    def __init__(self, dataset, batch_size, shuffle=True, device=None, drop_last=False):
        self.batch_size, self.shuffle, self.drop_last = int(batch_size), bool(shuffle), bool(drop_last)
        self.n = len(dataset)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        items = [dataset[i] for i in range(self.n)]
        collate = torch.utils.data.default_collate
        host = collate(items)                                   # ((f, m, ids, mask), label) stacked
        pin = self.device.type == "cuda"

        def stage(t):
            t = t.contiguous()
            if pin:
                t = t.pin_memory()
            return t.to(self.device, non_blocking=pin)

        self.data = _tree_map(stage, host)
        if pin:
            torch.cuda.current_stream(self.device).synchronize()

    def __len__(self):
        return self.n // self.batch_size if self.drop_last else (self.n + self.batch_size - 1) // self.batch_size

    def _order(self):
        # the DataLoader iterator draws its worker base seed first (_BaseDataLoaderIter.__init__), then
        # RandomSampler.__iter__ draws the permutation seed: consume the global RNG the same way
        torch.empty((), dtype=torch.int64).random_()
        if not self.shuffle:
            return torch.arange(self.n)
        seed = int(torch.empty((), dtype=torch.int64).random_().item())     # RandomSampler.__iter__
        g = torch.Generator()
        g.manual_seed(seed)
        return torch.randperm(self.n, generator=g)

    def __iter__(self):
        order = self._order().to(self.device)
        for i in range(len(self)):
            idx = order[i * self.batch_size:(i + 1) * self.batch_size]
            yield _tree_map(lambda t: t.index_select(0, idx), self.data)


def _tree_map(fn, x):
    if isinstance(x, (list, tuple)):
        return type(x)(_tree_map(fn, v) for v in x) if isinstance(x, tuple) else [_tree_map(fn, v) for v in x]
    return fn(x)


def get_data(cfg):
    """data.py:37-45.  cfg.device_loader = True (optional, not in the reference) serves both splits
    through DeviceBatchLoader instead of DataLoader (same batches, resident in HBM)."""
    if getattr(cfg, "device_loader", False):
        tr, va = (MultiModalDataset_ti('feature/train_EEG.csv', 'feature/action/train_clip_v2.pickle',
                                       'feature/EEG/train_bert.pickle'),
                  MultiModalDataset_ti('feature/test_EEG.csv', 'feature/action/test_clip_v2.pickle',
                                       'feature/EEG/test_bert.pickle'))
        print(len(va))
        return (DeviceBatchLoader(tr, cfg.batch_size, shuffle=True),
                DeviceBatchLoader(va, cfg.batch_size, shuffle=True))
    batch_size = cfg.batch_size
    if cfg.data_name == 'EEG':
        train_dataset = MultiModalDataset_ti('feature/train_EEG.csv', 'feature/action/train_clip_v2.pickle',
                                             'feature/EEG/train_bert.pickle')
        val_dataset = MultiModalDataset_ti('feature/test_EEG.csv', 'feature/action/test_clip_v2.pickle',
                                           'feature/EEG/test_bert.pickle')
        print(len(val_dataset))
        train_dataloader = torch.utils.data.DataLoader(train_dataset, batch_size=batch_size, shuffle=True)
        val_dataloader = torch.utils.data.DataLoader(val_dataset, batch_size=batch_size, shuffle=True)
    return train_dataloader, val_dataloader


class WindowDataset(Dataset):
    """Synthetic contract-W stream (BASELINE configs 2-5): EEG windows [C, T] ~ N(0,1), action
    vectors [A] ~ N(0, 0.5^2) (CLIP-feature std), labels ~ Bernoulli(0.66) (train-set positive rate
    1589/2402).  Deterministic per (seed, index); `shard`/`num_shards` give disjoint rank shards."""

    def __init__(self, n, channels=64, steps=256, act_dim=32, seed=980616, shard=0, num_shards=1):
        self.idx = list(range(shard, n, num_shards))
        self.c, self.t, self.a, self.seed = channels, steps, act_dim, seed

    def __len__(self):
        return len(self.idx)

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + self.idx[i])
        eeg = torch.randn(self.c, self.t, generator=g)
        act = torch.randn(self.a, generator=g) * 0.5
        label = torch.LongTensor([int(torch.rand(1, generator=g).item() < 0.66)])
        return (eeg, act), label
