"""Drop-in for the reference's past_acc.py (PriGumbel "newfrac"): ConcatModel(epsilon),
cal_loss, MultiModalDataset_ti (5-tuple variant) and the two-optimizer training loop main2."""
import os

import numpy as np
import pandas as pd
import torch
import torch.nn.functional as F
from torch.optim import Adam
from torch.utils.data import Dataset

from data import load_feature_pickle
from eegfusion.modules import PriGumbelModel


def set_seed(seed):
    """past_acc.py:21-31"""
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)


class MultiModalDataset_ti(Dataset):
    """past_acc.py:42-69 (returns a flat 5-tuple)"""

    def __init__(self, eeg_df_path, action_path, eeg_path):
        self.eeg_df = pd.read_csv(eeg_df_path)
        self.label = self.eeg_df['label']
        self.train_clip_feature = load_feature_pickle(action_path)
        self.train_text_embedding = load_feature_pickle(eeg_path)

    def __len__(self):
        return len(self.eeg_df)

    def __getitem__(self, idx):
        video_feature = torch.tensor(self.train_clip_feature[idx]).unsqueeze(0)
        mask = torch.tensor([1])
        input_ids = torch.tensor(self.train_text_embedding[idx]['input_ids'])
        attention_mask = torch.tensor(self.train_text_embedding[idx]['attention_mask'])
        label = self.label[idx]
        if pd.isnull(label):
            label = 0
        return video_feature, mask, input_ids, attention_mask, torch.LongTensor([label])


def cal_loss(prediction, label):
    """past_acc.py:71-77"""
    label = label.squeeze(dim=1)
    loss = F.cross_entropy(prediction, label)
    with torch.no_grad():
        pred_label_id = torch.argmax(prediction, dim=1)
        accuracy = (label == pred_label_id).float().sum() / label.shape[0]
    return loss, accuracy, pred_label_id, label


class ConcatModel(PriGumbelModel):
    """past_acc.py:79-139"""

    def __init__(self, epsilon):
        super().__init__(float(epsilon), contract="T")


def feawei_init(model, dataloader, k=1.0, zscore=True, device=None):
    """feawei DP initialisation (past_acc.py:98-103; past_acc_feawei.py:127-163): a train-mode,
    hard=False feature pass over `dataloader` (reference 5-tuples), column means of the normalised
    features, z-score (zscore=True) and DP = cat(0.4, 0.5, 0.3) + 1 - sigmoid(k z) - 0.5.  Runs on
    the device (eegfusion.feawei); sets and returns model.DP."""
    from eegfusion.feawei import init_dp_
    device = device or model.arena.device
    model.train()

    def batches():
        for frame_input, vedio_mask, title_input, text_mask, *_ in dataloader:
            yield model._token_batch(*(t.to(device) for t in (frame_input, vedio_mask, title_input, text_mask)))

    return init_dp_(model, batches(), k=k, zscore=zscore)


def main2(epsilon, suffix, batch_size=8, epochs=50, learning_rate=1e-6, feature_dir='feature',
          record_dir='model_dict/eps_experiment/', device=None):
    """past_acc.py:142-250: DP pass (hard=False) -> DP Adam; model pass (hard=True) -> model Adam."""
    from sklearn.metrics import f1_score
    device = device or torch.device('cuda')
    train_dataset = MultiModalDataset_ti(f'{feature_dir}/train_EEG.csv', f'{feature_dir}/action/train_clip_v2.pickle',
                                         f'{feature_dir}/EEG/train_bert.pickle')
    val_dataset = MultiModalDataset_ti(f'{feature_dir}/test_EEG.csv', f'{feature_dir}/action/test_clip_v2.pickle',
                                       f'{feature_dir}/EEG/test_bert.pickle')
    train_dataloader = torch.utils.data.DataLoader(train_dataset, batch_size=batch_size, shuffle=True)
    val_dataloader = torch.utils.data.DataLoader(val_dataset, batch_size=batch_size, shuffle=True)
    model = ConcatModel(epsilon)
    DP_params = [p for n, p in model.named_parameters() if 'DP' in n]
    model_params = [p for n, p in model.named_parameters() if 'DP' not in n]
    model_optimizer = Adam(model_params, lr=learning_rate)
    DP_optimizer = Adam(DP_params, lr=learning_rate)
    os.makedirs(record_dir + suffix, exist_ok=True)
    whole_record_path = record_dir + suffix + 'whole_record.txt'
    best_record_path = record_dir + suffix + 'best_record.txt'
    save_model_path = record_dir + suffix + 'best_f1.pickle'
    model = model.to(device)
    f1_score_best = 0.5
    for epoch in range(epochs):
        epoch_acc_train = epoch_loss_train = epoch_acc_val = epoch_loss_val = 0
        sample_size_train = sample_size_val = 0
        model.train()
        for frame_input, vedio_mask, title_input, text_mask, label in train_dataloader:
            sample_size_train += 1
            DP_optimizer.zero_grad()
            frame_input, vedio_mask, title_input, text_mask, label = (t.to(device) for t in
                                                                      (frame_input, vedio_mask, title_input, text_mask,
                                                                       label))
            prediction = model(frame_input, vedio_mask, title_input, text_mask, hard=False)
            loss, accuracy, _, _ = cal_loss(prediction, label)
            loss.backward()
            DP_optimizer.step()
            model_optimizer.zero_grad()
            prediction = model(frame_input, vedio_mask, title_input, text_mask, hard=True)
            loss, accuracy, _, _ = cal_loss(prediction, label)
            epoch_loss_train += loss.item()
            epoch_acc_train += accuracy.item()
            loss.backward()
            model_optimizer.step()
        prediction_all, label_all = [], []
        with torch.no_grad():
            for frame_input, vedio_mask, title_input, text_mask, label in val_dataloader:
                sample_size_val += 1
                frame_input, vedio_mask, title_input, text_mask, label = (t.to(device) for t in
                                                                          (frame_input, vedio_mask, title_input,
                                                                           text_mask, label))
                prediction = model(frame_input, vedio_mask, title_input, text_mask, hard=True)
                loss, accuracy, pred_label_id, label_id = cal_loss(prediction, label)
                prediction_all.extend(pred_label_id.cpu().numpy())
                label_all.extend(label_id.cpu().numpy())
                epoch_loss_val += loss.item()
                epoch_acc_val += accuracy.item()
        f1_score_epoch = f1_score(prediction_all, label_all)
        record = f'''Epochs: {epoch + 1}
        | Train Loss: {epoch_loss_train/sample_size_train: .3f}
        | Train Accuracy: {epoch_acc_train/sample_size_train: .3f}
        | Val Loss: {epoch_loss_val/sample_size_val: .3f}
        | Val Accuracy: {epoch_acc_val/sample_size_val: .3f}
        | f_1 Score: {f1_score_epoch: .3f}\n'''
        print(record)
        with open(whole_record_path, "a") as file:
            file.write(record)
        if f1_score_epoch > f1_score_best:
            torch.save(model.state_dict(), save_model_path)
            f1_score_best = f1_score_epoch
            with open(best_record_path, "w") as file:
                file.write(record)
