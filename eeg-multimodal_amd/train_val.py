"""Drop-in for the reference's train_val.py (PriGumbel-v1): ConcatModel(tau, epsilon),
cal_loss, loss_function and the `pretrain` loop (train_val.py:72-277).

The model's gumbel_dropout (:95-101), GumbelSoftmaxDropout (:103-112) and Lap_noise (:114-123) run
fused inside the engine (eegf_v1_gate_fwd / bwd); `GumbelSoftmaxDropout` is the parameter-free holder
of tau, as in the reference.  loss_function's privacy term is the caller's torch expression on
model.w, exactly as in the reference (the engine's PriGumbelV1Trainer fuses it instead)."""
import os
import pickle

import numpy as np
import torch
import torch.nn.functional as F

from eegfusion.modules import GumbelSoftmaxDropout, PriGumbelV1Model  # noqa: F401
from past_acc import MultiModalDataset_ti, set_seed  # noqa: F401  (train_val.py:22-70: same dataset)


def cal_loss(prediction, label):
    """train_val.py:72-78"""
    label = label.squeeze(dim=1)
    loss = F.cross_entropy(prediction, label)
    with torch.no_grad():
        pred_label_id = torch.argmax(prediction, dim=1)
        accuracy = (label == pred_label_id).float().sum() / label.shape[0]
    return loss, accuracy, pred_label_id, label


def loss_function(prediction, label, model, alpha, epsilon):
    """train_val.py:80-93: alpha * CE + max_j((1 - w_j) e^eps + w_j)"""
    label = label.squeeze(dim=1)
    cross_entropy_loss = F.cross_entropy(prediction, label)
    with torch.no_grad():
        pred_label_id = torch.argmax(prediction, dim=1)
        accuracy = (label == pred_label_id).float().sum() / label.shape[0]
    tmp = (1 - model.w) * np.exp(epsilon) + model.w
    loss_w, _ = torch.max(tmp, dim=0)
    total_loss = alpha * cross_entropy_loss + loss_w
    return total_loss, accuracy, pred_label_id, label


class ConcatModel(PriGumbelV1Model):
    """train_val.py:125-158"""

    def __init__(self, tau, epsilon, **kw):
        super().__init__(tau, epsilon, contract=kw.pop("contract", "T"), **kw)


def pretrain(tau, epsilon, alpha, path, learning_rate, feature_dir='feature', epochs=30, batch_size=8):
    """train_val.py:160-277: Adam over all parameters; per epoch the train loop, the w statistics
    (privacy budget max / avg, dropout rate max / avg), evaluation in eval mode (hard masks), F1,
    records, best-F1 checkpoint, and result.pkl with the per-epoch lists."""
    from sklearn.metrics import f1_score

    from eegfusion.optim import Adam
    train_dataset = MultiModalDataset_ti(f'{feature_dir}/train_EEG.csv', f'{feature_dir}/action/train_clip_v2.pickle',
                                         f'{feature_dir}/EEG/train_bert.pickle')
    val_dataset = MultiModalDataset_ti(f'{feature_dir}/test_EEG.csv', f'{feature_dir}/action/test_clip_v2.pickle',
                                       f'{feature_dir}/EEG/test_bert.pickle')
    train_dataloader = torch.utils.data.DataLoader(train_dataset, batch_size=batch_size, shuffle=True)
    val_dataloader = torch.utils.data.DataLoader(val_dataset, batch_size=batch_size, shuffle=True)
    model = ConcatModel(tau, epsilon)
    optimizer = Adam(model.parameters(), lr=learning_rate)
    os.makedirs(path, exist_ok=True)
    whole_record_path, best_record_path, save_model_path = (path + 'whole_record.txt', path + 'best_record.txt',
                                                            path + 'best_f1.pickle')
    device = torch.device("cuda")
    model = model.to(device)
    train_acc_list, val_acc_list, w_list = [], [], []
    pb_max_list, pb_avg_list, dr_max_list, dr_avg_list = [], [], [], []
    f1_score_best = 0.5
    for epoch in range(epochs):
        epoch_acc_train = epoch_loss_train = epoch_acc_val = epoch_loss_val = 0
        sample_size_train = sample_size_val = 0
        model.train()
        for frame_input, vedio_mask, title_input, text_mask, label in train_dataloader:
            sample_size_train += 1
            optimizer.zero_grad()
            frame_input, vedio_mask, title_input, text_mask, label = (
                t.to(device) for t in (frame_input, vedio_mask, title_input, text_mask, label))
            prediction = model(frame_input, vedio_mask, title_input, text_mask)
            loss, accuracy, pred_label_id, label_id = loss_function(prediction, label, model, alpha, epsilon)
            epoch_loss_train += loss.item()
            epoch_acc_train += accuracy.item()
            loss.backward(retain_graph=True)
            optimizer.step()
        prediction_all, label_all = [], []
        model.eval()
        tmp = (1 - model.w) * np.exp(epsilon) + model.w
        privacy_budget_max, _ = torch.max(tmp, dim=0)
        privacy_budget_avg = torch.mean(tmp)
        drop_out_rate_max = model.w.max()
        drop_out_rate_avg = torch.mean(model.w)
        w_list.append(model.w.detach().cpu().clone())
        with torch.no_grad():
            for frame_input, vedio_mask, title_input, text_mask, label in val_dataloader:
                sample_size_val += 1
                frame_input, vedio_mask, title_input, text_mask, label = (
                    t.to(device) for t in (frame_input, vedio_mask, title_input, text_mask, label))
                prediction = model(frame_input, vedio_mask, title_input, text_mask)
                loss, accuracy, pred_label_id, label_id = loss_function(prediction, label, model, alpha, epsilon)
                prediction_all.extend(pred_label_id.cpu().numpy())
                label_all.extend(label_id.cpu().numpy())
                epoch_loss_val += loss.item()
                epoch_acc_val += accuracy.item()
        f1_score_epoch = f1_score(prediction_all, label_all)
        train_acc_list.append(epoch_acc_train / sample_size_train)
        val_acc_list.append(epoch_acc_val / sample_size_val)
        pb_max_list.append(float(privacy_budget_max))
        pb_avg_list.append(float(privacy_budget_avg))
        dr_max_list.append(float(drop_out_rate_max))
        dr_avg_list.append(float(drop_out_rate_avg))
        record = f'''Epochs: {epoch + 1}
        | Train Loss: {epoch_loss_train/sample_size_train: .3f}
        | Train Accuracy: {epoch_acc_train/sample_size_train: .3f}
        | Val Loss: {epoch_loss_val/sample_size_val: .3f}
        | Val Accuracy: {epoch_acc_val/sample_size_val: .3f}
        | f_1 Score: {f1_score_epoch: .3f}
        | privacy_budget_max: {privacy_budget_max: .3f}
        | privacy_budget_avg: {privacy_budget_avg: .3f}
        | drop_out_rate_max: {drop_out_rate_max: .3f}
        | drop_out_rate_avg: {drop_out_rate_avg: .3f}
        | alpha: {alpha:.3f}\n'''
        print(record)
        with open(whole_record_path, "a") as file:
            file.write(record)
        if f1_score_epoch > f1_score_best:
            torch.save(model.state_dict(), save_model_path)
            f1_score_best = f1_score_epoch
            with open(best_record_path, "w") as file:
                file.write(record)
    # the reference pickles its lists of tensors (:275-277); plain floats / CPU tensors here
    with open(path + 'result.pkl', 'wb') as f:
        pickle.dump((train_acc_list, val_acc_list, w_list, pb_max_list, pb_avg_list, dr_max_list, dr_avg_list), f)
    return model, f1_score_best
