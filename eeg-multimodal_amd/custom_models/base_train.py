"""Drop-in for python/src/custom_models/base_train.py: TrainAndTest (:47-553), the paper package's
harness, over this build's models and datasets.

  * 'lapacian_dropout' (:156-255): the PriGumbel two-optimizer loop for every modality pairing —
    DP Adam on a hard=False pass, model Adam on a hard=True pass — with the reference's per-pairing
    input casts, evaluation in eval mode (:214), sklearn F1 over the test split, the whole / best
    record files and the best-F1 checkpoint (threshold 0.5);
  * 'NDP' (:438-494): TICA_NonPrivate with one Adam over all parameters;
  * 'DPSGD' / 'lapacian_dropout_equal_weight' select TICA_DPSGD / TISC_LapDropoutEquWeight, which are
    not built (custom_models/models.py) and raise on construction.
Paths are the reference's (data/embedding/{EEG,act}/{txt,img}/<model>_<coef>/{train,test}.pickle,
data/processed/{train,test}_label.csv, models/custom/<train_type>/<suffix>, logs/...).  Unlike the
reference (:2) nothing sets CUDA_VISIBLE_DEVICES at import (it would break one-process-per-GPU runs).
"""
import os
import random
import time
from datetime import datetime

import numpy as np
import torch
import torch.nn.functional as F
from sklearn.metrics import f1_score
from torch.optim import Adam

try:                                                   # package import (tests) or script-style (reference)
    from .dataset import MultiModalDataset_ii, MultiModalDataset_it, MultiModalDataset_ti, MultiModalDataset_tt
    from .models import (IICA_LapDropout, ITCA_LapDropout, TICA_DPSGD, TICA_LapDropout, TICA_NonPrivate,
                         TISC_LapDropout, TISC_LapDropoutEquWeight, TTCA_LapDropout)
except ImportError:
    from dataset import MultiModalDataset_ii, MultiModalDataset_it, MultiModalDataset_ti, MultiModalDataset_tt
    from models import (IICA_LapDropout, ITCA_LapDropout, TICA_DPSGD, TICA_LapDropout, TICA_NonPrivate,
                        TISC_LapDropout, TISC_LapDropoutEquWeight, TTCA_LapDropout)


def set_seed(seed):
    """base_train.py:23-38"""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)


set_seed(980616)

_DATASETS = {"ti": MultiModalDataset_ti, "tt": MultiModalDataset_tt, "it": MultiModalDataset_it,
             "ii": MultiModalDataset_ii}
# (eeg side, act side) feature kinds per pairing
_KINDS = {"ti": ("txt", "img"), "tt": ("txt", "txt"), "it": ("img", "txt"), "ii": ("img", "img")}
# inputs the reference casts to float32 before the forward (:186-195): the image sides
_FLOAT = {"ti": (False, True), "it": (True, False), "ii": (True, True), "tt": (False, False)}


def _model(cross_atn_type, multimodal_type, dp_mode, coef):
    """base_train.py:131-154"""
    table = {("double_stream", "ti", "lapacian_dropout"): lambda: TICA_LapDropout(bert_coef=coef),
             ("double_stream", "ti", "DPSGD"): lambda: TICA_DPSGD(bert_coef=coef),
             ("double_stream", "ti", "NDP"): lambda: TICA_NonPrivate(bert_coef=coef),
             ("double_stream", "ti", "lapacian_dropout_equal_weight"):
                 lambda: TISC_LapDropoutEquWeight(bert_coef=coef, dropout_rate=0.5),
             ("double_stream", "tt", "lapacian_dropout"): lambda: TTCA_LapDropout(bert_coef=coef),
             ("double_stream", "it", "lapacian_dropout"): lambda: ITCA_LapDropout(bert_coef=coef),
             ("double_stream", "ii", "lapacian_dropout"): lambda: IICA_LapDropout(),
             ("single_stream", "ti", "lapacian_dropout"): lambda: TISC_LapDropout(bert_coef=coef)}
    key = (cross_atn_type, multimodal_type, dp_mode)
    if key not in table:
        raise ValueError(f"TrainAndTest: no model for {key} (the reference leaves `model` unbound here)")
    return table[key]()


class TrainAndTest(object):
    def __init__(self, batch_size=8, learning_rate=1e-6, epochs=50):
        self.batch_size = batch_size
        self.learning_rate = learning_rate
        self.epochs = epochs
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        set_seed(980616)

    def cal_loss(self, prediction, label):
        """base_train.py:58-64"""
        label = label.squeeze(dim=1)
        loss = F.cross_entropy(prediction, label)
        with torch.no_grad():
            pred_label_id = torch.argmax(prediction, dim=1)
            accuracy = (label == pred_label_id).float().sum() / label.shape[0]
        return loss, accuracy, pred_label_id, label

    def _loaders(self, multimodal_type, eeg_model, eeg_coef, act_model, act_coef):
        std = lambda c: c.replace("/", "_").replace("-", "_")      # noqa: E731
        ek, ak = _KINDS[multimodal_type]
        eeg_dir = f"data/embedding/EEG/{ek}/{eeg_model}_{std(eeg_coef)}/"
        act_dir = f"data/embedding/act/{ak}/{act_model}_{std(act_coef)}/"
        ds = _DATASETS[multimodal_type]
        out = []
        for split in ("train", "test"):
            d = ds(eeg_dir + f"{split}.pickle", act_dir + f"{split}.pickle", f"data/processed/{split}_label.csv")
            out.append(torch.utils.data.DataLoader(d, batch_size=self.batch_size, shuffle=True))
        return out

    def _inputs(self, batch, multimodal_type):
        e, em, a, am, y = (t.to(self.device) for t in batch)
        fe, fa = _FLOAT.get(multimodal_type, (False, False))
        return (e.to(torch.float32) if fe else e), em, (a.to(torch.float32) if fa else a), am, y

    def _evaluate(self, model, loader, fwd, multimodal_type):
        model.eval()
        preds, labels, loss_sum, acc_sum, n = [], [], 0.0, 0.0, 0
        with torch.no_grad():
            for batch in loader:
                n += 1
                e, em, a, am, y = self._inputs(batch, multimodal_type)
                loss, acc, p, lab = self.cal_loss(fwd(e, em, a, am, True), y)
                preds.extend(p.cpu().numpy())
                labels.extend(lab.cpu().numpy())
                loss_sum += loss.item()
                acc_sum += acc.item()
        return preds, labels, loss_sum, acc_sum, n

    def train(self, train_type, path_suffix, multimodal_type, dp_mode, eeg_model, eeg_model_coef, act_model,
              act_model_coef, cross_atn_type, epsilon):
        """multimodal_type = "ti","tt","it","ii"; dp_mode: "lapacian_dropout" | "NDP" (base_train.py:66-553)"""
        set_seed(980616)
        train_dataloader, test_dataloader = self._loaders(multimodal_type, eeg_model, eeg_model_coef, act_model,
                                                          act_model_coef)
        model = _model(cross_atn_type, multimodal_type, dp_mode, eeg_model_coef)
        model_path = "models/custom/" + train_type + "/" + path_suffix
        log_path = "logs/" + train_type + "/" + path_suffix
        for path in (model_path, log_path):
            os.makedirs(path, exist_ok=True)
        save_model_path, whole_log_path = model_path + "best_f1.pickle", log_path + "whole_record.txt"
        best_log_path = log_path + "best_record.txt"
        f1_score_best = 0.5
        device = self.device

        if dp_mode == "lapacian_dropout":
            DP_params = [p for n, p in model.named_parameters() if 'DP' in n]
            model_params = [p for n, p in model.named_parameters() if 'DP' not in n]
            model_optimizer = Adam(model_params, lr=self.learning_rate)
            DP_optimizer = Adam(DP_params, lr=self.learning_rate)
            fwd = lambda e, em, a, am, hard: model(e, em, a, am, epsilon, hard=hard)      # noqa: E731

            def step(e, em, a, am, y):
                DP_optimizer.zero_grad()
                loss, _, _, _ = self.cal_loss(fwd(e, em, a, am, False), y)
                loss.backward()
                DP_optimizer.step()
                model_optimizer.zero_grad()
                loss, accuracy, _, _ = self.cal_loss(fwd(e, em, a, am, True), y)
                loss.backward()
                model_optimizer.step()
                return loss, accuracy
        elif dp_mode == "NDP":
            optimizer = Adam(model.parameters(), lr=self.learning_rate)
            fwd = lambda e, em, a, am, hard: model(e, em, a, am)                           # noqa: E731

            def step(e, em, a, am, y):
                optimizer.zero_grad()
                loss, accuracy, _, _ = self.cal_loss(fwd(e, em, a, am, True), y)
                loss.backward()
                optimizer.step()
                return loss, accuracy
        else:
            raise ValueError(f"TrainAndTest: dp_mode {dp_mode!r}")
        model = model.to(device)

        for epoch in range(self.epochs):
            start_time = time.time()
            loss_tr = acc_tr = 0.0
            n_tr = 0
            model.train()
            for batch in train_dataloader:
                n_tr += 1
                model.train()
                loss, accuracy = step(*self._inputs(batch, multimodal_type))
                loss_tr += loss.item()
                acc_tr += accuracy.item()
            preds, labels, loss_te, acc_te, n_te = self._evaluate(model, test_dataloader, fwd, multimodal_type)
            f1_score_epoch = f1_score(preds, labels)
            time_cost = time.time() - start_time
            formatted_datetime = datetime.now().strftime("%Y-%m-%d %H:%M:%S")
            record = (f"Epochs: {epoch + 1}\n                | Train Loss: {loss_tr / n_tr: .3f}\n"
                      f"                | Train Accuracy: {acc_tr / n_tr: .3f}\n"
                      f"                | Test Loss: {loss_te / n_te: .3f}\n"
                      f"                | Test Accuracy: {acc_te / n_te: .3f}\n"
                      f"                | f_1 Score: {f1_score_epoch: .3f}\n"
                      f"                | Time Cost: {time_cost: .1f}\n"
                      f"                | Record Time: {formatted_datetime} \n")
            print(record)
            with open(whole_log_path, "a") as file:
                file.write(record)
            if f1_score_epoch > f1_score_best:
                torch.save(model.state_dict(), save_model_path)
                f1_score_best = f1_score_epoch
                with open(best_log_path, "w") as file:
                    file.write(record)
        return model
