"""Drop-in for the reference's main_0430.py (PriConcat): DP_guarantee, ConcatModel(args, dp_mode),
cal_loss, MultiModalDataset_ti and the two-stage `train` / `main` (main_0430.py:129-235):

  * pretrain=True: only bert.encoder.layer[-1], fc_layers and classifier train, with DP-SGD through
    eegfusion.dpsgd.PrivacyEngine.make_private_with_epsilon (opacus semantics: Poisson sampling,
    per-sample clipping to MAX_GRAD_NORM, Gaussian noise, RDP accounting; delta = 1 / len(loader));
  * pretrain=False: plain Adam fine-tuning, optionally starting from the pretrain checkpoint with
    load_state_dict(strict=False) (main_0430.py:137-139);
  * each epoch: train loop, an evaluation pass in train mode (the reference never calls
    model.eval()), sklearn F1, the record appended to whole_record.txt, the state_dict saved to
    best_f1.pickle on a new best F1 (> 0.5 initially).
Everything but the metrics' host reduction runs on the engine (libeegfusion.so)."""
import os

import torch


from eegfusion import _lib
from eegfusion.modules import PriConcatModel
from past_acc import MultiModalDataset_ti, cal_loss  # noqa: F401  (main_0430.py:39-74: the same 5-tuple dataset and loss)


def DP_guarantee(feature, EPSILON, dp_mode=None, row_noise=None, seed=0, offset=0):
    """main_0430.py:76-85 on device: identity for dp_mode=None, else min-max + one Laplace(0, 1/EPSILON)
    draw per row (Philox, or `row_noise` [B] injected)."""
    if dp_mode != 'feature_all_lap':
        return feature
    f = feature.contiguous().float()
    if not f.is_cuda:
        raise RuntimeError("eegfusion: DP_guarantee runs on the GPU only")
    B, D = f.shape
    out = torch.empty_like(f)
    xn = torch.empty_like(f)
    amin = torch.empty(B, dtype=torch.int32, device=f.device)
    amax = torch.empty_like(amin)
    rg = torch.empty(B, device=f.device)
    import math
    _lib.call("eegf_fusion_fwd", _lib.F32, B, _lib.FUSE_PRICONCAT_LAP, f.data_ptr(), D, f[:, 768:].data_ptr(), D,
              f[:, 1536:].data_ptr(), D, None, None, None, None if row_noise is None else row_noise.data_ptr(), 0, 0,
              math.exp(EPSILON), 1.0 / EPSILON, seed, offset, out.data_ptr(), xn.data_ptr(), amin.data_ptr(),
              amax.data_ptr(), rg.data_ptr(), torch.cuda.current_stream().cuda_stream)
    return out


class ConcatModel(PriConcatModel):
    """main_0430.py:88-123"""

    def __init__(self, args, dp_mode=None, **kw):
        super().__init__(args, dp_mode=dp_mode, contract=kw.pop("contract", "T"), **kw)


def mkpath(path):
    """main_0430.py:125-126"""
    return path + '/whole_record.txt', path + '/best_record.txt', path + '/best_f1.pickle'


def train(args, train_dataset, val_dataset, model, pretrain=False, load_stat=False, privacy_engine=None):
    """main_0430.py:129-225.  Returns (model, best F1)."""
    from sklearn.metrics import f1_score

    from eegfusion.dpsgd import PrivacyEngine
    from eegfusion.optim import Adam
    train_dataloader = torch.utils.data.DataLoader(train_dataset, batch_size=args.batch_size, shuffle=True)
    val_dataloader = torch.utils.data.DataLoader(val_dataset, batch_size=args.batch_size, shuffle=True)
    optimizer = Adam(model.parameters(), lr=args.learning_rate)
    if pretrain:
        os.makedirs(args.path + '/pretrain', exist_ok=True)
        whole_record_path, best_record_path, save_model_path = mkpath(args.path + '/pretrain')
    else:
        if load_stat:
            load_model_path = args.path + '/pretrain/best_f1.pickle'
            model.load_state_dict(torch.load(load_model_path, weights_only=True), strict=False)
        os.makedirs(args.path, exist_ok=True)
        whole_record_path, best_record_path, save_model_path = mkpath(args.path)

    if pretrain:
        trainable_layers = [model.bert.encoder.layer[-1], model.fc_layers, model.classifier]
        for p in model.parameters():
            p.requires_grad = False
        for layer in trainable_layers:
            for p in layer.parameters():
                p.requires_grad = True
        DELTA = 1 / len(train_dataloader)
        privacy_engine = privacy_engine or PrivacyEngine()
        model, optimizer, train_dataloader = privacy_engine.make_private_with_epsilon(
            module=model, optimizer=optimizer, data_loader=train_dataloader, target_delta=DELTA,
            target_epsilon=args.EPSILON, epochs=args.epochs, max_grad_norm=args.MAX_GRAD_NORM)

    device = torch.device("cuda")
    model = model.to(device)
    f1_score_best = 0.5
    for epoch in range(args.epochs):
        epoch_acc_train = epoch_loss_train = epoch_acc_val = epoch_loss_val = 0
        sample_size_train = sample_size_val = 0
        model.train()
        for frame_input, vedio_mask, title_input, text_mask, label in train_dataloader:
            sample_size_train += 1
            model.train()
            optimizer.zero_grad()
            frame_input, vedio_mask, title_input, text_mask, label = (
                t.to(device) for t in (frame_input, vedio_mask, title_input, text_mask, label))
            prediction = model(frame_input, vedio_mask, title_input, text_mask)
            loss, accuracy, _, _ = cal_loss(prediction, label)
            epoch_loss_train += loss.item()
            epoch_acc_train += accuracy.item()
            loss.backward()
            optimizer.step()
        prediction_all, label_all = [], []
        with torch.no_grad():
            for frame_input, vedio_mask, title_input, text_mask, label in val_dataloader:
                sample_size_val += 1
                frame_input, vedio_mask, title_input, text_mask, label = (
                    t.to(device) for t in (frame_input, vedio_mask, title_input, text_mask, label))
                prediction = model(frame_input, vedio_mask, title_input, text_mask)
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
    return model, f1_score_best


def main(args, feature_dir='feature'):
    """main_0430.py:227-235: DP-SGD pretrain, then fine-tuning with the feature mechanism."""
    train_dataset = MultiModalDataset_ti(f'{feature_dir}/train_EEG.csv', f'{feature_dir}/action/train_clip_v2.pickle',
                                         f'{feature_dir}/EEG/train_bert.pickle')
    val_dataset = MultiModalDataset_ti(f'{feature_dir}/test_EEG.csv', f'{feature_dir}/action/test_clip_v2.pickle',
                                       f'{feature_dir}/EEG/test_bert.pickle')
    model = ConcatModel(args)
    train(args, train_dataset, val_dataset, model, pretrain=True, load_stat=False)
    model = ConcatModel(args, dp_mode='feature_all_lap')
    train(args, train_dataset, val_dataset, model, pretrain=False, load_stat=True)
