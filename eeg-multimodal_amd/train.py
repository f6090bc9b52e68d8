"""Drop-in for the reference's train.py (train.py:1-151): ConcatModel (model.py) trained with one
Adam over the non-DP parameters, CrossEntropyLoss(reduction='none').sum(), n_para repeats per
batch, evaluation every `interval` epochs with n_eval repeated forwards, metrics, best-accuracy
checkpoint (model.pth) and the per-epoch results file (results.pth).

Differences, all forced by the image: torchmetrics is absent, so the metrics come from
eegfusion.metrics (on-device restatements of its multiclass defaults); results.pth is read back
with torch.load(weights_only=True).  `.cuda()` becomes `.to(DEVICE)`: the MI355X engine when a GPU is
present, else the host path (configs[0], "CPU PyTorch via train.py").
The reference's quirks are kept: labels are collected in a separate shuffled pass over the
validation loader (train.py:83-86) and evaluation re-shuffles (train.py:122-136).
"""
import argparse
import logging
import os
import sys
from collections import defaultdict

import numpy as np
import torch
import torch.nn as nn
from torch.optim import Adam

from data import get_data
from eegfusion.metrics import METRICS
from model import get_model


def set_seed(seed):
    """train.py:15-22"""
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)


def parse_args(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--exp", type=str, default='test')
    parser.add_argument("--name", type=str, default='test')
    parser.add_argument("--batch_size", "-bs", type=int, default=8)
    parser.add_argument("--data_name", "-d", type=str, default="EEG")
    parser.add_argument("--eps", "-e", type=float, default=2.0)
    parser.add_argument("--n_class", "-c", type=int, default=2)
    parser.add_argument("--n_dp", "-nd", type=int, default=1)
    parser.add_argument("--n_para", "-np", type=int, default=1)
    parser.add_argument("--n_eval", "-ne", type=int, default=5)
    parser.add_argument("--n_epochs", "-n", type=int, default=50)
    parser.add_argument("--interval", type=int, default=1)
    parser.add_argument("--metrics", "-m", type=str, default='Accuracy')
    return parser.parse_args(argv)


DEVICE = torch.device("cuda" if torch.cuda.is_available() else "cpu")   # the reference's .cuda(); host
# memory where no GPU exists (configs[0]'s plumbing run: model.get_model keeps the model there too)


def _to_cuda(inputs):
    return list(i.to(DEVICE) for i in inputs) if isinstance(inputs, (list, tuple)) else inputs.to(DEVICE)


def main(cfg):
    """train.py:46-151"""
    base_path = f'experiment/{cfg.exp}/{cfg.name}/'
    os.makedirs(base_path, exist_ok=True)
    logging.basicConfig(level=logging.DEBUG, format='%(asctime)s - %(levelname)s - %(message)s',
                        handlers=[logging.FileHandler(base_path + 'debug.log', 'w'),
                                  logging.FileHandler(base_path + 'info.log', 'w'),
                                  logging.StreamHandler(sys.stdout)], force=True)
    logger = logging.getLogger()
    logger.handlers[1].setLevel(logging.INFO)
    logger.info(cfg)

    train_loader, val_loader = get_data(cfg)
    model = get_model(cfg)
    criterion = nn.CrossEntropyLoss(reduction='none')
    model_params = [p for n, p in model.named_parameters() if 'DP' not in n]
    model_optimizer = Adam(model_params, lr=1e-6)
    results = defaultdict(list)
    unknown = [m for m in cfg.metrics.split(',') if m not in METRICS]
    if unknown:
        raise ValueError(f"unsupported metrics {unknown}; available: {sorted(METRICS)}")
    metrics = {i: METRICS[i](task="multiclass", num_classes=cfg.n_class).to(DEVICE) for i in cfg.metrics.split(',')}
    best_acc = 0.0

    for inputs, labels in val_loader:
        results['labels'].append(labels.to(DEVICE).view(-1))
    results['labels'] = torch.cat(results['labels'])

    for epoch in range(cfg.n_epochs):
        model.train()
        for i, (inputs, labels) in enumerate(train_loader):
            inputs = _to_cuda(inputs)
            labels = labels.view(-1).to(DEVICE)
            model_optimizer.zero_grad()
            for _ in range(cfg.n_para):
                loss = criterion(model(inputs, hard=True), labels)
                loss.sum().backward()
                results['train_loss'].append(loss.detach())
            model_optimizer.step()
            logger.debug(f'Train Epoch: {epoch:3d} [{i + 1:3d}/{len(train_loader):3d}]'
                         f" loss {torch.cat(results['train_loss'][-cfg.n_para:]).mean().item():.4f}")

        if (epoch + 1) % cfg.interval == 0:
            model.eval()
            eval_metrics = defaultdict(list)
            with torch.no_grad():
                for inputs, labels in val_loader:
                    inputs = _to_cuda(inputs)
                    labels = labels.view(-1).to(DEVICE)
                    for _ in range(cfg.n_eval):
                        logits = model(inputs, hard=True)
                        eval_metrics['logits'].append(logits)
                        eval_metrics['pred'].append(logits.max(1)[1])
                        eval_metrics['val_loss'].append(criterion(logits, labels))
            info = f'Eval  Epoch: {epoch:3d}'
            for k, v in eval_metrics.items():
                results[k].append(torch.cat(v).view(-1, cfg.n_eval, *v[-1].shape[1:]))
            for m, func in metrics.items():
                vl = [func(results['pred'][-1][:, i], results['labels']) for i in range(cfg.n_eval)]
                results[m].append(v := torch.stack(vl).cpu())
                info += f' | {m}: {v.mean().item():5.2f}'
            results['DP_params'].append(model.DP.data.clone() if hasattr(model, "DP") else torch.zeros(0))
            logger.info(info)
            acc_key = 'Accuracy' if 'Accuracy' in results else next(iter(metrics))
            if (acc := results[acc_key][-1].mean()) > best_acc:
                best_acc = acc
                torch.save(model.state_dict(), os.path.join(base_path, 'model.pth'))
        torch.save({k: torch.cat([t.cpu() for t in v]) for k, v in results.items() if k not in ('labels', 'inputs')},
                   os.path.join(base_path, 'results.pth'))
        res = torch.load(os.path.join(base_path, 'results.pth'), weights_only=True)
        for k, v in res.items():
            print(k, ':', tuple(v.shape))
    return results


if __name__ == '__main__':
    set_seed(980616)
    main(parse_args())
