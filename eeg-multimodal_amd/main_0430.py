"""Drop-in for the reference's main_0430.py (PriConcat): DP_guarantee, ConcatModel(args, dp_mode),
cal_loss.  The opacus DP-SGD pretrain of `train(pretrain=True)` is out of scope (opacus absent;
SURVEY §8(f) rank 3)."""
import math

import torch

from eegfusion import _lib
from eegfusion.modules import PriConcatModel
from past_acc import cal_loss  # noqa: F401  (same function, main_0430.py:68-74)


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
    _lib.call("eegf_fusion_fwd", _lib.F32, B, _lib.FUSE_PRICONCAT_LAP, f.data_ptr(), D, f[:, 768:].data_ptr(), D,
              f[:, 1536:].data_ptr(), D, None, None, None, None if row_noise is None else row_noise.data_ptr(), 0, 0,
              math.exp(EPSILON), 1.0 / EPSILON, seed, offset, out.data_ptr(), xn.data_ptr(), amin.data_ptr(),
              amax.data_ptr(), rg.data_ptr(), torch.cuda.current_stream().cuda_stream)
    return out


class ConcatModel(PriConcatModel):
    """main_0430.py:88-123"""

    def __init__(self, args, dp_mode=None):
        super().__init__(args, dp_mode=dp_mode, contract="T")


def train(*a, pretrain=False, **k):
    if pretrain:
        raise NotImplementedError("opacus DP-SGD pretraining (main_0430.py:143-162) is out of scope for this build")
    raise NotImplementedError("use past_acc.main2-style loops or eegfusion.trainer.SinglePassTrainer")
