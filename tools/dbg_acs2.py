"""Debug: GEMM with A nonzero only in one K-tile (K-tile kt of 32 columns), 4-wave and default."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "eeg-multimodal_amd"))
import torch
from eegfusion import _lib, kernels as kk
lib = _lib.lib()
lib.eegf_tune.argtypes = [_lib.i32, _lib.i32]
M, N, K = 4096, 768, 2304
for key1 in (-1, 6):
    lib.eegf_tune(1, key1)
    for kt in (0, 1, 5):
        torch.manual_seed(13)
        dy = torch.zeros(M, K, device="cuda")
        dy[:, kt * 32:(kt + 1) * 32] = torch.randn(M, 32, device="cuda")
        dy = dy.to(torch.bfloat16)
        w = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
        c = kk.linear_dgrad(dy, w)
        torch.cuda.synchronize()
        ref = dy.double() @ w.double()
        e = (c.double() - ref).abs()
        print("key1", key1, "kt", kt, "max err", e.max().item(), "of", ref.abs().max().item(), "nan", torch.isnan(c).sum().item())
lib.eegf_tune(1, -1)
