"""A/B of eegf_ln_fwd rows-per-wave (eegf_tune key 6) at the BERT shape: 65536 x 768 bf16, residual,
attention-output dropout (mode 1, p 0.1), residual-sum store (pass 2) and without it (pass 1).
Prints us per call and the algorithmic GB/s; checks every variant's output equals rpw=1's."""
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "eeg-multimodal_amd"), str(ROOT)]
from eegfusion import _lib  # noqa: E402
from eegfusion._lib import BF16, call  # noqa: E402

R, W = 65536, 768
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(R, W, device=dev, generator=g).bfloat16()
r = torch.randn(R, W, device=dev, generator=g).bfloat16()
gam = torch.randn(W, device=dev, generator=g)
bet = torch.randn(W, device=dev, generator=g)
y = torch.empty(R, W, device=dev, dtype=torch.bfloat16)
s = torch.empty_like(y)
mean = torch.empty(R, device=dev)
rstd = torch.empty(R, device=dev)
st = torch.cuda.current_stream()
P = float(os.environ.get("LNB_P", "0.1"))   # dropout probability of the forward (LNB_P=0: no RNG)


def run(save):
    call("eegf_ln_fwd", BF16, R, W, x.data_ptr(), r.data_ptr(), None, 1, None, gam.data_ptr(), bet.data_ptr(),
         1e-12, P, 1, 7, 11, y.data_ptr(), s.data_ptr() if save else None, mean.data_ptr(), rstd.data_ptr(),
         st.cuda_stream)


ref = {}
for rpw in (1, 4, 16, 32):
    _lib.lib().eegf_tune(6, rpw)
    for save in (False, True):
        for _ in range(3):
            run(save)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        n = 50
        for _ in range(n):
            run(save)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / n
        nbytes = R * W * 2 * (3 + save) + R * 8
        out = (y.clone(), s.clone() if save else None, mean.clone())
        if (rpw == 1):
            ref[save] = out
        same = torch.equal(out[0], ref[save][0]) and torch.equal(out[2], ref[save][2]) and (
            not save or torch.equal(out[1], ref[save][1]))
        print(f"rpw {rpw:2d} save {int(save)}: {us:7.1f} us  {nbytes / us / 1e3:6.0f} GB/s  same={same}", flush=True)
_lib.lib().eegf_tune(6, 16)

# backward: rows per workgroup (eegf_tune key 7); partial buffers sized by eegf_ln_bwd_partial_rows
dy = torch.randn(R, W, device=dev, generator=g).bfloat16()
dx = torch.empty_like(y)
dr = torch.empty_like(y)
run(True)
refb = None
for rpb in (64, 128, 256, 32):
    _lib.lib().eegf_tune(7, rpb)
    nb = -(-R // _lib.lib().eegf_ln_bwd_partial_rows(R))
    part = torch.empty(2, nb, W, device=dev)

    def runb():
        call("eegf_ln_bwd", BF16, R, W, dy.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
             gam.data_ptr(), 0.1, 1, 7, 11, dx.data_ptr(), dr.data_ptr(), part[0].data_ptr(), part[1].data_ptr(),
             st.cuda_stream)
    for _ in range(3):
        runb()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        runb()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 50
    dg = part[0].double().sum(0)
    out = (dx.clone(), dr.clone(), dg)
    refb = refb or out
    same = torch.equal(out[0], refb[0]) and torch.equal(out[1], refb[1]) and float((dg - refb[2]).abs().max()) < 1e-3
    print(f"bwd rpb {rpb:3d}: {us:7.1f} us  {R * W * 2 * 4 / us / 1e3:6.0f} GB/s  same={same}", flush=True)
_lib.lib().eegf_tune(7, 64)
