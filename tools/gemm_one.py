"""Run one GEMM shape of tools/gemm_bench.py repeatedly (for rocprofv3 PMC passes).
Usage: python tools/gemm_one.py <shape> <variant|torch> [iters]   (variant as gemm_bench --ab)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
sys.path.insert(0, str(ROOT / "tools"))
import torch  # noqa: E402

import gemm_bench as gb  # noqa: E402
from eegfusion import kernels as K  # noqa: E402
from eegfusion import _lib  # noqa: E402

name, var = sys.argv[1], sys.argv[2]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
shape = next(s for s in gb.SHAPES if s[0] == name)
_, M, N, Kd, layout, epi = shape
dt, dev = torch.bfloat16, "cuda"
A = torch.rand(M, Kd, device=dev).to(dt) * 2 - 1
B = torch.rand(N, Kd, device=dev).to(dt) * 2 - 1
C = torch.empty(M, N, device=dev, dtype=dt)
lib = _lib.lib()
lib.eegf_tune.argtypes = [_lib.i32, _lib.i32]
if var == "torch":
    f = lambda: torch.nn.functional.linear(A, B)
else:
    v = int(var)
    lib.eegf_tune(1, {8: 6}.get(v, v))        # -1 auto, 0 2-phase, 4 8-phase, 8 4-wave
    f = lambda: K.gemm(A, B, C, M=M, N=N, K=Kd, a_kc=1, b_kc=1, lda=Kd, ldb=Kd, ldc=N)
for _ in range(iters):
    f()
torch.cuda.synchronize()
print("ok", name, var)
