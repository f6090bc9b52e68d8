"""Weight-gradient GEMMs of the bench step with and without the fused bias gradient (row sums of dY
on the VALU in the workgroups of tile column 0, eegf_gemm_wgrad_bias) against the plain split-K weight
gradient (eegf_gemm): what the row sums cost.  usage: python tools/wgrad_probe.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
import torch  # noqa: E402

from eegfusion import _lib  # noqa: E402
from eegfusion import kernels as K  # noqa: E402

R = 256 * 256
SHAPES = [("qkv_wgrad", 2304, 768), ("ao_wgrad", 768, 768), ("ffn1_wgrad", 3072, 768), ("ffn2_wgrad", 768, 3072)]


def timed(fn, n=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    lib = _lib.lib()
    dev, dt = "cuda", torch.bfloat16
    ws = torch.empty(64 << 20, device=dev)
    P = lambda t: t.data_ptr()
    for name, M, N in SHAPES:        # dW [M][N] = dY^T X over R tokens; dY [R][M], X [R][N]
        dy = torch.randn(R, M, device=dev, dtype=dt)
        x = torch.randn(R, N, device=dev, dtype=dt)
        dw = torch.zeros(M, N, device=dev)
        db = torch.zeros(M, device=dev)
        fb = lambda: lib.eegf_gemm_wgrad_bias(_lib.BF16, M, N, R, P(dy), M, P(x), N,
                                              P(dw), N, 1.0, P(db), P(ws), ws.numel() * 4, 0)
        fp = lambda: K.gemm(dy, x, dw, M=M, N=N, K=R, a_kc=0, b_kc=0, lda=M, ldb=N, ldc=N, beta=1.0, workspace=ws)
        r = {"bias": [], "plain": []}
        for _ in range(5):
            r["bias"].append(timed(fb))
            r["plain"].append(timed(fp))
        med = {k: sorted(v)[2] for k, v in r.items()}
        print(f"{name:12s} {M}x{N}x{R}  with bias grad {med['bias']:7.1f} us   plain {med['plain']:7.1f} us   "
              f"({2.0 * M * N * R / med['bias'] / 1e6:6.1f} / {2.0 * M * N * R / med['plain'] / 1e6:6.1f} TF)", flush=True)


if __name__ == "__main__":
    main()
