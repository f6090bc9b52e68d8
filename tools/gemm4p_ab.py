"""A/B of the persistent bf16 GEMM (eegf_tune key 11 = 1, the default) against the non-persistent routing (key 0) on the bench
shapes, interleaved rounds in one process; also checks that both produce the same output bits.
Usage: python tools/gemm4p_ab.py [shape ...]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
import torch  # noqa: E402

from eegfusion import _lib  # noqa: E402
from eegfusion import kernels as K  # noqa: E402

R = 256 * 256
SHAPES = [("qkv_fwd", R, 2304, 768, "fwd", "bias"), ("ao_fwd", R, 768, 768, "fwd", "bias"),
          ("ffn1_fwd_p1", R, 3072, 768, "fwd", "bias_gelu"), ("ffn1_fwd_gelu_d", R, 3072, 768, "fwd", "bias_gelu_d"),
          ("ffn2_fwd", R, 768, 3072, "fwd", "bias"), ("ffn2_dgrad_mulaux", R, 3072, 768, "dgrad", "mul_aux"),
          ("ffn1_dgrad", R, 768, 3072, "dgrad", "none"), ("qkv_dgrad", R, 768, 2304, "dgrad", "none"),
          ("ao_dgrad", R, 768, 768, "dgrad", "none")]


def main():
    lib = _lib.lib()
    lib.eegf_tune.argtypes = [_lib.i32, _lib.i32]
    only = sys.argv[1:]
    dev, dt = "cuda", torch.bfloat16
    for name, M, N, Kd, layout, epi in SHAPES:
        if only and name not in only:
            continue
        torch.manual_seed(0)
        A = torch.randn(M, Kd, device=dev, dtype=dt)
        if layout == "fwd":
            B = torch.randn(N, Kd, device=dev, dtype=dt) * 0.05
            bias = torch.randn(N, device=dev)
            aux = torch.empty(M, N, device=dev, dtype=dt) if epi == "bias_gelu_d" else None
            kw = dict(a_kc=1, b_kc=1, lda=Kd, ldb=Kd, ldc=N, epi=epi, bias=bias, aux=aux, ldaux=N)
        else:
            B = torch.randn(Kd, N, device=dev, dtype=dt) * 0.05
            aux = torch.randn(M, N, device=dev, dtype=dt) if epi != "none" else None
            kw = dict(a_kc=1, b_kc=0, lda=Kd, ldb=N, ldc=N, epi=epi, aux=aux, ldaux=N)
        C = torch.empty(M, N, device=dev, dtype=dt)
        f = lambda: K.gemm(A, B, C, M=M, N=N, K=Kd, **kw)   # noqa: E731
        outs = {}
        for v in (0, 1):
            lib.eegf_tune(11, v)
            C.zero_()
            if aux is not None and epi == "bias_gelu_d":
                aux.zero_()
            f()
            torch.cuda.synchronize()
            outs[v] = (C.clone(), aux.clone() if (aux is not None and epi == "bias_gelu_d") else None)
        same = torch.equal(outs[0][0], outs[1][0]) and (outs[0][1] is None or torch.equal(outs[0][1], outs[1][1]))
        diff = (outs[0][0].float() - outs[1][0].float()).abs().max().item()
        times = {0: [], 1: []}
        for _ in range(5):
            for v in (0, 1):
                lib.eegf_tune(11, v)
                f()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    f()
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / 10)
        med = {v: sorted(t)[2] for v, t in times.items()}
        fl = 2.0 * M * N * Kd
        print(f"{name:18s} {M}x{N}x{Kd} key0 {med[0]*1e3:7.1f} us ({fl/med[0]/1e9:6.1f} TF) | persistent "
              f"{med[1]*1e3:7.1f} us ({fl/med[1]/1e9:6.1f} TF) | identical {same} maxdiff {diff:.3g}", flush=True)
    lib.eegf_tune(11, 1)


if __name__ == "__main__":
    main()
