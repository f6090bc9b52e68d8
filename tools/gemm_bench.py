"""Time eegf_gemm on every GEMM shape of the B=256 PriGumbel step (and torch.matmul on the same
shapes as a calibration point for what the chip sustains).  Usage: python tools/gemm_bench.py"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
import torch  # noqa: E402

from eegfusion import kernels as K  # noqa: E402

R = 256 * 256
# (name, M, N, K, layout, epi)
SHAPES = [
    ("qkv_fwd", R, 2304, 768, "fwd", "bias"),
    ("ao_fwd", R, 768, 768, "fwd", "bias"),
    ("ffn1_fwd", R, 3072, 768, "fwd", "bias_gelu"),
    ("ffn1_fwd_nogelu", R, 3072, 768, "fwd", "bias"),
    ("ffn1_fwd_gelu_d", R, 3072, 768, "fwd", "bias_gelu_d"),
    ("ffn2_dgrad_mulaux", R, 3072, 768, "dgrad", "mul_aux"),
    ("ffn2_fwd", R, 768, 3072, "fwd", "bias"),
    ("ffn2_dgrad_dgelu", R, 3072, 768, "dgrad", "dgelu"),
    ("ffn2_dgrad_plain", R, 3072, 768, "dgrad", "none"),
    ("ffn1_dgrad", R, 768, 3072, "dgrad", "none"),
    ("qkv_dgrad", R, 768, 2304, "dgrad", "none"),
    ("ao_dgrad", R, 768, 768, "dgrad", "none"),
    # the step's BERT input gradients accumulate into the residual gradient (beta = 1)
    ("ffn1_dgrad_acc", R, 768, 3072, "dgrad", "none+acc"),
    ("qkv_dgrad_acc", R, 768, 2304, "dgrad", "none+acc"),
    ("ao_dgrad_acc", R, 768, 768, "dgrad", "none+acc"),
    ("qkv_wgrad", 2304, 768, R, "wgrad", "none"),
    ("ffn1_wgrad", 3072, 768, R, "wgrad", "none"),
    ("ffn2_wgrad", 768, 3072, R, "wgrad", "none"),
    ("ao_wgrad", 768, 768, R, "wgrad", "none"),
    ("wide_fwd_k3072", R, 3072, 3072, "fwd", "none"),
    ("sq4k", 4096, 4096, 4096, "fwd", "none"),       # the guide's 8-phase template reference shape
    ("sq8k", 8192, 8192, 8192, "fwd", "none"),
]


def run(name, M, N, Kd, layout, epi, iters=20):
    dt = torch.bfloat16
    dev = "cuda"
    ws = torch.empty(24 << 20, device=dev)
    if layout == "fwd":
        A = torch.randn(M, Kd, device=dev, dtype=dt)
        B = torch.randn(N, Kd, device=dev, dtype=dt) * 0.05
        C = torch.empty(M, N, device=dev, dtype=dt)
        bias = torch.randn(N, device=dev)
        aux = torch.empty(M, N, device=dev, dtype=dt) if epi in ("bias_gelu", "bias_gelu_d") else None
        f = lambda: K.gemm(A, B, C, M=M, N=N, K=Kd, a_kc=1, b_kc=1, lda=Kd, ldb=Kd, ldc=N, epi=epi, bias=bias,
                           aux=aux, ldaux=N)
        bb = bias.to(dt)
        tf = lambda: torch.nn.functional.linear(A, B, bb)
    elif layout == "dgrad":
        beta = 1.0 if epi.endswith("+acc") else 0.0
        epi = epi.split("+")[0]
        A = torch.randn(M, Kd, device=dev, dtype=dt)
        B = torch.randn(Kd, N, device=dev, dtype=dt) * 0.05
        C = torch.randn(M, N, device=dev, dtype=dt) * 0.01
        aux = torch.randn(M, N, device=dev, dtype=dt) if epi != "none" else None
        f = lambda: K.gemm(A, B, C, M=M, N=N, K=Kd, a_kc=1, b_kc=0, lda=Kd, ldb=N, ldc=N, epi=epi, aux=aux, ldaux=N,
                           beta=beta)
        tf = lambda: A @ B
    else:
        A = torch.randn(Kd, M, device=dev, dtype=dt)
        B = torch.randn(Kd, N, device=dev, dtype=dt)
        C = torch.zeros(M, N, device=dev, dtype=torch.float32)
        f = lambda: K.gemm(A, B, C, M=M, N=N, K=Kd, a_kc=0, b_kc=0, lda=M, ldb=N, ldc=N, beta=1.0, workspace=ws)
        tf = lambda: A.t() @ B
    from eegfusion import _lib
    lib = _lib.lib()
    lib.eegf_tune.argtypes = [_lib.i32, _lib.i32]

    def timed(fn, n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / n

    def tf_(ms):
        return 2.0 * M * N * Kd / ms / 1e9

    if AB:   # interleaved rounds of the two schedules in one process (key 1: 8-phase forward)
        for fn in (f, tf):
            fn()
        torch.cuda.synchronize()
        r = {v: [] for v in VARIANTS}
        for _ in range(5):
            for v in VARIANTS:
                if KEY is not None:       # --key=K: the variants are values of eegf_tune key K
                    lib.eegf_tune(KEY, v)
                    f()
                    torch.cuda.synchronize()
                    r[v].append(timed(f, iters))
                    continue
                # -1: default routing; 0: 2-phase 8-wave; 4: 8-phase 8-wave; 8: 4-wave (key 1 = 6);
                # 9: default routing with the 256x128 two-workgroup kernel for every short-K GEMM (key 8)
                # 20 + G: default routing with the grouped tile raster of G row panels (key 9)
                lib.eegf_tune(1, -1 if v in (-1, 9) or v >= 20 else {8: 6}.get(v, v))
                lib.eegf_tune(8, 1 if v == 9 else 2 if (v == -1 or v >= 20) else 0)
                lib.eegf_tune(9, v - 20 if 20 <= v < 40 else -1 if v == -1 else 0)
                f()
                torch.cuda.synchronize()
                r[v].append(timed(f, iters))
        if KEY is not None:
            lib.eegf_tune(KEY, VARIANTS[0])
        else:
            lib.eegf_tune(1, -1)
            lib.eegf_tune(8, 2)
            lib.eegf_tune(9, -1)
        med = {v: sorted(x)[len(x) // 2] for v, x in r.items()}
        tt = timed(tf, iters)
        print(f"{name:16s} {M}x{N}x{Kd} " + " | ".join(f"v{v} {tf_(med[v]):6.1f} ({med[v] * 1e3:5.1f} us)" for v in med)
              + f" | torch {tf_(tt):6.1f} TF", flush=True)
        return
    res = []
    for fn in (f, tf):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ms = timed(fn, iters)
        res.append((ms, tf_(ms)))
    print(f"{name:20s} M={M:6d} N={N:5d} K={Kd:6d}  eegf {res[0][0]*1e3:8.1f} us {res[0][1]:7.1f} TF | "
          f"torch {res[1][0]*1e3:8.1f} us {res[1][1]:7.1f} TF", flush=True)


AB = "--ab" in sys.argv
KEY = next((int(a.split("=")[1]) for a in sys.argv if a.startswith("--key=")), None)
VARIANTS = [int(x) for x in next((a.split("=")[1] for a in sys.argv if a.startswith("--variants=")), "-1,0,4,8").split(",")]


if __name__ == "__main__":
    only = [a for a in sys.argv[1:] if not a.startswith("--")]
    for s in SHAPES:
        if not only or s[0] in only:
            run(*s)
