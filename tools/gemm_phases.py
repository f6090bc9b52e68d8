"""Per-phase times of the 256x256 GEMM kernels (eegf_gemm_big_timestamps): prologue, K-loop, epilogue
per workgroup, the dispatch gap between consecutive workgroups on one CU slot, and how many
workgroups are in each phase over time.

usage: python tools/gemm_phases.py [shape ...]   (names from tools/gemm_bench.py SHAPES)
       EEGF_GEMM8=6 selects the 4-wave kernel for every shape."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
sys.path.insert(0, str(ROOT / "tools"))
import torch  # noqa: E402

from gemm_bench import SHAPES  # noqa: E402
from eegfusion import _lib, kernels as K  # noqa: E402


def main():
    lib = _lib.lib()
    names = sys.argv[1:] or ["ffn1_fwd_nogelu", "ffn1_fwd", "ffn1_fwd_gelu_d", "ffn2_fwd"]
    for name, M, N, Kd, layout, epi in SHAPES:
        if name not in names:
            continue
        dt, dev = torch.bfloat16, "cuda"
        A = torch.randn(M, Kd, device=dev, dtype=dt)
        if layout == "fwd":
            B = torch.randn(N, Kd, device=dev, dtype=dt) * 0.05
            bkc, ldb = 1, Kd
        else:
            B = torch.randn(Kd, N, device=dev, dtype=dt) * 0.05
            bkc, ldb = 0, N
        C = torch.empty(M, N, device=dev, dtype=dt)
        bias = torch.randn(N, device=dev)
        aux = torch.randn(M, N, device=dev, dtype=dt) if epi not in ("bias", "none") else None
        f = lambda: K.gemm(A, B, C, M=M, N=N, K=Kd, a_kc=1, b_kc=bkc, lda=Kd, ldb=ldb, ldc=N, epi=epi,   # noqa: E731
                           bias=bias if layout == "fwd" else None, aux=aux, ldaux=N)
        tiles = (M // 256) * ((N + 127) // 128)          # enough for the 256x128 kernel's grid
        ts = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        lib.eegf_gemm_big_timestamps(ts.data_ptr())
        f()
        torch.cuda.synchronize()
        lib.eegf_gemm_big_timestamps(None)
        raw = ts.view(tiles, 8).cpu()
        ok = (raw[:, 0] > 0) & (raw[:, 3] > 0)
        raw = raw[ok]
        cu = raw[:, 4].tolist()
        t = raw[:, :4].double() * 0.01      # us
        t0 = t[:, 0].min()
        t = t - t0
        span = float(t[:, 3].max())
        pro, loop, epi_t = (t[:, 1] - t[:, 0]), (t[:, 2] - t[:, 1]), (t[:, 3] - t[:, 2])
        ncu = len(set(cu))
        busy = float((t[:, 3] - t[:, 0]).sum()) / (ncu * span)
        tf = 2.0 * M * N * Kd / ms / 1e9
        print(f"{name:18s} {M}x{N}x{Kd} {ms * 1e3:7.1f} us {tf:6.1f} TF  wgs={int(ok.sum())} span={span:6.1f} us  "
              f"prologue {float(pro.mean()):5.2f}  loop {float(loop.mean()):6.2f} (min {float(loop.min()):6.2f})  "
              f"epilogue {float(epi_t.mean()):5.2f}  us/wg;  occupancy {busy:.3f}", flush=True)
        # phase histogram over time: how many workgroups are in prologue / loop / epilogue per 5 % slice
        sl = []
        for q in range(20):
            x = span * (q + 0.5) / 20
            inp = int(((t[:, 0] <= x) & (x < t[:, 1])).sum())
            inl = int(((t[:, 1] <= x) & (x < t[:, 2])).sum())
            ine = int(((t[:, 2] <= x) & (x < t[:, 3])).sum())
            sl.append(f"{inp}/{inl}/{ine}")
        print("   pro/loop/epi over time: " + " ".join(sl), flush=True)
        # co-residency: per CU, sample the states of its workgroups; with two resident, how often is
        # one in its epilogue while the other runs its K-loop (overlap) vs both in the epilogue
        by = {}
        for r, c in enumerate(cu):
            by.setdefault(c, []).append(r)
        both_epi = ovl = one_epi = 0
        for c, rows in by.items():
            tt = t[rows]
            for q in range(400):
                x = span * (q + 0.5) / 400
                epi_n = int(((tt[:, 2] <= x) & (x < tt[:, 3])).sum())
                loop_n = int(((tt[:, 1] <= x) & (x < tt[:, 2])).sum())
                if epi_n >= 2:
                    both_epi += 1
                elif epi_n == 1 and loop_n >= 1:
                    ovl += 1
                elif epi_n == 1:
                    one_epi += 1
        tot = max(1, both_epi + ovl + one_epi)
        print(f"   CUs {ncu}, max wgs per CU {max(len(v) for v in by.values())}; epilogue samples: both-in-epilogue "
              f"{both_epi / tot:.2f}, epilogue beside a K-loop {ovl / tot:.2f}, epilogue alone {one_epi / tot:.2f}",
              flush=True)


if __name__ == "__main__":
    main()
