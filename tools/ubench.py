"""Issue cost of single VALU instructions on gfx950 (tools/ubench.hip; build: bash tools/ubench_build.sh).
Prints cycles per instruction (s_memtime delta / instructions, median over waves) at 1 and 2 waves
per SIMD.  Usage: python tools/ubench.py"""
import ctypes
import sys
from pathlib import Path

import torch

OPS = ["v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_fma_f32", "v_xor_b32", "v_mad_u64_u32", "v_exp_f32",
       "v_pk_fma_f32", "v_mul_u32_u24", "v_rcp_f32", "v_fma_f32 x64", "v_exp_f32 x64", "v_mad_u64 x64",
       "v_pk_fma_f32 x64", "v_cvt_pk_bf16 x64", "v_accvgpr_rd x64"]
PER_ITER = [8] * 10 + [64] * 6      # instructions per loop iteration (the x64 forms amortise the branch)


def main():
    lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "libubench.so"))
    blocks, iters = 256, 2000
    torch.zeros(1, device="cuda")
    for threads in (256, 512):
        for op, name in enumerate(OPS):
            cyc = torch.zeros(2 * blocks * threads // 64, dtype=torch.int64, device="cuda")
            sink = torch.zeros(blocks * threads, dtype=torch.int32, device="cuda")
            for _ in range(2):
                rc = lib.ubench(op, blocks, threads, iters, ctypes.c_void_p(cyc.data_ptr()),
                                ctypes.c_void_p(sink.data_ptr()))
                assert rc == 0, rc
            torch.cuda.synchronize()
            c = cyc.view(-1, 2)[:, 0].double().sort().values
            rt = cyc.view(-1, 2)[:, 1].double().sort().values
            ns = float(rt[len(rt) // 2]) * 10.0 / (iters * PER_ITER[op])       # wall ns per instruction of one wave
            print(f"{name:16s} waves/SIMD {threads // 256}: {float(c[len(c) // 2]) / (iters * PER_ITER[op]):6.2f} cyc/inst "
                  f"(s_memtime)  {ns:6.3f} ns/inst per wave  SIMD rate {threads // 256 / ns:6.3f} inst/ns",
                  flush=True)


def dma():
    """LDS-DMA source pattern (ubench.hip dma_kernel): 16 rows x 64 B vs 8 rows x 128 B per wave-instruction"""
    lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "libubench.so"))
    K = 768
    blocks = 256
    A = torch.randn(blocks * 256, K, device="cuda").to(torch.bfloat16)
    for panels in (256, 8, 1):
        for rounds in (4,):
            for pat in (0, 1, 2, 3, 0, 1, 2, 3):
                cyc = torch.zeros(blocks, dtype=torch.int64, device="cuda")
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                args = (pat, blocks, ctypes.c_void_p(A.data_ptr()), K, rounds, panels, ctypes.c_void_p(cyc.data_ptr()))
                lib.ubench_dma(*args)
                torch.cuda.synchronize()
                s.record()
                rc = lib.ubench_dma(*args)
                e.record()
                torch.cuda.synchronize()
                assert rc == 0, rc
                ms = s.elapsed_time(e)
                per_cu = 256 * K * 2 * rounds
                c = cyc.double().sort().values
                print(f"dma pat {pat} ({['16 rows x 64 B global', '8 rows x 128 B global', '16 rows x 64 B buffer', '8 rows x 128 B buffer'][pat]}) panels {panels:3d} rounds "
                      f"{rounds}: {ms * 1e3:8.1f} us  {per_cu * blocks / ms / 1e6:7.1f} GB/s  per CU "
                      f"{per_cu / float(c[len(c) // 2]):.1f} B/cyc (s_memtime)", flush=True)


if __name__ == "__main__":
    if "--dma" in sys.argv:
        sys.exit(dma())
    sys.exit(main())
