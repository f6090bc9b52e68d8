"""Bit-identity of the production GEMM epilogues across two library builds: runs every epilogue form
of the persistent K = 768 GEMMs (bias, GELU with the pre-activation, GELU + GELU', the input gradients
x aux and with beta = 1) on fixed seeded inputs at a production shape and prints one sha256 per output.
Run it once per build (EEGF_LIB=<other .so> for the second) and compare the lines: a schedule-only
change of an epilogue must print the same digests.
usage: python tools/epi_bits.py [rows]"""
import hashlib
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
import torch  # noqa: E402

from eegfusion import kernels as K  # noqa: E402


def digest(t):
    return hashlib.sha256(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev, dt = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(1234)
    rn = lambda *s: torch.randn(*s, device=dev, dtype=torch.float32, generator=g)
    for N, Kd in ((3072, 768), (2304, 768), (768, 3072)):
        A = (rn(M, Kd) * 2).to(dt)
        B = (rn(N, Kd) * 0.05).to(dt)
        bias = rn(N)
        for epi in ("bias", "bias_gelu", "bias_gelu_d"):
            if epi != "bias" and N != 3072:
                continue
            C = torch.empty(M, N, device=dev, dtype=dt)
            aux = torch.empty(M, N, device=dev, dtype=dt) if epi != "bias" else None
            K.gemm(A, B, C, M=M, N=N, K=Kd, a_kc=1, b_kc=1, lda=Kd, ldb=Kd, ldc=N, epi=epi, bias=bias, aux=aux,
                   ldaux=N)
            torch.cuda.synchronize()
            print(f"fwd   {N:5d}x{Kd:5d} {epi:12s} C {digest(C)}" + (f" aux {digest(aux)}" if aux is not None else ""))
    # input gradients: dY [M, K] (k-contiguous) x W [K, N] (k-major)
    for N, Kd, epi, beta in ((3072, 768, "mul_aux", 0.0), (3072, 768, "dgelu", 0.0), (768, 3072, "none", 1.0),
                             (768, 2304, "none", 1.0), (768, 768, "none", 0.0)):
        A = rn(M, Kd).to(dt)
        B = (rn(Kd, N) * 0.05).to(dt)
        C = (rn(M, N) * 0.01).to(dt)
        aux = rn(M, N).to(dt) if epi != "none" else None
        K.gemm(A, B, C, M=M, N=N, K=Kd, a_kc=1, b_kc=0, lda=Kd, ldb=N, ldc=N, epi=epi, aux=aux, ldaux=N, beta=beta)
        torch.cuda.synchronize()
        print(f"dgrad {N:5d}x{Kd:5d} {epi:8s} beta={beta:g} C {digest(C)}")
    # weight gradients with the fused bias gradient (eegf_gemm_wgrad_bias): dW [Mo][N] += dY^T X, db += dY.sum(0)
    from eegfusion import _lib
    lib = _lib.lib()
    ws = torch.empty(64 << 20, device=dev)
    R = 4 * M
    for Mo, N in ((2304, 768), (768, 3072)):
        dy = rn(R, Mo).to(dt)
        x = rn(R, N).to(dt)
        dw = rn(Mo, N) * 0.01
        db = rn(Mo) * 0.01
        st = lib.eegf_gemm_wgrad_bias(_lib.BF16, Mo, N, R, dy.data_ptr(), Mo, x.data_ptr(), N, dw.data_ptr(), N, 1.0,
                                      db.data_ptr(), ws.data_ptr(), ws.numel() * 4, 0)
        torch.cuda.synchronize()
        print(f"wgrad {Mo:5d}x{N:5d} K={R} st={st} dW {digest(dw)} db {digest(db)}")
    # the L = 256 attention kernels (dropout 0.1, regenerated masks and exported bits)
    B, L = 64, 256
    qkv = (rn(B, L, 2304) * 2).to(dt)
    dout = rn(B, L, 768).to(dt)
    s = torch.cuda.current_stream().cuda_stream
    for use_bits in (False, True):
        out = torch.empty(B, L, 768, device=dev, dtype=dt)
        lse = torch.empty(B, 12, L, device=dev)
        dqkv = torch.empty_like(qkv)
        bits = torch.zeros(B * 12 * L * L // 32, device=dev, dtype=torch.int32) if use_bits else None
        bp = bits.data_ptr() if use_bits else None
        _lib.call("eegf_attn_fwd", _lib.BF16, B, 12, L, qkv.data_ptr(), 2304, None, 0.125, 0.1, 7, 3, out.data_ptr(), 768,
                  lse.data_ptr(), bp, s)
        _lib.call("eegf_attn_bwd", _lib.BF16, B, 12, L, qkv.data_ptr(), 2304, None, 0.125, 0.1, 7, 3, out.data_ptr(),
                  dout.data_ptr(), 768, lse.data_ptr(), bp, dqkv.data_ptr(), None, s)
        torch.cuda.synchronize()
        print(f"attn  bits={int(use_bits)} out {digest(out)} lse {digest(lse)} dqkv {digest(dqkv)}"
              + (f" keep {digest(bits)}" if use_bits else ""))


if __name__ == "__main__":
    main()
