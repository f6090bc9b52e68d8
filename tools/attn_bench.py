"""Time eegf_attn_fwd / eegf_attn_bwd at the bench shape (B=256, L=256, 12 heads, bf16, p=0.1).
Usage: python tools/attn_bench.py   (EEGF_ATTN256=0 selects the generic kernels)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
import torch  # noqa: E402

from eegfusion import _lib  # noqa: E402


def main(B=256, L=256, p=0.1, iters=20, use_bits=True):
    dev = "cuda"
    qkv = torch.randn(B, L, 2304, device=dev).to(torch.bfloat16)
    out = torch.empty(B, L, 768, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, 12, L, device=dev)
    dout = torch.randn(B, L, 768, device=dev).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    bits = torch.empty(B * 12 * L * L // 32, device=dev, dtype=torch.int32)
    bp = bits.data_ptr() if use_bits else None
    ws = torch.empty(max(_lib.lib().eegf_attn_bwd_workspace(B, L), 1), device=dev)
    s = torch.cuda.current_stream().cuda_stream
    fwd = lambda: _lib.call("eegf_attn_fwd", _lib.BF16, B, 12, L, qkv.data_ptr(), 2304, None, 0.125, p, 7, 3,
                            out.data_ptr(), 768, lse.data_ptr(), bp, s)
    bwd = lambda: _lib.call("eegf_attn_bwd", _lib.BF16, B, 12, L, qkv.data_ptr(), 2304, None, 0.125, p, 7, 3,
                            out.data_ptr(), dout.data_ptr(), 768, lse.data_ptr(), bp, dqkv.data_ptr(), ws.data_ptr(), s)
    for name, fn, flops in (("fwd", fwd, 4.0 * B * 12 * L * L * 64), ("bwd", bwd, 10.0 * B * 12 * L * L * 64)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        print(f"attn_{name} B={B} L={L} p={p} bits={int(use_bits)}: {ms * 1e3:8.1f} us  {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    nobits = "--nobits" in sys.argv        # only the regenerated-mask path (the engine's)
    ps = [float(x) for x in sys.argv[1:] if not x.startswith("--")] or [0.1]
    for p in ps:
        if not nobits or p == 0:
            main(p=p, use_bits=True)
        if p > 0:
            main(p=p, use_bits=False)
