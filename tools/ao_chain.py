"""Why the attention out-projection forward (gemm4h, 65536 x 768 x 768) takes ~115 us inside the step
but ~83 us alone: time it alone, right after the attention forward that writes its input, and after
the attention forward followed by an unrelated kernel.  Usage: python tools/ao_chain.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
import torch  # noqa: E402

from eegfusion import _lib  # noqa: E402
from eegfusion import kernels as K  # noqa: E402


def main():
    dev, dt = "cuda", torch.bfloat16
    B, L = 256, 256
    R = B * L
    qkv = torch.randn(R, 2304, device=dev).to(dt)
    ctx = torch.empty(R, 768, device=dev, dtype=dt)
    lse = torch.empty(B, 12, L, device=dev)
    W = (torch.randn(768, 768, device=dev) * 0.03).to(dt)
    bias = torch.randn(768, device=dev)
    out = torch.empty(R, 768, device=dev, dtype=dt)
    junk = torch.empty(64 << 20, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    attn = lambda: _lib.call("eegf_attn_fwd", _lib.BF16, B, 12, L, qkv.data_ptr(), 2304, None, 0.125, 0.1, 7, 3,
                             ctx.data_ptr(), 768, lse.data_ptr(), None, s)
    ao = lambda: K.linear(ctx, W, bias, out=out)
    attn()
    torch.cuda.synchronize()

    def timed(pre, n=20):
        ts = []
        for _ in range(n):
            pre()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ao()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        return ts[len(ts) // 2]

    for rep in range(2):
        print(f"AO alone                 {timed(lambda: None):7.1f} us", flush=True)
        print(f"AO after attn_fwd        {timed(attn):7.1f} us", flush=True)
        print(f"AO after attn + fill     {timed(lambda: (attn(), junk.fill_(1.0))):7.1f} us", flush=True)
        print(f"AO after 256 MB fill     {timed(lambda: junk.fill_(2.0)):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
