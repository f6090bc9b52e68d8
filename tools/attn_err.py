"""Error of the L = 256 bf16 attention kernels against a float64 reference with the replayed dropout mask
(tests/philox_ref.attn_probs_mask), per output, at p = 0 and p = 0.1: a fwd / bwd mask disagreement shows
as a p = 0.1 error far above the p = 0 one.  Usage: python tools/attn_err.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "eeg-multimodal_amd"), str(ROOT / "tests")]
import torch  # noqa: E402

from eegfusion import _lib  # noqa: E402


def rel(a, b):
    return float((a.double() - b).abs().max() / b.abs().max())


def main():
    from philox_ref import attn_probs_mask
    B, L, dt = int(sys.argv[1]) if len(sys.argv) > 1 else 8, 256, torch.bfloat16
    for p in (0.0, 0.1):
        for typ, code in ((torch.bfloat16, _lib.BF16), (torch.float32, _lib.F32)):
            torch.manual_seed(4)
            qkv = torch.randn(B, L, 2304, device="cuda").to(typ)
            out = torch.empty(B, L, 768, device="cuda", dtype=typ)
            lse = torch.empty(B, 12, L, device="cuda")
            s = torch.cuda.current_stream().cuda_stream
            _lib.call("eegf_attn_fwd", code, B, 12, L, qkv.data_ptr(), 2304, None, 0.125, p, 123, 9, out.data_ptr(), 768,
                      lse.data_ptr(), None, s)
            qr = qkv.double().clone().requires_grad_()
            q, k, v = (t.transpose(1, 2) for t in qr.view(B, L, 3, 12, 64).unbind(2))
            P = (q @ k.transpose(-1, -2) / 8.0).softmax(-1)
            if p > 0:
                import numpy as np
                z = attn_probs_mask(123, 9, np.arange(B * 12 * L * L, dtype=np.uint64), p, L)
                P = P * torch.from_numpy(z).view(B, 12, L, L).cuda()
            ref = (P @ v).transpose(1, 2).reshape(B, L, 768)
            dout = torch.randn(B, L, 768, device="cuda").to(typ)
            ref.backward(dout.double())
            dqkv = torch.empty_like(qkv)
            ws = torch.empty(max(_lib.lib().eegf_attn_bwd_workspace(B, L), 1), device="cuda")
            _lib.call("eegf_attn_bwd", code, B, 12, L, qkv.data_ptr(), 2304, None, 0.125, p, 123, 9, out.data_ptr(),
                      dout.data_ptr(), 768, lse.data_ptr(), None, dqkv.data_ptr(), ws.data_ptr(), s)
            torch.cuda.synchronize()
            g = qr.grad
            print(f"{str(typ):15s} p={p}: out {rel(out, ref.detach()):.2e}  dq {rel(dqkv[..., :768], g[..., :768]):.2e}  "
                  f"dk {rel(dqkv[..., 768:1536], g[..., 768:1536]):.2e}  dv {rel(dqkv[..., 1536:], g[..., 1536:]):.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
