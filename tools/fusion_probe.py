"""Where the fusion forward's time goes (B = 256): graph-replayed launches of eegf_fusion_fwd as the
bench times it (PriGumbel, Philox draws), with the Laplace / Gumbel draws injected (no Philox, no logs),
and as PriConcat (concat + min-max only: the kernel's floor).  usage: python tools/fusion_probe.py"""
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
import torch  # noqa: E402

from eegfusion import _lib  # noqa: E402


def timed(fn, reps=20, replays=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (replays * reps)


def main():
    dev, B, HID = "cuda", 256, 768
    F32 = _lib.F32
    P = lambda t: None if t is None else t.data_ptr()
    st = lambda: torch.cuda.current_stream().cuda_stream
    r = lambda *s: torch.randn(*s, device=dev)
    pooled, vis, cross = r(B, HID), r(B, HID), r(B, HID)
    DP = r(1, 3 * HID) * 0.1
    noise, gum = r(B, 3 * HID), r(2, B, 3 * HID)
    gout, xn = torch.empty(B, 3 * HID, device=dev), torch.empty(B, 3 * HID, device=dev)
    amin, amax = torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev)
    rng = torch.empty(B, device=dev)
    ea = math.exp(1.0)

    def fwd(variant, nz, gm):
        return lambda: _lib.call("eegf_fusion_fwd", F32, B, variant, P(pooled), HID, P(vis), HID, P(cross), HID,
                                 P(DP), P(nz), P(gm), None, 1, 0, ea, 1.0, 980616, 200, P(gout), P(xn), P(amin),
                                 P(amax), P(rng), st())
    for name, fn in [("prigumbel, Philox draws (the bench's form)", fwd(_lib.FUSE_PRIGUMBEL, None, None)),
                     ("prigumbel, injected draws", fwd(_lib.FUSE_PRIGUMBEL, noise, gum)),
                     ("priconcat (concat + min-max)", fwd(_lib.FUSE_PRICONCAT, None, None))]:
        print(f"fusion_fwd {name:45s} {timed(fn):7.2f} us", flush=True)


if __name__ == "__main__":
    main()
