"""Interleaved A/B of a routing key (eegf_tune) on the whole bench step, in one process: the same
PriGumbel B=256 bf16 step (bench.py's workload) timed in rounds alternating the key's values, median
ms per step per value.  Clock / thermal drift between separate bench runs cannot bias it.
Usage: python tools/step_ab.py --key 11 --values 0,2 [--rounds 5] [--steps 10]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "eeg-multimodal_amd"), str(ROOT)]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", type=int, required=True)
    ap.add_argument("--values", required=True)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    from eegfusion import _lib
    from eegfusion.modules import PriGumbelModel
    from eegfusion.trainer import PriGumbelTrainer
    lib = _lib.lib()
    lib.eegf_tune.argtypes = [_lib.i32, _lib.i32]
    vals = [int(v) for v in args.values.split(",")]
    dev = torch.device("cuda")
    torch.manual_seed(980616)
    m = PriGumbelModel(1.0, contract="W", dropout=0.1).to(dev).set_compute_dtype(torch.bfloat16)
    tr = PriGumbelTrainer(m.engine, lr=1e-6)
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(7)
    batch = {"eeg": torch.randn(B, 64, 256, generator=g, device=dev),
             "act": torch.randn(B, 32, generator=g, device=dev) * 0.5}
    labels = (torch.rand(B, generator=g, device=dev) < 0.66).long()
    old = lib.eegf_tune(args.key, vals[0])
    res = {v: [] for v in vals}
    for _ in range(args.rounds):
        for v in vals:
            lib.eegf_tune(args.key, v)
            for _ in range(2):
                tr.step(batch, labels)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.steps):
                tr.step(batch, labels)
            e.record()
            torch.cuda.synchronize()
            res[v].append(s.elapsed_time(e) / args.steps)
    lib.eegf_tune(args.key, old)
    for v in vals:
        x = sorted(res[v])
        print(f"key {args.key} = {v}: median {x[len(x) // 2]:.3f} ms/step  ({B / x[len(x) // 2] * 1e3:.1f} samples/s)  "
              f"all {[round(t, 3) for t in res[v]]}", flush=True)


if __name__ == "__main__":
    main()
