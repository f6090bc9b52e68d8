"""Contract T pad skipping measured: ConcatModel train step (fwd + bwd + Adam,
train.py:94-113) on token batches of length 512 whose real lengths follow the reference's
feature/EEG/*_bert.pickle (33-65 tokens, mean 51.3: SURVEY §0), bf16, packed vs padded BERT.

usage: python tools/varlen_bench.py [B ...]      (default 32 256)
Prints one JSON line per (B, varlen) with samples/s and ms per step.
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
import torch  # noqa: E402


def main():
    from eegfusion.modules import ConcatModel
    from eegfusion.trainer import SinglePassTrainer
    sizes = [int(x) for x in sys.argv[1:]] or [32, 256]
    for B in sizes:
        g = torch.Generator().manual_seed(980616)
        L = 512
        lens = torch.randint(33, 66, (B,), generator=g)
        ids = torch.randint(1000, 30000, (B, L), generator=g)
        mask = (torch.arange(L)[None, :] < lens[:, None]).long()
        ids = ids * mask
        batch = {"title_input": ids.cuda(), "text_mask": mask.cuda(),
                 "frame_input": (torch.randn(B, 1, 512, generator=g) * 0.5).cuda()}
        labels = (torch.rand(B, generator=g) < 0.66).long().cuda()
        for varlen in (False, True):
            torch.manual_seed(980616)
            m = ConcatModel(contract="T", dropout=0.1).cuda().set_compute_dtype(torch.bfloat16)
            m.engine.cfg.varlen = varlen
            tr = SinglePassTrainer(m.engine, lr=1e-6)
            for _ in range(3):
                tr.step(batch, labels)
            torch.cuda.synchronize()
            steps = 10
            t0 = time.perf_counter()
            for _ in range(steps):
                loss, _ = tr.step(batch, labels)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            print(json.dumps({"B": B, "L": L, "varlen": varlen, "mean_len": round(lens.float().mean().item(), 2),
                              "ms_per_step": round(dt * 1e3, 3), "samples_per_s": round(B / dt, 1),
                              "loss": round(float(loss.item()), 5)}), flush=True)
            del tr, m
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
