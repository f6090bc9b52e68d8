#!/usr/bin/env python3
"""bench.py — samples/sec of the EEG+action fusion training iteration on MI355X.

Workload (BASELINE.json configs[2]/[3]: PriGumbel eps=1.0 "newfrac", bf16, batch 256 per GPU,
synthetic 64-channel x 256-step EEG windows + 32-d action vectors, contract W): one step is one
full PriGumbel iteration of past_acc.py:194-212 — pass 1 (hard=False) forward + DP-gradient
backward + DP Adam, pass 2 (hard=True) forward + full backward + model Adam — all in
libeegfusion.so HIP kernels, gradients averaged over ranks with RCCL all-reduce when N > 1.
Per-GPU batch is fixed as N grows (weak scaling).  `--variant priconcat` times the single-pass
PriConcat step (configs[1]) instead.

Run: python bench.py [--gpus N --steps K --warmup W]   (N > 1 under torch.distributed.run)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HID, L, C, A = 768, 256, 64, 32
F_PER_SAMPLE = 46.03e9            # forward GEMM+attention FLOPs per sample, contract W
PEAK_BF16 = 2500.0                # TFLOP/s dense bf16 MFMA (MI355X_MICROARCH.md)
METRIC = "samples/sec at batch 256, 64ch×256 EEG + 32-d action, 1/2/4/8 GPUs"


def flops_per_sample(variant: str) -> float:
    # PriGumbel iteration = pass-1 fwd + pass-2 fwd+bwd = 4F; PriConcat step = fwd+bwd = 3F
    return (4.0 if variant == "prigumbel" else 3.0) * F_PER_SAMPLE


def cpu_baseline(variant: str, batch: int = 2, iters: int = 3) -> dict:
    """The CPU oracle (torch fp32 restatement, oracle/fusion_oracle.py) timed on the host cores on a
    bounded sample of the same iteration."""
    from oracle import fusion_oracle as O
    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(0)
    shapes = O.param_shapes("W", "prigumbel" if variant == "prigumbel" else "priconcat")
    p = {}
    for k, s in shapes.items():
        if "LayerNorm.weight" in k or ".norm" in k and k.endswith("weight"):
            t = torch.ones(s)
        elif len(s) >= 2:
            t = torch.randn(s, generator=g) * 0.02
        else:
            t = torch.zeros(s)
        p[k] = t.requires_grad_()
    eeg = torch.randn(batch, C, L, generator=g)
    act = torch.randn(batch, A, generator=g) * 0.5
    labels = torch.randint(0, 2, (batch,), generator=g)
    batch_d = dict(eeg=eeg, act=act)
    model_p = [v for k, v in p.items() if k != "DP"]
    mopt = torch.optim.Adam(model_p, lr=1e-6)
    dopt = torch.optim.Adam([p["DP"]], lr=1e-6) if "DP" in p else None
    lap = torch.distributions.laplace.Laplace(torch.tensor([0.0]), torch.tensor([1.0]))

    def draws():
        n = lap.sample((batch, 3 * HID)).view(batch, 3 * HID)
        gm = -torch.empty(2, batch, 3 * HID).exponential_().log()
        return n, gm

    def iteration():
        if variant == "prigumbel":
            dopt.zero_grad()
            with torch.no_grad():
                pooled, img, cross = O.encoders(p, batch_d, O.PathConfig(contract="W"))
            n, gm = draws()
            f = O.minmax(torch.cat((pooled, img, cross), 1))
            logits = O.head(p, O.prigumbel_gate(f, p["DP"], n, gm, 1.0, "newfrac", False))
            O.cal_loss(logits, labels)[0].backward()
            dopt.step()
            mopt.zero_grad()
            n, gm = draws()
            pc = O.PathConfig(contract="W", variant="prigumbel", hard=True)
            O.cal_loss(O.forward(p, batch_d, pc, noise=n, gumbels=gm), labels)[0].backward()
            mopt.step()
        else:
            mopt.zero_grad()
            pc = O.PathConfig(contract="W", variant="priconcat")
            torch.nn.functional.cross_entropy(O.forward(p, batch_d, pc), labels).backward()
            mopt.step()

    iteration()                                        # warm-up
    t0 = time.perf_counter()
    for _ in range(iters):
        iteration()
    dt = time.perf_counter() - t0
    return {"value": round(batch * iters / dt, 4), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/fusion_oracle.py {variant} iteration (torch CPU fp32, dropout 0), batch {batch}, "
                      f"64x256 EEG + 32-d action, {iters} timed iterations after 1 warm-up, {dt:.1f} s"}


def load_traffic(tag: str):
    f = ROOT / "profiles" / "traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        return d.get(tag, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--variant", default="prigumbel", choices=["prigumbel", "priconcat"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=8)
    ap.add_argument("--cpu-iters", type=int, default=4)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from eegfusion.modules import PriConcatModel, PriGumbelModel
    from eegfusion.trainer import GradReducer, PriGumbelTrainer, SinglePassTrainer

    torch.manual_seed(980616)                              # identical init on every rank
    if args.variant == "prigumbel":
        model = PriGumbelModel(1.0, contract="W", eps_mode="newfrac", dropout=0.1, seed=980616 + rank)
    else:
        model = PriConcatModel(None, contract="W", dropout=0.1, seed=980616 + rank)
    model = model.to(dev).set_compute_dtype(torch.bfloat16)
    eng = model.engine
    reducer = GradReducer()
    trainer = (PriGumbelTrainer if args.variant == "prigumbel" else SinglePassTrainer)(eng, lr=1e-6, reducer=reducer)

    B = args.batch
    g = torch.Generator(device=dev).manual_seed(980616 + 7919 * rank)   # disjoint synthetic shard per rank
    eeg = torch.randn(B, C, L, generator=g, device=dev)
    act = torch.randn(B, A, generator=g, device=dev) * 0.5
    labels = (torch.rand(B, generator=g, device=dev) < 0.66).long()
    batch = {"eeg": eeg, "act": act}

    for _ in range(args.warmup):
        trainer.step(batch, labels)
    tags = ("ffn1_fwd", "qkv_fwd", "ffn2_fwd", "attn_fwd")
    eng.probe = {t: [] for t in tags}
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, _ = trainer.step(batch, labels)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    probe, eng.probe = eng.probe, None
    kms = {t: sum(s.elapsed_time(e) for s, e in v) / max(len(v), 1) for t, v in probe.items()}

    if rank == 0:
        value = world * B * args.steps / dt
        R = B * L
        ffn1_flops = 2.0 * R * 3072 * 768                 # algorithmic FLOPs per FFN1 launch
        ach = ffn1_flops / (kms["ffn1_fwd"] * 1e-3) / 1e12
        step_tf = value / world * flops_per_sample(args.variant) / 1e12
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": ("PriGumbel eps=1.0 newfrac iteration (past_acc.py:194-212): pass-1 fwd + DP "
                                    "Adam, pass-2 fwd/bwd + model Adam" if args.variant == "prigumbel" else
                                    "PriConcat eps=1.0 step (main_0430.py): fwd/bwd + Adam"),
                       "global_batch": world * B, "per_gpu_batch": B, "seq_len": L, "eeg": f"{C}ch x {L}",
                       "action_dim": A, "encoder": "BERT-base 12x768 over per-step Linear(64,768) tokens",
                       "parallelism": f"dp{world}"},
            "roofline": {"kernel": "ffn1_fwd (BertIntermediate GEMM 65536x3072x768 + bias + GELU)", "bound": "mfma",
                         "achieved": round(ach, 1), "peak": PEAK_BF16, "unit": "TFLOP/s",
                         "frac": round(ach / PEAK_BF16, 4), "traffic": load_traffic("ffn1_fwd"),
                         "avg_ms": round(kms["ffn1_fwd"], 4)},
            "step_roofline": {"achieved": round(step_tf, 1), "unit": "TFLOP/s", "frac": round(step_tf / PEAK_BF16, 4),
                              "flops_per_sample": flops_per_sample(args.variant)},
            "kernel_ms": {k: round(v, 4) for k, v in kms.items()},
            "loss": float(loss[-1].item()),
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.variant, args.cpu_batch, args.cpu_iters)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
