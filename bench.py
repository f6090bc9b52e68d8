#!/usr/bin/env python3
"""bench.py — samples/sec of the EEG+action fusion training iteration on MI355X.

Workload (BASELINE.json configs[2]/[3]: PriGumbel eps=1.0 "newfrac", bf16, batch 256 per GPU,
synthetic 64-channel x 256-step EEG windows + 32-d action vectors, contract W): one step is one
full PriGumbel iteration of past_acc.py:194-212 — pass 1 (hard=False) forward + DP-gradient
backward + DP Adam, pass 2 (hard=True) forward + full backward + model Adam — all in
libeegfusion.so HIP kernels, gradients averaged over ranks with RCCL all-reduce when N > 1.
Per-GPU batch is fixed as N grows (weak scaling).

Modes:
  (default)              configs[2] (N = 1) / configs[3] (N = 8): PriGumbel, B = 256 per GPU
  --variant priconcat    configs[1]: the single-pass PriConcat step
  --eps-sweep 0.1,1,3,5,10 --feawei 2048 --batch 512
                         configs[4]: a feawei feature pass (forward-only over N synthetic samples,
                         DP initialised on the device, past_acc_feawei.py:127-163), then K timed
                         iterations per eps of the sweep (fresh optimizer state per eps, as each
                         past_acc.py:254-260 run starts one); value = all timed samples / all timed time

Multi-GPU: one process per GPU over RCCL.  Under torch.distributed.run the world size comes from
WORLD_SIZE and must equal --gpus (else exit 2).  `python bench.py --gpus N` without a launcher starts
N fresh rank processes through torch.distributed.run itself (before any GPU call) and exits with
their status.  The JSON line reports the world size the process group saw.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import hashlib
import subprocess
import sys
import time
import types
from pathlib import Path

ROOT = Path(__file__).resolve().parent

HID, L, C, A = 768, 256, 64, 32
F_PER_SAMPLE = 46.03e9            # forward GEMM+attention FLOPs per sample, contract W
PEAK_BF16 = 2500.0                # TFLOP/s dense bf16 MFMA (MI355X_MICROARCH.md)
METRIC = "samples/sec at batch 256, 64ch×256 EEG + 32-d action, 1/2/4/8 GPUs"
PMC_FILE = "pmc_r6f.json"          # profiles/: tools/pmc_table.py output (HBM bytes, MFMA busy per group)
# probed kernel groups (HIP events around each launch on the launch stream, engine.probe)
KERNEL_GROUPS = {
    "ffn1_fwd": "BertIntermediate GEMM + bias + GELU, pass 1 (no save), 65536x3072x768",
    "ffn1_fwd_gd": "BertIntermediate GEMM + bias + GELU + GELU' saved for the backward, pass 2, 65536x3072x768",
    "qkv_fwd": "fused Q|K|V projection GEMM + bias, 65536x2304x768",
    "ao_fwd": "attention output projection GEMM + bias, 65536x768x768",
    "ffn2_fwd": "BertOutput GEMM + bias, 65536x768x3072",
    "attn_fwd": "fused self-attention forward (QK^T, softmax, dropout, PV), 256x12 heads x 256^2 x 64",
    "attn_bwd": "fused self-attention backward (dQ, dK, dV)",
    "dgrad_qkv": "input gradient through the Q|K|V projection, 65536x768x2304",
    "dgrad_ffn1": "input gradient through BertIntermediate, 65536x768x3072",
    "dgrad_out": "input gradient through the attention output projection, 65536x768x768",
    "dgrad_ffn2": "input gradient through BertOutput with the GELU' product, 65536x3072x768",
    "wgrad": "weight gradients (split-K over 65536 tokens) with the bias gradients fused (row sums)",
    # HBM-bound kernels, reported in GB/s (the gate / min-max / CE / LN /
    # Adam kernels separately): engine.probe records their algorithmic bytes per launch
    "fusion_fwd": "concat + row min-max + PriGumbel gate (Laplace, Gumbel-softmax, eps_hat), fp32 [B, 2304]",
    "fusion_bwd": "its backward: min-max / gate gradients to the three encoders (+ the DP gradient rows, pass 1)",
    "cross_entropy": "F.cross_entropy(mean) + argmax count + logit gradients, [B, 2]",
    "ln_fwd768": "BERT hidden dropout + residual + LayerNorm forward, [65536, 768] bf16",
    "adam": "fused Adam (+ bf16 shadow) over the used arena ranges",
}
HBM_TAGS = ("fusion_fwd", "fusion_bwd", "cross_entropy", "ln_fwd768", "adam")
PEAK_HBM = 8000.0                 # GB/s HBM3E (MI355X_MICROARCH.md)
T_ORIGIN = time.perf_counter()    # process start: the CPU-baseline budget guard counts from here
# The kernel (rocprof symbol) each probed group runs on: the roofline object reports the SYMBOL with the
# most time per step, combining the groups that share it, with the PMC traffic of that symbol
# (profiles/PMC_FILE key).  Algorithmic bytes per launch: A + W + C (+ aux) of each shape, bf16.
R_TOK = 256 * L
KERNEL_SYMBOLS = {
    "gemm4r_kernel<true, 1, false>": {
        "tags": ("qkv_fwd", "ao_fwd", "ffn2_fwd"), "pmc": "fwd_bias_qkv_ao_ffn2",
        "what": "persistent 256x256 bf16 GEMM, bias epilogue: the QKV, attention-output and FFN2 forwards",
        "bytes": {"qkv_fwd": 2 * (R_TOK * 768 + 2304 * 768 + R_TOK * 2304),
                  "ao_fwd": 2 * (R_TOK * 768 + 768 * 768 + R_TOK * 768),
                  "ffn2_fwd": 2 * (R_TOK * 3072 + 768 * 3072 + R_TOK * 768)}},
    "gemm4w_kernel<false, false, 0, float, true> + splitk_rowsum_reduce": {
        "tags": ("wgrad",), "pmc": "wgrad",
        "what": "split-K weight-gradient GEMM with the bias row sums, and its fixed-order slab reduction"},
    "gemm4r_kernel<false, 0, true>": {
        "tags": ("dgrad_qkv", "dgrad_ffn1"), "pmc": "dgrad_qkv_ffn1",
        "what": "persistent GEMM, input gradients accumulating onto the residual gradient (beta = 1)"},
    "gemm4r_kernel<true, 8, false>": {"tags": ("ffn1_fwd_gd",), "pmc": "ffn1_fwd",
                                      "what": "persistent GEMM, FFN1 + bias + GELU + GELU' (pass 2)"},
    "gemm4r_kernel<true, 2, false>": {"tags": ("ffn1_fwd",), "pmc": "ffn1_fwd",
                                      "what": "persistent GEMM, FFN1 + bias + GELU (pass 1)"},
    "gemm4r_kernel<false, 9, false>": {"tags": ("dgrad_ffn2",), "pmc": "dgrad_ffn2",
                                       "what": "persistent GEMM, FFN2 input gradient x GELU'"},
    "gemm4r_kernel<false, 0, false>": {"tags": ("dgrad_out",), "pmc": "dgrad_out",
                                       "what": "persistent GEMM, attention-output input gradient"},
    "attn_bwd256_kernel<true>": {"tags": ("attn_bwd",), "pmc": "attn_bwd", "what": "L = 256 attention backward"},
    "attn_fwd256_kernel<true, false>": {"tags": ("attn_fwd",), "pmc": "attn_fwd", "what": "L = 256 attention forward"},
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)   # ~2.8 s timed: long enough for an smi sampler to see the GPU busy
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--variant", default="prigumbel", choices=["prigumbel", "priconcat"])
    ap.add_argument("--eps", type=float, default=1.0)
    ap.add_argument("--eps-sweep", default="", help="comma-separated eps values (configs[4]: 0.1,1,3,5,10)")
    ap.add_argument("--eps-mode", default="newfrac", choices=["newfrac", "new"])
    ap.add_argument("--feawei", type=int, default=0, help="feawei feature pass over this many synthetic samples")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true",
                    help="no HIP-event probes in the timed loop (no per-kernel roofline; A/B of the probes' cost)")
    ap.add_argument("--cpu-batch", type=int, default=256,
                    help="CPU-baseline batch (BASELINE.md section 3: the bench's batch, 256; ~107 s per iteration "
                         "on a GPU box's 16-CPU share)")
    ap.add_argument("--cpu-iters", type=int, default=3, help="CPU-baseline timed iterations after one warm-up")
    ap.add_argument("--cpu-warm-batch", type=int, default=16,
                    help="batch of the CPU-baseline warm-up iteration (0 = --cpu-batch; the batch-256 sample "
                         "warms up at 16: thread pool and allocator, not another 2-4 minutes of page faults)")
    ap.add_argument("--cpu-budget", type=float, default=450.0,
                    help="seconds since process start the run may reach: the CPU leg stops after the last "
                         "iteration whose successor would end past it (the count is stated in the line)")
    ap.add_argument("--cpu-baseline-only", action="store_true",
                    help="time only the CPU baseline (e.g. --cpu-batch 256 --cpu-iters 3, BASELINE.md §3) and print "
                         "its JSON; profiles/" + "cpu_baseline_b256.json holds that run for the bench line")
    ap.add_argument("--cpu-baseline-out", default="",
                    help="with --cpu-baseline-only: also merge the result into this JSON file under the variant's key")
    ap.add_argument("--master-port", type=int, default=29531)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1: nccl (= RCCL, one GPU per rank) or gloo (device "
                         "tensors through host memory; lets N ranks share one GPU to exercise the DDP body "
                         "where only one GPU exists — its timing is not an RCCL measurement)")
    ap.add_argument("--check-replicas", action="store_true",
                    help="after the timed loop, all-gather a SHA-256 of every rank's fp32 master weights and Adam "
                         "moments and report whether the replicas are bitwise identical")
    ap.add_argument("--selftest", action="store_true",
                    help="launcher / process-group check only (gloo, CPU): rank 0 prints the world size")
    return ap.parse_args(argv)


def launch_ranks(args) -> int:
    """`--gpus N` outside a launcher: N fresh rank processes (torch.distributed.run, 127.0.0.1),
    started before this process touches the GPU; returns their exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={args.master_port}", str(Path(__file__).resolve()),
           *sys.argv[1:]]
    return subprocess.call(cmd, env={**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0"})


def flops_per_sample(variant: str) -> float:
    # PriGumbel iteration = pass-1 fwd + pass-2 fwd+bwd = 4F; PriConcat step = fwd+bwd = 3F
    return (4.0 if variant == "prigumbel" else 3.0) * F_PER_SAMPLE


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> dict:
    """Host CPUs this process may use: the affinity mask, the cgroup CPU quota (cpu.max; a GPU box shows
    the whole machine in its affinity mask but grants one GPU's share) and OMP_NUM_THREADS."""
    avail = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    threads = min(x for x in (avail, quota, omp) if x)
    return {"threads": threads, "affinity": avail, "cgroup_quota": quota, "omp_num_threads": omp}


def cpu_baseline(variant: str, batch: int, iters: int, warm_batch: int = 0, budget_s: float = 0.0) -> dict:
    """The CPU oracle (torch fp32 restatement, oracle/fusion_oracle.py; pinned against the reference's
    own outputs by tests/test_oracle_golden.py) timed on the host cores on a bounded sample of the
    same iteration: the bench's batch (256), dropout 0.1 at every reference site as on the GPU leg,
    PriConcat with the honoured feature_all_lap mechanism, one warm-up iteration then `iters` timed.
    Threads = the CPUs this process may run on (sched_getaffinity), capped by the cgroup quota and
    OMP_NUM_THREADS (the GPU box's CPU share): cpu_share().  budget_s > 0: stop after the last timed
    iteration whose successor, at the mean iteration time so far, would end more than budget_s after
    process start (at least one iteration always runs); the line states how many ran."""
    import torch
    import torch.nn.functional as F
    from oracle import fusion_oracle as O

    def progress(msg):
        print(f"[bench cpu_baseline] {msg}", file=sys.stderr, flush=True)

    share = cpu_share()
    avail, threads = share["affinity"], share["threads"]
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    O.set_dropout_replay(lambda site, x: F.dropout(x, 0.1, training=True))
    shapes = O.param_shapes("W", "prigumbel" if variant == "prigumbel" else "priconcat")
    p = {}
    for k, s in shapes.items():
        if ("LayerNorm" in k or ".norm" in k) and k.endswith("weight"):
            t = torch.ones(s)
        elif len(s) >= 2:
            t = torch.randn(s, generator=g) * 0.02
        else:
            t = torch.zeros(s)
        p[k] = t.requires_grad_()
    def make_batch(n):
        eeg = torch.randn(n, C, L, generator=g)
        act = torch.randn(n, A, generator=g) * 0.5
        return dict(eeg=eeg, act=act), (torch.rand(n, generator=g) < 0.66).long()

    model_p = [v for k, v in p.items() if k != "DP"]
    mopt = torch.optim.Adam(model_p, lr=1e-6)
    dopt = torch.optim.Adam([p["DP"]], lr=1e-6) if "DP" in p else None
    lap = torch.distributions.laplace.Laplace(torch.tensor([0.0]), torch.tensor([1.0]))

    def draws(n):
        noise = lap.sample((n, 3 * HID)).view(n, 3 * HID)
        gm = -torch.empty(2, n, 3 * HID).exponential_().log()
        return noise, gm

    def iteration(batch_d, labels):
        nb = labels.shape[0]
        if variant == "prigumbel":
            dopt.zero_grad()
            with torch.no_grad():
                pooled, img, cross = O.encoders(p, batch_d, O.PathConfig(contract="W"))
            n, gm = draws(nb)
            f = O.minmax(torch.cat((pooled, img, cross), 1))
            logits = O.head(p, O.prigumbel_gate(f, p["DP"], n, gm, 1.0, "newfrac", False))
            O.cal_loss(logits, labels)[0].backward()
            dopt.step()
            mopt.zero_grad()
            n, gm = draws(nb)
            pc = O.PathConfig(contract="W", variant="prigumbel", hard=True)
            O.cal_loss(O.forward(p, batch_d, pc, noise=n, gumbels=gm), labels)[0].backward()
            mopt.step()
        else:
            mopt.zero_grad()
            pc = O.PathConfig(contract="W", variant="priconcat", honor_dp_mode=True)
            row = lap.sample((nb,)).view(nb)
            torch.nn.functional.cross_entropy(O.forward(p, batch_d, pc, row_noise=row), labels).backward()
            mopt.step()

    # a heartbeat line every 30 s: one batch-256 iteration runs for minutes with nothing else to say
    import threading
    t_start, done = time.perf_counter(), threading.Event()

    def heartbeat():
        while not done.wait(30.0):
            progress(f"... {time.perf_counter() - t_start:.0f} s")

    threading.Thread(target=heartbeat, daemon=True).start()
    warm_batch = warm_batch or batch
    warm_d, warm_l = make_batch(warm_batch)
    batch_d, labels = make_batch(batch)
    try:
        progress(f"{variant} batch {batch}, {threads} threads: warm-up at batch {warm_batch}")
        t0 = time.perf_counter()
        iteration(warm_d, warm_l)                      # warm-up (allocations, thread pool)
        warm = time.perf_counter() - t0
        del warm_d, warm_l
        t0 = time.perf_counter()
        done_iters = 0
        for i in range(iters):
            iteration(batch_d, labels)
            done_iters += 1
            now = time.perf_counter()
            progress(f"iteration {i + 1}/{iters}: {now - t0:.1f} s")
            if budget_s > 0 and done_iters < iters and (now - T_ORIGIN) + (now - t0) / done_iters > budget_s:
                progress(f"budget: stopping after {done_iters} iteration(s), {now - T_ORIGIN:.0f} s since start")
                break
        dt = time.perf_counter() - t0
    finally:
        done.set()
        O.set_dropout_replay(None)
    out = {"value": round(batch * done_iters / dt, 4), "unit": "samples/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(), "cpus_available": avail, "cpu_share": share, "batch": batch,
           "timed_iterations": done_iters, "seconds_per_iteration": round(dt / done_iters, 2),
           "warmup_seconds": round(warm, 2),
           "sample": f"oracle/fusion_oracle.py {variant} iteration (torch CPU fp32, dropout 0.1"
                     f"{', feature_all_lap honoured' if variant != 'prigumbel' else ''}), batch {batch}, "
                     f"64x256 EEG + 32-d action, {done_iters} timed iteration(s) after 1 warm-up"
                     f"{f' at batch {warm_batch}' if warm_batch != batch else ''}, {dt:.1f} s timed"}
    if done_iters < iters:
        out["deviation"] = (f"{done_iters} of {iters} timed iterations: the next one would have ended past the "
                            f"{budget_s:.0f} s run budget (bench.py --cpu-budget)")
    return out


def hbm_kernel_graph_times(dev, B: int, adam_elems: int, seed: int, reps: int = 20, replays: int = 5) -> dict:
    """Per-launch device time of the small HBM-bound kernels at the bench's shapes, from a hipGraph of
    `reps` back-to-back launches replayed `replays` times (torch.cuda.graph: the C-ABI calls enqueue on
    the capture stream).  In the step these kernels are launch-latency bound and a HIP-event pair around
    one of them also times the host's launch gap; the graph replay removes the host, leaving the kernel
    plus one kernel boundary (~1.1-1.5 us, MI355X_MICROARCH.md).  Synthetic inputs of the step's shapes;
    the same kernels and arguments as the engine's calls (engine.py fuse_head_fwd / _bwd, ln_fwd, the
    trainer's CE and FlatAdam)."""
    import math
    import torch
    from eegfusion import _lib
    F32, BF16 = _lib.F32, _lib.BF16

    def P(t):
        return None if t is None else t.data_ptr()

    def st():
        return torch.cuda.current_stream().cuda_stream

    g = torch.Generator(device=dev).manual_seed(7)
    r = lambda *s: torch.randn(*s, generator=g, device=dev)
    pooled, vis, cross = r(B, HID), r(B, HID), r(B, HID)
    DP = r(1, 3 * HID) * 0.1
    gout, xn = torch.empty(B, 3 * HID, device=dev), torch.empty(B, 3 * HID, device=dev)
    amin, amax = torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev)
    rng = torch.empty(B, device=dev)
    dg, ddp = r(B, 3 * HID), torch.empty(B, 3 * HID, device=dev)
    dp_, dv_, dc_ = (torch.empty(B, HID, device=dev) for _ in range(3))
    logits, labels = r(B, 2), (torch.rand(B, generator=g, device=dev) < 0.66).long()
    loss, correct, dl = torch.empty(1, device=dev), torch.empty(1, dtype=torch.int32, device=dev), torch.empty(B, 2, device=dev)
    R = B * L
    x, res = r(R, HID).bfloat16(), r(R, HID).bfloat16()
    gam, bet = torch.ones(HID, device=dev), torch.zeros(HID, device=dev)
    y, ssum = torch.empty(R, HID, device=dev, dtype=torch.bfloat16), torch.empty(R, HID, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(R, device=dev), torch.empty(R, device=dev)
    n = int(adam_elems)
    pw, gw, mw, vw = r(n) * 0.02, r(n) * 1e-3, torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
    ea = math.exp(1.0)
    calls = {
        "fusion_fwd": (lambda: _lib.call("eegf_fusion_fwd", F32, B, _lib.FUSE_PRIGUMBEL, P(pooled), HID, P(vis), HID,
                                         P(cross), HID, P(DP), None, None, None, 1, 0, ea, 1.0, seed, 200, P(gout),
                                         P(xn), P(amin), P(amax), P(rng), st()),
                       B * (3 * 3 * HID * 4 + 12) + 3 * HID * 4),
        # the pass-1 form: the per-row DP gradient written too (pass 2's has no DP gradient)
        "fusion_bwd": (lambda: _lib.call("eegf_fusion_bwd", F32, B, _lib.FUSE_PRIGUMBEL, P(dg), P(xn), P(amin), P(amax),
                                         P(rng), P(DP), None, None, 0, 0, ea, seed, 200, P(dp_), HID, P(dv_), HID,
                                         P(dc_), HID, P(ddp), st()),
                       B * (4 * 3 * HID * 4 + 12) + 3 * HID * 4),
        "cross_entropy": (lambda: _lib.call("eegf_cross_entropy", F32, B, 2, P(logits), P(labels), 0, 1.0, P(loss),
                                            P(correct), P(dl), st()),
                          2 * B * 2 * 4 + B * 8 + 8),
        # pass 2's form: dropout + residual + LN, the pre-LN sum and the row statistics saved
        "ln_fwd768": (lambda: _lib.call("eegf_ln_fwd", BF16, R, HID, P(x), P(res), None, 1, None, P(gam), P(bet), 1e-12,
                                        0.1, 1, seed, 11, P(y), P(ssum), P(mean), P(rstd), st()),
                      R * HID * 2 * 4 + R * 8 + 2 * HID * 4),
        "adam": (lambda: _lib.call("eegf_adam", n, P(pw), P(gw), P(mw), P(vw), P(sh), 1e-6, 0.9, 0.999, 1e-8, 0.0, 1.0,
                                   1, st()),
                 n * 30),
    }
    out = {}
    for tag, (fn, nbytes) in calls.items():
        reps_t = max(4, reps // 4) if tag == "adam" else reps
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()                                    # warm (outside the graph)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            for _ in range(reps_t):
                fn()
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(replays):
            graph.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (replays * reps_t)
        out[tag] = {"us": us, "bytes": nbytes}
        del graph
    return out


def load_profile_json(name: str, tag: str):
    f = ROOT / "profiles" / name
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text()).get(tag)
    except Exception:
        return None


def probe_stats(probe: dict) -> dict:
    out = {}
    for tag, v in probe.items():
        if not v:
            continue
        ms = [s.elapsed_time(e) for s, e, _, _ in v]
        fl = sum(x[2] for x in v)
        by = sum(x[3] for x in v)
        out[tag] = {"launches": len(v), "avg_ms": sum(ms) / len(ms), "tflops": fl / (sum(ms) * 1e-3) / 1e12,
                    "flops_per_launch": fl / len(v)}
        if by > 0:
            out[tag].update(bytes_per_launch=by / len(v), gbps=by / (sum(ms) * 1e-3) / 1e9)
    return out


def main():
    args = parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world_env = int(env_world or "1")
    if world_env != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}; refusing to report a mismatched run",
              file=sys.stderr)
        sys.exit(2)

    sys.path.insert(0, str(ROOT / "eeg-multimodal_amd"))
    sys.path.insert(0, str(ROOT))
    if args.cpu_baseline_only:
        cb = cpu_baseline(args.variant, args.cpu_batch, args.cpu_iters, args.cpu_warm_batch)
        print(json.dumps(cb), flush=True)
        if args.cpu_baseline_out:
            f = Path(args.cpu_baseline_out)
            d = json.loads(f.read_text()) if f.exists() else {}
            d[args.variant] = cb
            f.write_text(json.dumps(d, indent=1) + "\n")
        return
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world, backend = 1, None
    if args.selftest:
        if world_env > 1:
            dist.init_process_group("gloo")
        w = dist.get_world_size() if world_env > 1 else 1
        t = torch.ones(1)
        if w > 1:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"selftest": True, "world_size": w, "allreduce": float(t.item()),
                              "backend": dist.get_backend() if w > 1 else None}), flush=True)
        if w > 1:
            dist.destroy_process_group()
        return
    # nccl: one GPU per rank (LOCAL_RANK); gloo may put several ranks on one GPU (device_count()
    # does not initialise the GPU)
    ndev = torch.cuda.device_count() if args.dist_backend == "gloo" else 0
    dev_idx = local % max(1, ndev) if args.dist_backend == "gloo" else local
    if world_env > 1:
        torch.cuda.set_device(dev_idx)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group("gloo")
        world, backend = dist.get_world_size(), dist.get_backend()
        if world != args.gpus:
            print(f"bench.py: process group has {world} ranks, --gpus {args.gpus}", file=sys.stderr)
            sys.exit(2)
    dev = torch.device("cuda", dev_idx)

    from eegfusion.modules import PriConcatModel, PriGumbelModel
    from eegfusion.trainer import GradReducer, PriGumbelTrainer, SinglePassTrainer

    sweep = [float(x) for x in args.eps_sweep.split(",") if x.strip()] or [args.eps]
    torch.manual_seed(980616)                              # identical init on every rank
    if args.variant == "prigumbel":
        model = PriGumbelModel(sweep[0], contract="W", eps_mode=args.eps_mode, dropout=0.1, seed=980616 + rank)
    else:
        # configs[1] "PriConcat eps=1.0": the feature_all_lap mechanism honoured so eps
        # takes effect (main_0430.py:118 passes dp_mode=None, which would make it an identity)
        model = PriConcatModel(types.SimpleNamespace(EPSILON=1.0), dp_mode="feature_all_lap", honor_dp_mode=True,
                               contract="W", dropout=0.1, seed=980616 + rank)
    model = model.to(dev).set_compute_dtype(torch.bfloat16)
    eng = model.engine
    reducer = GradReducer(scale_in_optimizer=True)     # 1/N applied inside the fused Adam
    trainer_cls = PriGumbelTrainer if args.variant == "prigumbel" else SinglePassTrainer

    B = args.batch
    g = torch.Generator(device=dev).manual_seed(980616 + 7919 * rank)   # disjoint synthetic shard per rank
    eeg = torch.randn(B, C, L, generator=g, device=dev)
    act = torch.randn(B, A, generator=g, device=dev) * 0.5
    labels = (torch.rand(B, generator=g, device=dev) < 0.66).long()
    batch = {"eeg": eeg, "act": act}

    feawei = None
    if args.feawei > 0 and args.variant == "prigumbel":
        from eegfusion.feawei import FeatureMean
        # forward-only pass (train mode, hard=False) over this rank's shard of args.feawei samples,
        # column sums all-reduced so every rank initialises the same DP
        per_rank = (args.feawei + world - 1) // world
        acc = FeatureMean(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.no_grad():
            for i in range(0, per_rank, B):
                nb = min(B, per_rank - i)
                fb = {"eeg": torch.randn(nb, C, L, generator=g, device=dev),
                      "act": torch.randn(nb, A, generator=g, device=dev) * 0.5}
                _, sv = eng.forward(fb, False, True, save=False)
                acc.add(sv.t["fuse"]["xn"])
            if world > 1:
                dist.all_reduce(acc.sum)
                acc.count *= world
            dp0 = acc.dp_init(k=1.0, zscore=True)
        torch.cuda.synchronize()
        feawei = {"samples": acc.count, "seconds": round(time.perf_counter() - t0, 3), "k": 1.0, "zscore": True}

    tags = tuple(KERNEL_GROUPS)
    total_dt, per_eps, loss = 0.0, [], None
    probe_all = {t: [] for t in tags}
    for eps in sweep:
        eng.cfg.eps = eps
        model.eps = torch.tensor(eps)
        if feawei is not None:
            model.DP.data.copy_(dp0)
        trainer = trainer_cls(eng, lr=1e-6, reducer=reducer)      # fresh Adam state per run
        for _ in range(args.warmup):
            trainer.step(batch, labels)
        # the HIP-event probes cost ~1.3 ms per probed step (an event pair around ~230 launches,
        # profiles/r5l_probe_cost.log), so they are live only on the last steps of the timed region
        # (one in ten, at least one): the per-kernel averages come from the timed region, and the
        # step time carries ~0.1 ms of probe cost per step instead of 1.3
        n_probe = 0 if args.no_probe else max(1, args.steps // 10)
        probe_on = {t: [] for t in tags}
        eng.probe = None
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            if i == args.steps - n_probe:
                eng.probe = probe_on
            loss, _ = trainer.step(batch, labels)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = t.item()
        for t in tags:
            probe_all[t] += probe_on[t]
        eng.probe = None
        total_dt += dt
        per_eps.append({"eps": eps, "samples_per_s": round(world * B * args.steps / dt, 2),
                        "ms_per_step": round(dt / args.steps * 1e3, 3), "loss": float(loss[-1].item())})

    # the small HBM-bound kernels timed by hipGraph replay (after the timed region; no effect on value)
    hbm_times = {}
    if world == 1 and not args.no_probe:
        try:
            adam_elems = sum(hi - lo for lo, hi in trainer.model_opt.sub) if hasattr(trainer, "model_opt") else \
                sum(hi - lo for lo, hi in trainer.opt.sub)
            hbm_times = hbm_kernel_graph_times(dev, B, adam_elems, eng.cfg.seed)
        except Exception as exc:          # a diagnostic leg: report, never fail the bench line
            print(f"[bench] hbm kernel graph timing failed: {exc!r}", file=sys.stderr)

    replicas = None
    if args.check_replicas:
        torch.cuda.synchronize()
        h = hashlib.sha256(eng.a.master.cpu().numpy().tobytes())
        for opt in (getattr(trainer, "model_opt", None), getattr(trainer, "dp_opt", None), getattr(trainer, "opt", None)):
            if opt is not None:
                h.update(opt.m.cpu().numpy().tobytes())
                h.update(opt.v.cpu().numpy().tobytes())
        digests = [None] * world
        if world > 1:
            dist.all_gather_object(digests, h.hexdigest())
        else:
            digests = [h.hexdigest()]
        replicas = {"identical": len(set(digests)) == 1, "sha256": digests[0][:16], "ranks": world}

    if rank == 0:
        steps = args.steps * len(sweep)
        probed_steps = max(1, (0 if args.no_probe else max(1, args.steps // 10)) * len(sweep))
        value = world * B * steps / total_dt
        ks = probe_stats(probe_all)
        step_tf = value / world * flops_per_sample(args.variant) / 1e12
        # the dominant kernel: the rocprof symbol with the largest total probed time in this run (the groups
        # that share a symbol combined: achieved = their FLOPs / their time), with that symbol's PMC traffic
        sym_stats = {}
        for sym, d in KERNEL_SYMBOLS.items():
            parts = [ks[t] for t in d["tags"] if t in ks]
            if not parts:
                continue
            n = sum(p["launches"] for p in parts)
            ms = sum(p["avg_ms"] * p["launches"] for p in parts)
            fl = sum(p["flops_per_launch"] * p["launches"] for p in parts)
            by = d.get("bytes")
            alg = (sum(by[t] * ks[t]["launches"] for t in d["tags"] if t in ks) / n) if by else None
            sym_stats[sym] = {"launches": n, "ms": ms, "flops_per_launch": fl / n, "avg_ms": ms / n,
                              "tflops": fl / (ms * 1e-3) / 1e12, "alg_bytes": alg}
        dom_sym = max(sym_stats, key=lambda k: sym_stats[k]["ms"]) if sym_stats else None
        dom = sym_stats.get(dom_sym)
        pmc = load_profile_json(PMC_FILE, KERNEL_SYMBOLS[dom_sym]["pmc"]) if dom else None
        pmc = pmc or {}
        roofline = {"kernel": (f"{dom_sym}: {KERNEL_SYMBOLS[dom_sym]['what']} (the kernel with the most time per "
                               f"step in this run: {dom['ms'] / probed_steps:.2f} ms over {dom['launches'] / probed_steps:.0f} "
                               f"launches; probe groups {', '.join(KERNEL_SYMBOLS[dom_sym]['tags'])})")
                    if dom else None,
                    "bound": "mfma", "achieved": round(dom["tflops"], 1) if dom else None, "peak": PEAK_BF16,
                    "unit": "TFLOP/s", "frac": round(dom["tflops"] / PEAK_BF16, 4) if dom else None,
                    "traffic": pmc.get("hbm_bytes_per_launch"),
                    "algorithmic_bytes_per_launch": dom["alg_bytes"] if dom else None,
                    "mfma_busy": pmc.get("mfma_busy"), "pmc_round": pmc.get("round"),
                    "avg_ms": round(dom["avg_ms"], 4) if dom else None,
                    "flops_per_launch": dom["flops_per_launch"] if dom else None}
        kernels_by_symbol = {k: {"ms_per_step": round(v["ms"] / probed_steps, 3), "avg_ms": round(v["avg_ms"], 4),
                                 "tflops": round(v["tflops"], 1), "frac": round(v["tflops"] / PEAK_BF16, 4)}
                             for k, v in sorted(sym_stats.items(), key=lambda kv: -kv[1]["ms"])}
        f1p = [ks[t] for t in ("ffn1_fwd", "ffn1_fwd_gd") if t in ks]     # both FFN1 forms (pass 1, pass 2)
        f1 = None
        if f1p:
            n1 = sum(p["launches"] for p in f1p)
            ms1 = sum(p["avg_ms"] * p["launches"] for p in f1p)
            f1 = {"avg_ms": ms1 / n1, "tflops": sum(p["flops_per_launch"] * p["launches"] for p in f1p) / (ms1 * 1e-3) / 1e12}
        ffn1 = load_profile_json(PMC_FILE, "ffn1_fwd") or {}
        hbm = {}
        for t in HBM_TAGS:
            gt = hbm_times.get(t)
            if not gt:
                continue
            gbps = gt["bytes"] / (gt["us"] * 1e-6) / 1e9
            e = {"avg_us": round(gt["us"], 2), "alg_bytes_per_launch": int(gt["bytes"]), "achieved": round(gbps, 1),
                 "peak": PEAK_HBM, "unit": "GB/s", "frac": round(gbps / PEAK_HBM, 4), "what": KERNEL_GROUPS[t],
                 "timing": "hipGraph replay of back-to-back launches at the step's shapes (kernel + one boundary)",
                 "graph_replay": {"avg_us": round(gt["us"], 2), "alg_bytes_per_launch": int(gt["bytes"]),
                                  "achieved": round(gbps, 1)}}
            if t in ks:
                e["launches_per_step"] = round(ks[t]["launches"] / probed_steps, 2)
                e["in_step_event_us"] = round(ks[t]["avg_ms"] * 1e3, 2)   # includes the host's launch gap
                ib = ks[t].get("bytes_per_launch")
                if ib and ks[t]["avg_ms"] > 0:
                    ig = ib / (ks[t]["avg_ms"] * 1e-3) / 1e9
                    e["in_step"] = {"avg_us": round(ks[t]["avg_ms"] * 1e3, 2), "alg_bytes_per_launch": int(ib),
                                    "achieved": round(ig, 1)}
                    # kernels of >= 40 us: the step's own events (its real mix of forms and buffers; the host's
                    # launch gap is small against them) are the primary figure; back-to-back graph replays of
                    # one long streaming kernel ran 20-40 % slower than the same kernel in the step
                    if ks[t]["avg_ms"] * 1e3 >= 40.0:
                        e.update(avg_us=round(ks[t]["avg_ms"] * 1e3, 2), alg_bytes_per_launch=int(ib),
                                 achieved=round(ig, 1), frac=round(ig / PEAK_HBM, 4),
                                 timing="the step's own HIP events on the launch stream (>= 40 us per launch)")
            p = load_profile_json(PMC_FILE, t)
            if p:
                e.update(traffic=p.get("hbm_bytes_per_launch"), pmc_round=p.get("round"))
            hbm[t] = e
        # non-default routing switches: the symbol names above assume the default routes
        routing_env = {k: v for k, v in os.environ.items()
                       if k.startswith("EEGF_") and k not in ("EEGF_LIB", "EEGF_BERT_WEIGHTS")}
        if routing_env:
            roofline["routing"] = ("assumed default routing; EEGF_* switches set: " +
                                   ", ".join(f"{k}={v}" for k, v in sorted(routing_env.items())))
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(total_dt / steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": ("PriGumbel eps=%s %s iteration (past_acc.py:194-212): pass-1 fwd + DP Adam, "
                                    "pass-2 fwd/bwd + model Adam" % (",".join(map(str, sweep)), args.eps_mode)
                                    if args.variant == "prigumbel" else
                                    "PriConcat eps=1.0 step (main_0430.py): fwd/bwd + Adam"),
                       "global_batch": world * B, "per_gpu_batch": B, "seq_len": L, "eeg": f"{C}ch x {L}",
                       "action_dim": A, "encoder": "BERT-base 12x768 over per-step Linear(64,768) tokens",
                       "parallelism": f"dp{world}", "process_group": {"world_size": world, "backend": backend}},
            "roofline": roofline,
            "roofline_ffn1": ({"kernel": "ffn1_fwd (BertIntermediate GEMM + bias + GELU)", "bound": "mfma",
                               "achieved": round(f1["tflops"], 1), "peak": PEAK_BF16, "unit": "TFLOP/s",
                               "frac": round(f1["tflops"] / PEAK_BF16, 4), "avg_ms": round(f1["avg_ms"], 4),
                               "traffic": ffn1.get("hbm_bytes_per_launch"), "mfma_busy": ffn1.get("mfma_busy"),
                               "pmc_round": ffn1.get("round")} if f1 else None),
            "step_roofline": {"achieved": round(step_tf, 1), "unit": "TFLOP/s", "frac": round(step_tf / PEAK_BF16, 4),
                              "flops_per_sample": flops_per_sample(args.variant)},
            "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in ks.items()},
            "kernels_by_symbol": kernels_by_symbol,
            "hbm_kernels": hbm,
            "loss": float(loss[-1].item()),
        }
        if len(sweep) > 1 or feawei is not None:
            out["sweep"] = per_eps
            out["feawei"] = feawei
        if replicas is not None:
            out["replicas"] = replicas
        if world == 1 and not args.no_cpu_baseline:
            # batch 256 (the GPU leg's batch), 1 warm-up + 3 timed iterations, in this run;
            # the stderr heartbeat every 30 s keeps the ~5.5 min leg visibly alive
            cb = cpu_baseline(args.variant, args.cpu_batch, args.cpu_iters, args.cpu_warm_batch, args.cpu_budget)
            if args.cpu_batch != B:
                cb["deviation"] = (cb.get("deviation", "") + "; " if "deviation" in cb else "") + (
                    f"sample at batch {args.cpu_batch}, the GPU leg runs batch {B} (--cpu-batch)")
            # an earlier separate run of the same sample on a GPU box (bench.py --cpu-baseline-only): a cross-check
            ref = load_profile_json("cpu_baseline_b256.json", args.variant)
            if ref:
                cb["crosscheck_b256_separate_run"] = {k: ref[k] for k in ("value", "seconds_per_iteration", "sample")
                                                      if k in ref}
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
