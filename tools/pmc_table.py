"""Per-kernel PMC table (MFMA busy, VALU/MFMA instruction mix, LDS conflicts, HBM bytes) from
rocprofv3 counter passes over the same bench command.

usage: python tools/pmc_table.py <tag> <steps traced> <pass_dir> [<pass_dir> ...]

Each <pass_dir> holds one `rocprofv3 --kernel-trace --pmc ... --output-format csv` run
(`*counter_collection.csv` and `*kernel_trace.csv`).  Launches are grouped by (kernel, grid), so
GEMM shapes that share a kernel symbol stay apart.  Per group and per launch:

  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
              (BUSY counts SIMD cycles, 32 per v_mfma_f32_32x32x16_bf16; GRBM_GUI_ACTIVE is summed
              over the 8 XCDs — MI355X_MICROARCH.md, cycle constants and DVFS notes)
  hbm_bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024   (gfx950: FETCH_SIZE counts half the bytes of
              16-B-per-lane streaming reads — MI355X_MICROARCH.md §HBM)
  clock_ghz = GRBM_GUI_ACTIVE / 8 / duration, per dispatch with both from the SAME pass (median over
              dispatches), and only for kernels of >= 50 us: GRBM_GUI_ACTIVE counts the counter window,
              which for short kernels is longer than the kernel (the r2 tables divided one pass's
              counter by another pass's durations and printed impossible > 3 GHz rows)

Writes profiles/<tag>_pmc_table.md and profiles/pmc_<tag>.json (read by bench.py: roofline traffic and
mfma_busy of the named kernel groups).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
N_SIMD = 1024

# bench.py roofline groups -> kernel-name fragments (mangled or demangled) + grid filters
GROUPS = {     # bf16 instantiations appear mangled in rocprofv3's CSV (DF16b), the others demangled
    # round 3: every BERT forward / input gradient runs on the persistent kernel gemm4p<BKC, EPI, ACC>;
    # its grid is one workgroup per CU for every shape, so the three bias-only forwards share a row
    "ffn1_fwd": ("gemm8_kernelILb1ELb1ELi2EDF16bLb0E", "gemm8_kernelILb1ELb1ELi8EDF16bLb0E",
                 "gemm4p_kernel<true, 2, false>", "gemm4p_kernel<true, 8, false>",
                 "gemm4p_kernelILb1ELi2ELb0E", "gemm4p_kernelILb1ELi8ELb0E",
                 # round 4: the K-contiguous forwards run on gemm4q (K-tile pairs in whole lines)
                 "gemm4q_kernel<true, 2, false>", "gemm4q_kernel<true, 8, false>",
                 # round 5: gemm4r (rolling A fragments) replaces gemm4q
                 "gemm4r_kernel<true, 2, false>", "gemm4r_kernel<true, 8, false>"),
    "fwd_bias_qkv_ao_ffn2": ("gemm4p_kernel<true, 1, false>", "gemm4p_kernelILb1ELi1ELb0E",
                             "gemm4q_kernel<true, 1, false>", "gemm4r_kernel<true, 1, false>"),
    "qkv_fwd": ("gemm8_kernelILb1ELb1ELi1EDF16bLb0E",),
    "ffn2_fwd": ("gemm4w_kernelILb1ELb1ELi1EDF16bLb0E",),
    "dgrad_qkv_ffn1": ("gemm4w_kernelILb1ELb0ELi0EDF16bLb0E", "gemm4p_kernel<false, 0, true>",
                       "gemm4p_kernelILb0ELi0ELb1E", "gemm4q_kernel<false, 0, true>",
                       "gemm4r_kernel<false, 0, true>"),
    "ao_fwd": ("gemm4h_kernelILb1ELi1E", "gemm4h_kernel<true, 1>"),
    "dgrad_out": ("gemm4h_kernelILb0ELi0E", "gemm4h_kernel<false, 0>", "gemm4p_kernel<false, 0, false>",
                  "gemm4p_kernelILb0ELi0ELb0E", "gemm4q_kernel<false, 0, false>",
                  "gemm4r_kernel<false, 0, false>"),
    "dgrad_ffn2": ("gemm8_kernelILb1ELb0ELi9EDF16bLb0E", "gemm4p_kernel<false, 9, false>", "gemm4p_kernelILb0ELi9ELb0E",
                   "gemm4q_kernel<false, 9, false>", "gemm4r_kernel<false, 9, false>"),
    "wgrad": ("gemm4w_kernel<false, false, 0, float, true", "gemm4w_kernelILb0ELb0ELi0EfLb1E"),
    "attn_fwd": ("attn_fwd256_kernel",),
    "attn_bwd": ("attn_bwd256_kernel",),
    "ln_fwd": ("ln_fwd_kernel", "ln_fwd768_kernel"),
    "ln_bwd": ("ln_bwd_kernel",),
    # the HBM-bound kernels bench.py reports in GB/s (its hbm_kernels object)
    "fusion_fwd": ("fusion_fwd_kernel",),
    "fusion_bwd": ("fusion_bwd_kernel",),
    "cross_entropy": ("ce_kernel",),
    "ln_fwd768": ("ln_fwd768_kernel",),
    "adam": ("adam_kernel",),
}
HBM_GROUPS = ("fusion_fwd", "fusion_bwd", "cross_entropy", "ln_fwd768", "adam")
# bench.py probes the QKV and FFN1 input gradients separately; they share one kernel and grid here
# (and, on the persistent kernel, the three bias-only forwards share one)
ALIASES = {"dgrad_qkv": "dgrad_qkv_ffn1", "dgrad_ffn1": "dgrad_qkv_ffn1", "qkv_fwd": "fwd_bias_qkv_ao_ffn2",
           "ffn2_fwd": "fwd_bias_qkv_ao_ffn2", "ao_fwd": "fwd_bias_qkv_ao_ffn2"}


def short(name):
    return name if len(name) < 96 else name[:93] + "..."


def read_pass(d):
    d = Path(d)
    cc = next(d.rglob("*counter_collection.csv"), None)
    kt = next(d.rglob("*kernel_trace.csv"), None)
    dur = {}
    if kt is not None:
        for r in csv.DictReader(open(kt)):
            dur[r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    per = defaultdict(dict)          # dispatch -> {counter: value, _name, _grid}
    if cc is None:
        return per, dur
    for r in csv.DictReader(open(cc)):
        k = r["Dispatch_Id"]
        e = per[k]
        e["_name"] = r["Kernel_Name"]
        e["_grid"] = r.get("Grid_Size", "")
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if "Start_Timestamp" in r and r.get("End_Timestamp"):
            dur.setdefault(k, float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return per, dur


def main():
    tag, steps, dirs = sys.argv[1], float(sys.argv[2]), sys.argv[3:]
    agg = defaultdict(lambda: defaultdict(float))     # (name, grid) -> counter sums
    cnt = defaultdict(lambda: defaultdict(int))       # (name, grid) -> launches seen per counter
    tsum = defaultdict(float)
    tn = defaultdict(int)
    clk = defaultdict(list)                           # (name, grid) -> same-pass GUI/8/duration samples
    for d in dirs:
        per, dur = read_pass(d)
        for k, e in per.items():
            key = (e["_name"], e["_grid"])
            if "GRBM_GUI_ACTIVE" in e and dur.get(k):
                clk[key].append(e["GRBM_GUI_ACTIVE"] / 8 / dur[k])
            for c, v in e.items():
                if not c.startswith("_"):
                    agg[key][c] += v
                    cnt[key][c] += 1
            if k in dur:
                tsum[key] += dur[k]
                tn[key] += 1

    def avg(key, c):
        n = cnt[key].get(c, 0)
        return agg[key][c] / n if n else None

    rows = []
    for key in agg:
        if not tn[key]:
            continue
        t_ns = tsum[key] / tn[key]
        launches = max(cnt[key].values()) / max(1, len(dirs))
        gui = avg(key, "GRBM_GUI_ACTIVE")
        busy = avg(key, "SQ_VALU_MFMA_BUSY_CYCLES")
        fetch, write = avg(key, "FETCH_SIZE"), avg(key, "WRITE_SIZE")
        hbm = 2 * fetch * 1024 + write * 1024 if fetch is not None and write is not None else None
        cyc = gui / 8 if gui else None
        cs = sorted(clk[key])
        clock = cs[len(cs) // 2] if cs and t_ns >= 50e3 else None
        rows.append({
            "kernel": key[0], "grid": key[1], "avg_us": t_ns / 1e3,
            "ms_per_step": tsum[key] / tn[key] * (tn[key] / len(dirs)) / steps / 1e6 if tn[key] else None,
            "launches_per_step": tn[key] / len(dirs) / steps,
            "mfma_busy": busy / (N_SIMD * cyc) if busy is not None and cyc else None,
            "clock_ghz": clock,
            "valu_insts": avg(key, "SQ_INSTS_VALU"), "mfma_insts": avg(key, "SQ_INSTS_MFMA"),
            "lds_conflict_frac": (avg(key, "SQ_LDS_BANK_CONFLICT") / avg(key, "SQ_LDS_IDX_ACTIVE")
                                  if avg(key, "SQ_LDS_IDX_ACTIVE") else None),
            "hbm_bytes": hbm, "hbm_gbs": hbm / t_ns if hbm is not None else None,
            "fetch_kb": fetch, "write_kb": write,
            "l2_hit": (avg(key, "TCC_HIT_sum") / (avg(key, "TCC_HIT_sum") + avg(key, "TCC_MISS_sum"))
                       if avg(key, "TCC_HIT_sum") is not None and avg(key, "TCC_MISS_sum") else None),
        })
    rows.sort(key=lambda r: -(r["ms_per_step"] or 0))

    def f(v, fmt):
        return "—" if v is None else format(v, fmt)

    out = [f"# rocprofv3 PMC table — {tag}", "",
           f"bench.py PriGumbel B=256 bf16, {steps:g} iterations traced per pass; passes: "
           + ", ".join(Path(d).name for d in dirs), "",
           "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE/8); HBM = 2 x FETCH_SIZE + WRITE_SIZE; "
           "clock = GRBM_GUI_ACTIVE/8 / duration per dispatch, both from the same pass (median; kernels >= 50 us only)", "",
           "| ms/step | launches/step | avg us | mfma_busy | clock GHz | VALU/MFMA insts | LDS conflict | HBM MB/launch "
           "| HBM GB/s | L2 hit | kernel (grid) |",
           "|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---|"]
    for r in rows[:20]:
        mix = (r["valu_insts"] / r["mfma_insts"]) if r["valu_insts"] and r["mfma_insts"] else None
        out.append(f"| {f(r['ms_per_step'], '.3f')} | {r['launches_per_step']:.1f} | {r['avg_us']:.1f} | "
                   f"{f(r['mfma_busy'], '.3f')} | {f(r['clock_ghz'], '.2f')} | {f(mix, '.2f')} | "
                   f"{f(r['lds_conflict_frac'], '.3f')} | {f(r['hbm_bytes'] and r['hbm_bytes'] / 1e6, '.1f')} | "
                   f"{f(r['hbm_gbs'], '.0f')} | {f(r['l2_hit'], '.3f')} | `{short(r['kernel'])}` ({r['grid']}) |")
    # the small HBM-bound kernels whatever their rank (the top-20 cut drops kernels of a few us)
    out += ["", "HBM-bound kernels (bench.py hbm_kernels): HBM bytes from FETCH_SIZE / WRITE_SIZE as above", "",
            "| ms/step | launches/step | avg us | HBM MB/launch | HBM GB/s | L2 hit | kernel (grid) |",
            "|---:|---:|---:|---:|---:|---:|---|"]
    for r in rows:
        if any(fr in r["kernel"] for g in HBM_GROUPS for fr in GROUPS[g]):
            out.append(f"| {f(r['ms_per_step'], '.3f')} | {r['launches_per_step']:.1f} | {r['avg_us']:.1f} | "
                       f"{f(r['hbm_bytes'] and r['hbm_bytes'] / 1e6, '.2f')} | {f(r['hbm_gbs'], '.0f')} | "
                       f"{f(r['l2_hit'], '.3f')} | `{short(r['kernel'])}` ({r['grid']}) |")
    (ROOT / "profiles" / f"{tag}_pmc_table.md").write_text("\n".join(out) + "\n")
    print("\n".join(out))

    groups = {}
    for g, frags in GROUPS.items():
        sel = [r for r in rows if any(fr in r["kernel"] for fr in frags)]
        if not sel:
            continue
        w = sum(r["launches_per_step"] for r in sel)

        def wavg(field):
            vs = [(r[field], r["launches_per_step"]) for r in sel if r[field] is not None]
            return sum(v * n for v, n in vs) / sum(n for _, n in vs) if vs else None

        groups[g] = {"launches_per_step": w, "avg_us": wavg("avg_us"), "mfma_busy": wavg("mfma_busy"),
                     "hbm_bytes_per_launch": wavg("hbm_bytes"), "clock_ghz": wavg("clock_ghz"),
                     "lds_conflict_frac": wavg("lds_conflict_frac"), "round": tag}
    for a, g in ALIASES.items():
        if g in groups and a not in groups:
            groups[a] = dict(groups[g], alias_of=g)
    (ROOT / "profiles" / f"pmc_{tag}.json").write_text(json.dumps(groups, indent=1) + "\n")
    print(json.dumps(groups, indent=1))


if __name__ == "__main__":
    main()
