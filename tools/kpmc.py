"""Raw per-kernel PMC averages from rocprofv3 counter passes (one directory per pass).

usage: python tools/kpmc.py <name-substring>[,<substring>...] <pass_dir> [<pass_dir> ...]

Prints, per kernel whose name contains one of the substrings, the per-dispatch mean of every
counter collected in the passes, plus derived stall shares: with W = SQ_WAVE_CYCLES (quad-cycles),
SQ_WAIT_ANY / W (parked on waitcnt / barrier), SQ_WAIT_INST_ANY / W (issue stall: dependency or
pipe busy), SQ_ACTIVE_INST_ANY / W (issuing); SQ_ACTIVE_INST_VALU / SQ_ACTIVE_INST_LDS etc. / W;
LDS busy = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE/8 x CUs) when both are present."""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def load(d):
    cc = next(Path(d).rglob("*counter_collection.csv"), None)
    if cc is None:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(lambda: defaultdict(float))     # (kernel, dispatch) -> counter -> value
    with open(cc) as f:
        for r in csv.DictReader(f):
            k = (r["Kernel_Name"], r["Dispatch_Id"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return per


def main():
    subs = sys.argv[1].split(",")
    agg = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[2:]:
        for (name, _), cs in load(d).items():
            if any(s in name for s in subs):
                for c, v in cs.items():
                    agg[name][c].append(v)
    for name, cs in agg.items():
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        print(f"== {name[:110]}  ({n} dispatches)")
        for c in sorted(mean):
            print(f"   {c:32s} {mean[c]:16.1f}")
        W = mean.get("SQ_WAVE_CYCLES")
        if W:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_VMEM"):
                if c in mean:
                    print(f"   {c + ' / WAVE_CYCLES':45s} {mean[c] / W:8.3f}")
        if "SQ_LDS_IDX_ACTIVE" in mean and "GRBM_GUI_ACTIVE" in mean:
            print(f"   {'LDS busy (IDX_ACTIVE / CU-cycles)':45s} {mean['SQ_LDS_IDX_ACTIVE'] / (mean['GRBM_GUI_ACTIVE'] / 8 * 256):8.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and "GRBM_GUI_ACTIVE" in mean:
            print(f"   {'MFMA busy':45s} {mean['SQ_VALU_MFMA_BUSY_CYCLES'] / (mean['GRBM_GUI_ACTIVE'] / 8 * 1024):8.3f}")
        if "SQ_INSTS_VALU" in mean and "SQ_INSTS_MFMA" in mean and mean["SQ_INSTS_MFMA"]:
            print(f"   {'VALU / MFMA instructions':45s} {mean['SQ_INSTS_VALU'] / mean['SQ_INSTS_MFMA']:8.2f}")


if __name__ == "__main__":
    main()
