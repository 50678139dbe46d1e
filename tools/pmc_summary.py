"""Average rocprofv3 --pmc counters per kernel (counter_collection.csv of one
or more passes) and derive the usual ratios.

    python tools/pmc_summary.py DIR [DIR...] [--filter NAME]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def load(dirs):
    per = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> values
    dur = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r.get("Kernel_Name", "")
                per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return per, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    per, dur = load(a.dirs)
    for k, cs in per.items():
        if a.filter and a.filter not in k:
            continue
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"### `{k[:110]}`  ({len(next(iter(cs.values())))} dispatches)")
        for c in sorted(avg):
            print(f"- {c}: {avg[c]:.4g}")
        if "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
            w = avg["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in avg:
                    print(f"  - {c}/WAVE_CYCLES = {avg[c] / w:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg and avg["GRBM_GUI_ACTIVE"]:
            # MFMA busy cycles summed over CUs (4 SIMDs each) vs GPU active cycles
            print(f"  - MFMA busy per SIMD-cycle = "
                  f"{avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 256 * 4):.3f}")
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            t = avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]
            print(f"  - L2 hit rate = {avg['TCC_HIT_sum'] / t:.3f}" if t else "")
        ds = [d for n, v in dur.items() if n == k for d in v]
        if ds:
            print(f"  - mean duration (profiled) = {sum(ds) / len(ds) / 1e3:.1f} us")
        print()


if __name__ == "__main__":
    main()
