"""Per-kernel hardware-counter table (markdown) from rocprofv3 --pmc passes.

    python tools/pmc_table.py DIR [DIR...] [--match a,b,c]

Derived columns (gfx950 conventions of MI355X_MICROARCH.md):
  HBM rd TB/s   2 x FETCH_SIZE (wide streaming reads are tallied at half) / time
  HBM wr TB/s   WRITE_SIZE / time
  MFMA util     SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
  LDS confl.    SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS cycle)
  LDS busy      SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM_GUI_ACTIVE / 8): the share of CU-cycles
                the LDS array was active at all (a high conflict rate on an LDS that is
                almost idle costs nothing)
  L2 hit        TCC_HIT / (TCC_HIT + TCC_MISS)
  L2 lat        TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ (cycles per L1->L2 read)
  wait / busy   SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY as fractions of SQ_WAVE_CYCLES
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def row(name, cs, dur):
    a = {c: sum(v) / len(v) for c, v in cs.items()}
    ds = dur.get(name, [])
    t = sum(ds) / len(ds) / 1e9 if ds else 0.0
    f = lambda k: a.get(k)  # noqa: E731
    cells = [f"{t * 1e6:.1f}" if t else "-"]
    cells.append(f"{2 * f('FETCH_SIZE') * 1024 / t / 1e12:.2f}" if f("FETCH_SIZE") and t else "-")
    cells.append(f"{f('WRITE_SIZE') * 1024 / t / 1e12:.2f}" if f("WRITE_SIZE") and t else "-")
    g = f("GRBM_GUI_ACTIVE")
    cells.append(f"{f('SQ_VALU_MFMA_BUSY_CYCLES') / (1024 * g / 8):.3f}"
                 if f("SQ_VALU_MFMA_BUSY_CYCLES") is not None and g else "-")
    cells.append(f"{f('SQ_LDS_BANK_CONFLICT') / f('SQ_LDS_IDX_ACTIVE'):.3f}"
                 if f("SQ_LDS_IDX_ACTIVE") else "-")
    cells.append(f"{f('SQ_LDS_IDX_ACTIVE') / (256 * g / 8):.4f}"
                 if f("SQ_LDS_IDX_ACTIVE") is not None and g else "-")
    h, m = f("TCC_HIT_sum"), f("TCC_MISS_sum")
    cells.append(f"{h / (h + m):.2f}" if h is not None and m is not None and h + m else "-")
    cells.append(f"{f('TCP_TCC_READ_REQ_LATENCY_sum') / f('TCP_TCC_READ_REQ_sum'):.0f}"
                 if f("TCP_TCC_READ_REQ_sum") else "-")
    w = f("SQ_WAVE_CYCLES")
    cells.append(f"{f('SQ_WAIT_ANY') / w:.2f} / {f('SQ_ACTIVE_INST_ANY') / w:.2f}" if w else "-")
    return cells


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    per, dur = load(a.dirs)
    pats = [p for p in a.match.split(",") if p]
    print("| kernel | us | HBM rd TB/s | HBM wr TB/s | MFMA util | LDS confl. | LDS busy | L2 hit | "
          "L2 lat (cyc) | wait / active |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---|")
    for name, cs in sorted(per.items(), key=lambda kv: -sum(dur.get(kv[0], [0]))):
        if pats and not any(p in name for p in pats):
            continue
        print(f"| `{name[:60]}` | " + " | ".join(row(name, cs, dur)) + " |")


if __name__ == "__main__":
    main()
