"""Add decode-GEMM dispatch entries for shapes the table does not have yet,
from saved ``dgemm_bench --json`` timing rows (one file per model).  Shapes
already in config/dgemm_gfx950.json keep their (tuned) entries.

    python tools/dg_merge.py gpurun_out/dg_qwen3-8b.json [...] [--margin 0.03]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_mcp_amd.bench.dgemm_bench import table_from_rows  # noqa: E402

PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "llm_mcp_amd", "config", "dgemm_gfx950.json")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("rows", nargs="+")
    ap.add_argument("--margin", type=float, default=0.03)
    a = ap.parse_args()
    with open(PATH) as f:
        doc = json.load(f)
    have = {(e["N"], e["K"], e.get("epi", 0)) for e in doc["entries"]}
    added = []
    for path in a.rows:
        with open(path) as f:
            rows = json.load(f)
        tag = os.path.splitext(os.path.basename(path))[0].removeprefix("dg_")
        for e in table_from_rows(rows, a.margin):
            if (e["N"], e["K"], e["epi"]) in have:
                continue
            e["shape"] = f"{tag}.{e['shape']}"
            e["note"] = "bench/dgemm_bench.py (cold weights), round 6 family sweep"
            added.append(e)
        have |= {(e["N"], e["K"], e["epi"]) for e in added}
    doc["entries"] += added
    with open(PATH, "w") as f:
        json.dump(doc, f, indent=1)
    won = sum(1 for e in added if e["cfg"] >= 0)
    print(f"added {len(added)} entries ({won} hand-written, {len(added) - won} library) "
          f"for {len({(e['N'], e['K'], e['epi']) for e in added})} shapes")
    for e in added:
        if e["cfg"] >= 0:
            print(f"  {e['shape']:24s} M<={e['m_max']:3d} cfg {e['cfg']:4d} S={e['splits']}: "
                  f"{e['us']} us vs lib {e['lib_us']} us")


if __name__ == "__main__":
    main()
