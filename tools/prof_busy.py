"""GPU busy time against wall time for a multi-process run under
``rocprofv3 --kernel-trace -o %pid%`` (one database per process): per process
the kernel count, the union of its kernel intervals and the classes of its top
kernels; over all processes the union of every kernel interval (the one GPU's
busy time) against the span from the first kernel to the last.  Tells a
GPU-bound serving run (union ~ span) from a host- or queue-bound one.

    python tools/prof_busy.py gpurun_out/prof_c5
"""
import glob
import os
import sqlite3
import sys


def intervals(db):
    con = sqlite3.connect(db)
    try:
        rows = con.execute("select name, start, end from kernels").fetchall()
    finally:
        con.close()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(d):
    dbs = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))
    allv, lines = [], []
    for db in dbs:
        rows = intervals(db)
        if not rows:
            continue
        iv = [(s, e) for _, s, e in rows]
        allv += iv
        per = {}
        for n, s, e in rows:
            k = n.split("(")[0].split("<")[0].replace("void ", "")[:40]
            per[k] = per.get(k, 0) + (e - s)
        top = ", ".join(f"{k} {v / 1e6:.0f} ms" for k, v in sorted(per.items(), key=lambda x: -x[1])[:4])
        span = max(e for _, e in iv) - min(s for s, _ in iv)
        lines.append(f"| `{os.path.basename(db)[:40]}` | {len(rows)} | {union(iv) / 1e6:.0f} | "
                     f"{span / 1e6:.0f} | {top} |")
    if not allv:
        print("no kernels")
        return
    span = max(e for _, e in allv) - min(s for s, _ in allv)
    busy = union(allv)
    print(f"GPU busy (union of every process's kernels): {busy / 1e6:.0f} ms of a "
          f"{span / 1e6:.0f} ms span = {100 * busy / span:.1f} %\n")
    print("| process db | kernels | busy ms | span ms | top kernels |\n|---|---:|---:|---:|---|")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1])
