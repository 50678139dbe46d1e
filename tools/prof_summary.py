"""Summarise a rocprofv3 kernel-trace database (``*_results.db``) into a
markdown table: time per kernel, launches, share of GPU time.

    python tools/prof_summary.py gpurun_out/prof/run_results.db [--top 25]
"""
import argparse
import sqlite3


def summarize(db_path: str, top: int = 25, name_filter: str = "") -> str:
    db = sqlite3.connect(db_path)
    q = "select name, count(*), sum(end-start) from kernels"
    args = ()
    if name_filter:
        q += " where name like ?"
        args = (f"%{name_filter}%",)
    rows = db.execute(q + " group by name order by 3 desc", args).fetchall()
    total = sum(r[2] for r in rows) or 1
    out = [f"GPU kernel time: {total / 1e6:.1f} ms over {sum(r[1] for r in rows)} launches", "",
           "| ms | % | launches | us/launch | kernel |", "|---:|---:|---:|---:|---|"]
    for name, n, t in rows[:top]:
        out.append(f"| {t / 1e6:.2f} | {100 * t / total:.1f} | {n} | {t / n / 1e3:.1f} | "
                   f"`{name[:100]}` |")
    return "\n".join(out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    print(summarize(a.db, a.top, a.filter))
