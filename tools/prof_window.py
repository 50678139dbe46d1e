"""Per-step kernel breakdown of the LAST ``--steps`` engine steps in a
rocprofv3 kernel-trace database: steps are delimited by the sampler kernel
(one launch per engine step), so the window is pure decode (hipGraph
replays) once the prompts are prefilled.

    python tools/prof_window.py gpurun_out/prof_engine/run_results.db --steps 20
"""
import argparse
import sqlite3


def window(db_path: str, steps: int = 20, marker: str = "sample_kernel", top: int = 25) -> str:
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if marker in r[0]]
    if len(marks) < steps + 1:
        raise SystemExit(f"only {len(marks)} '{marker}' launches")
    lo, hi = marks[-steps - 1] + 1, marks[-1] + 1
    sel = rows[lo:hi]
    wall = (sel[-1][2] - sel[0][1]) / 1e6 / steps
    agg = {}
    for n, s, e in sel:
        a = agg.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += e - s
    busy = sum(v[1] for v in agg.values()) / 1e6 / steps
    out = [f"last {steps} steps: wall {wall:.3f} ms/step, kernel-busy {busy:.3f} ms/step", "",
           "| ms/step | launches/step | us/launch | kernel |", "|---:|---:|---:|---|"]
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        out.append(f"| {t / 1e6 / steps:.3f} | {c / steps:.1f} | {t / c / 1e3:.1f} | `{n[:96]}` |")
    return "\n".join(out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--marker", default="sample_kernel")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    print(window(a.db, a.steps, a.marker, a.top))
