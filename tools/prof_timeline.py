"""Where the wall time of a serving run goes, from a rocprofv3 kernel-trace
database: engine steps are delimited by the sampler kernel (one launch per
step); a step is "prefill" when it runs the paged prefill attention kernel,
"decode" otherwise.  For each class: steps, wall ms (first kernel start ->
sampler end), kernel-busy ms, and the host gap before the step (previous
sampler end -> this step's first kernel).  Gaps longer than ``--wave-gap`` ms
split the run into waves (bench.py's timed rounds); the summary is printed
per wave and for the last ``--waves`` waves together.

    python tools/prof_timeline.py gpurun_out/prof_bench/run_results.db --waves 2
"""
import argparse
import sqlite3


def steps_of(rows, marker="sample_kernel"):
    out, cur = [], []
    for r in rows:
        cur.append(r)
        if marker in r[0]:
            out.append(cur)
            cur = []
    return out


def summarise(steps, prev_end):
    cls = {}
    for st in steps:
        kind = "prefill" if any("paged_prefill" in n for n, _, _ in st) else "decode"
        wall = (st[-1][2] - st[0][1]) / 1e6
        busy = sum(e - s for _, s, e in st) / 1e6
        gap = (st[0][1] - prev_end) / 1e6 if prev_end else 0.0
        prev_end = st[-1][2]
        c = cls.setdefault(kind, [0, 0.0, 0.0, 0.0, 0.0])
        c[0] += 1
        c[1] += wall
        c[2] += busy
        c[3] += gap
        c[4] = max(c[4], gap)
    return cls


def report(db_path: str, waves: int = 2, wave_gap_ms: float = 30.0) -> str:
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    # waves: runs of kernels separated by an idle GPU longer than wave_gap_ms
    segs, cur = [], [rows[0]]
    for a, b in zip(rows, rows[1:]):
        if (b[1] - a[2]) / 1e6 > wave_gap_ms:
            segs.append(cur)
            cur = []
        cur.append(b)
    segs.append(cur)
    groups = [g for g in (steps_of(sg) for sg in segs) if g]
    steps = [st for g in groups for st in g]
    out = [f"{len(steps)} engine steps in {len(groups)} waves (split at idle > {wave_gap_ms} ms)", ""]
    out += ["| wave | span ms | class | steps | wall ms | busy ms | host gaps ms | max gap ms |",
            "|---:|---:|---|---:|---:|---:|---:|---:|"]
    for wi, g in enumerate(groups):
        span = (g[-1][-1][2] - g[0][0][1]) / 1e6
        for kind, (n, wall, busy, gap, mx) in sorted(summarise(g, None).items()):
            out.append(f"| {wi} | {span:.0f} | {kind} | {n} | {wall:.1f} | {busy:.1f} | {gap:.1f} | {mx:.2f} |")
    last = [s for g in groups[-waves:] for s in g]
    span = sum((g[-1][-1][2] - g[0][0][1]) / 1e6 for g in groups[-waves:])
    tot = summarise(last, None)
    out += ["", f"last {waves} waves: span {span:.0f} ms"]
    for kind, (n, wall, busy, gap, mx) in sorted(tot.items()):
        out.append(f"  {kind:8s} {n:5d} steps  wall {wall:8.1f} ms ({wall / max(n, 1):.2f}/step)  "
                   f"busy {busy:8.1f} ms  host gaps {gap:7.1f} ms (max {mx:.2f})")
    # kernel totals by class over the last waves
    agg = {}
    for st in last:
        kind = "prefill" if any("paged_prefill" in n for n, _, _ in st) else "decode"
        for n, s, e in st:
            a = agg.setdefault((kind, n), [0, 0])
            a[0] += 1
            a[1] += e - s
    out += ["", "| class | ms | launches | us/launch | kernel |", "|---|---:|---:|---:|---|"]
    for (kind, n), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        out.append(f"| {kind} | {t / 1e6:.1f} | {c} | {t / c / 1e3:.1f} | `{n[:90]}` |")
    return "\n".join(out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--waves", type=int, default=2)
    ap.add_argument("--wave-gap", type=float, default=30.0)
    a = ap.parse_args()
    print(report(a.db, a.waves, a.wave_gap))
