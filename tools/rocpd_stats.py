"""Kernel statistics from a rocprofv3 results database (``--kernel-trace`` writes ``*_results.db``, SQLite):

    python tools/rocpd_stats.py RUN_results.db OUT_kernel_stats.csv [--after-last NAME] [--window-from NAME]

Writes the per-kernel summary rocprofv3 --stats gives as CSV (Name, Calls, TotalDurationNs, AverageNs, MinNs, MaxNs,
Percentage) and prints a JSON line with the busy time (sum of kernel durations) against the wall span of the
window, i.e. how much of the window the GPU sat idle between kernels (host checks, launch gaps).  The window starts
at the first launch of the job proper: ``--window-from`` names a kernel whose FIRST launch after the warm-up marks it
(default: the whole trace)."""
import argparse
import csv
import json
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("out")
    ap.add_argument("--window-from", default=None, help="kernel name substring; the window starts at its n-th launch")
    ap.add_argument("--nth", type=int, default=1, help="which launch of --window-from opens the window (1-based)")
    ap.add_argument("--after-fill-run", type=int, default=0,
                    help="the window starts after the last run of at least this many consecutive torch elementwise "
                         "kernels (tools/c3_job_probe.py: the page pool's warm-up fill just before the job)")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, start, end, duration from kernels order by start").fetchall()
    if a.after_fill_run:
        last, i = 0, 0
        while i < len(rows):
            j = i
            while j < len(rows) and "vectorized_elementwise" in rows[j][0]:
                j += 1
            if j - i >= a.after_fill_run:
                last = j
            i = max(j, i + 1)
        rows = rows[last:]
    if a.window_from:
        hits = [i for i, r in enumerate(rows) if a.window_from in r[0]]
        if len(hits) < a.nth:
            raise SystemExit(f"{a.window_from}: {len(hits)} launches, fewer than --nth {a.nth}")
        rows = rows[hits[a.nth - 1]:]
    by = {}
    for name, _, _, dur in rows:
        by.setdefault(name, []).append(dur)
    total = sum(sum(v) for v in by.values())
    with open(a.out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
        for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), sum(v), statistics.mean(v), min(v), max(v), 100.0 * sum(v) / total])
    span = rows[-1][2] - rows[0][1] if rows else 0
    print(json.dumps({"kernels": len(rows), "busy_ns": total, "span_ns": span,
                      "busy_fraction": total / span if span else None}))


if __name__ == "__main__":
    main()
