"""Per-phase PMC counters of the coder kernel: rocprofv3 --pmc over tools/phase_timing.py.

tools/phase_timing.py launches each diagnostic phase (stream_no_cand, stream_cand, stream_cand_rank, full)
3 + STEPS times in that order; this groups the coder_step_kernel dispatches of every counter CSV given in
that order and prints the mean value of each counter per phase (per launch).

  python tools/pmc_phases.py --steps 10 OUT.json A.csv [B.csv ...]
"""
import argparse
import csv
import json
from collections import defaultdict

PHASES = ["stream_no_cand", "stream_cand", "stream_cand_rank", "full"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("out")
    ap.add_argument("csvs", nargs="+")
    a = ap.parse_args()
    per = 3 + a.steps
    res = defaultdict(dict)
    for path in a.csvs:
        rows = [r for r in csv.DictReader(open(path)) if "coder_step_kernel" in r["Kernel_Name"]]
        by_counter = defaultdict(list)
        for r in rows:
            by_counter[r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        for cname, vals in by_counter.items():
            vals.sort()
            if len(vals) != per * len(PHASES):
                raise SystemExit(f"{path}: {cname} has {len(vals)} dispatches, expected {per * len(PHASES)}")
            for i, ph in enumerate(PHASES):
                chunk = [v for _, v in vals[i * per + 3:(i + 1) * per]]  # skip the 3 warmup launches
                res[ph][cname] = sum(chunk) / len(chunk)
    json.dump(res, open(a.out, "w"), indent=1)
    names = sorted({c for ph in res.values() for c in ph})
    print("counter".ljust(28) + "".join(p.rjust(18) for p in PHASES))
    for c in names:
        print(c.ljust(28) + "".join(f"{res[p].get(c, float('nan')):18.4g}" for p in PHASES))


if __name__ == "__main__":
    main()
