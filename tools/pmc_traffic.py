"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM traffic of the coder kernel.

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE counts exactly half the bytes of a wide
coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for 16-B stores
and used as-is (KB * 1024).  Usage:
  python tools/pmc_traffic.py FETCH.csv WRITE.csv OUT.json --version "$(lib version)" --batch 4096 ...
"""
import argparse
import csv
import json
import statistics


def kernel_values(path, kernel="coder_step_kernel"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no {kernel} rows in {path}")
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("out")
    ap.add_argument("--version", required=True)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--vocab", type=int, default=50257)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--topk", type=int, default=300)
    ap.add_argument("--kernel", default="coder_step_kernel", help="kernel name substring")
    ap.add_argument("--L", type=int, default=None, help="attention: cache length of the run")
    ap.add_argument("--alg-bytes", type=float, default=None, help="algorithmic bytes per launch of the run")
    a = ap.parse_args()
    f = kernel_values(a.fetch_csv, a.kernel)
    w = kernel_values(a.write_csv, a.kernel)
    fetch_kb, write_kb = statistics.mean(f), statistics.mean(w)
    rec = {"library_version": a.version, "kernel": a.kernel, "batch": a.batch, "vocab": a.vocab, "dtype": a.dtype, "topk": a.topk,
           "launches": [len(f), len(w)], "fetch_size_kb_mean": fetch_kb, "write_size_kb_mean": write_kb,
           "read_bytes_corrected": 2.0 * fetch_kb * 1024.0, "write_bytes": write_kb * 1024.0,
           "traffic_bytes_per_launch": 2.0 * fetch_kb * 1024.0 + write_kb * 1024.0,
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write = WRITE_SIZE x 1024"}
    if a.L is not None:
        rec["L"] = a.L
    if a.alg_bytes is not None:
        rec["alg_bytes_per_launch"] = a.alg_bytes
        rec["traffic_over_alg"] = rec["traffic_bytes_per_launch"] / a.alg_bytes
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
