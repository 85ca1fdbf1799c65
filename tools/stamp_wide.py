"""Per-workgroup phase timeline of the one-pass wide kernel (api default quality) from in-kernel s_memtime
stamps (diagnostic build: tools/build_variant.sh wstamps -DNSG_STAMPS=1).

python tools/stamp_wide.py --lib neuralsteganography_amd/_build/variants/wstamps.so [--dtype f16]

Stamps (thread 0 of each stream's workgroup): 0 start, 1 sample prologue + first threshold, 2 streaming loop,
3 row statistics (block reductions), 4 buffer filter / merge (or the fallback sweeps), 5 LDS sort, 6 cutoff
(exps), 7 E + q + prefix, 8 selection + state update.  Streams handed to the list kernel have no stamp 8 and are
left out.  Prints one JSON object: per-phase us (mean / p50 / p99), workgroup durations, and the occupancy
profile (how many workgroups are inside each phase over the launch)."""
import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

NAMES = ["prologue", "stream", "rowstats", "filter", "sort", "cutoff", "cdf", "select"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--topk", type=int, default=50000)
    ap.add_argument("--precision", type=int, default=16)
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    os.environ["NSG_CODER_LIB"] = a.lib
    import numpy as np
    import torch

    from neuralsteganography_amd import _lib, synthetic
    from neuralsteganography_amd.coder import CoderContext, CoderParams, EncodeSession, row_stride

    L = _lib.lib()
    L.ns_set_stamps.restype = ctypes.c_int
    L.ns_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    V, B = 50257, a.batch
    params = CoderParams(vocab=V, precision=a.precision, temp=1.0, topk=a.topk, dtype=a.dtype)
    ctx = CoderContext(params, max_batch=B)
    ld = row_stride(V, a.dtype)
    g = torch.Generator(device="cuda")
    pool = []
    for i in range(3):
        g.manual_seed(i)
        pool.append((3.0 * torch.randn((B, ld), generator=g, device="cuda")).to(params.torch_dtype))
    sess = EncodeSession(ctx, [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 256)) for s in range(B)])
    stamps = torch.zeros((B, 16), dtype=torch.int64, device="cuda")
    per_phase, dur, ev, occ = [], [], [], None
    for t in range(a.steps):
        stamps.zero_()
        L.ns_set_stamps(ctx._h, ctypes.c_void_p(stamps.data_ptr() if t >= 2 else 0))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sess.step(pool[t % 3])
        e1.record()
        torch.cuda.synchronize()
        if t < 2:
            continue
        raw = stamps.cpu().numpy().astype(np.int64)
        mt, rt = raw[:, :9], raw[:, 9:11]
        ok = np.all(mt > 0, axis=1) & np.all(np.diff(mt, axis=1) >= 0, axis=1) & (rt[:, 1] > rt[:, 0])
        mt, rt = mt[ok], rt[ok]
        tpu = (mt[:, 8] - mt[:, 0]) / ((rt[:, 1] - rt[:, 0]) / 100.0)
        per_phase.append(np.diff(mt, axis=1) / tpu[:, None])
        dur.append((rt[:, 1] - rt[:, 0]) / 100.0)
        ev.append(e0.elapsed_time(e1) * 1e3)
        if occ is None:  # phase occupancy over time: workgroups inside each phase, sampled every 5 us
            base = rt[:, 0].min()
            t0 = (rt[:, 0] - base) / 100.0
            bounds = t0[:, None] + np.concatenate([np.zeros((len(mt), 1)),
                                                    np.cumsum(np.diff(mt, axis=1) / tpu[:, None], axis=1)], axis=1)
            span = float(bounds[:, -1].max())
            occ = {"valid_workgroups": int(ok.sum()), "span_us": round(span, 1), "samples": []}
            for ts in np.arange(0.0, span, 5.0):
                inside = [(bounds[:, i] <= ts) & (ts < bounds[:, i + 1]) for i in range(len(NAMES))]
                occ["samples"].append([round(float(ts), 1)] + [int(x.sum()) for x in inside])
    d = np.concatenate(per_phase)
    out = {"lib": Path(a.lib).name, "dtype": a.dtype, "event_us": round(float(np.median(ev)), 2), "phases_us": {}}
    for i, n in enumerate(NAMES):
        col = d[:, i]
        out["phases_us"][n] = {"mean": round(float(col.mean()), 2), "p50": round(float(np.median(col)), 2),
                               "p99": round(float(np.percentile(col, 99)), 2)}
    dd = np.concatenate(dur)
    out["workgroup_us"] = {q: round(float(np.percentile(dd, q)), 2) for q in (0, 10, 50, 90, 100)}
    out["occupancy"] = occ
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
