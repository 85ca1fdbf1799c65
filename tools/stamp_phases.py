"""Per-wave phase timeline of the coder kernel from in-kernel s_memtime stamps (diagnostic build).

Build the variant:  hipcc ... -DNSG_STAMPS=1 -o neuralsteganography_amd/_build/variants/stamps.so ...
Run:                python tools/stamp_phases.py --lib neuralsteganography_amd/_build/variants/stamps.so

Stamps (lane 0 of every wave): 0 start, 1 after the sample prologue, 2 after the streaming loop, 3 after the
speculation check, 4 after the raw->key conversion, 5 after the final compaction, 6 after the ranking,
7 after the CDF (before the state update), 8 end.  The s_memtime clock is calibrated against the launch's
HIP-event duration (span of all stamps ~ the kernel).  Prints one JSON object.
"""
import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

NAMES = ["prologue", "stream", "spec_check", "to_keys", "compact", "rank", "cdf", "state"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--topk", type=int, default=300)
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
    params = CoderParams(vocab=V, precision=26, temp=0.9, topk=a.topk, dtype=a.dtype)
    ctx = CoderContext(params, max_batch=B)
    ld = row_stride(V, a.dtype)
    g = torch.Generator(device="cuda")
    pool = []
    for i in range(4):
        g.manual_seed(i)
        pool.append((3.0 * torch.randn((B, ld), generator=g, device="cuda")).to(params.torch_dtype))
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 1024)) for s in range(B)]
    sess = EncodeSession(ctx, bits)
    stamps = torch.zeros((B, 16), dtype=torch.int64, device="cuda")
    per_phase = []   # us per phase per wave (s_memtime calibrated per wave with s_memrealtime, 100 MHz)
    timeline = []    # s_memrealtime start / end per wave, us from the launch's first start
    ev = []
    for t in range(a.steps):
        L.ns_set_stamps(ctx._h, ctypes.c_void_p(stamps.data_ptr() if t >= 2 else 0))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sess.step(pool[t % 4])
        e1.record()
        torch.cuda.synchronize()
        if t < 2:
            continue
        raw = stamps.cpu().numpy().astype(np.int64)
        mt, rt = raw[:, :9], raw[:, 9:11]
        ok = np.all(mt > 0, axis=1) & np.all(np.diff(mt, axis=1) >= 0, axis=1) & (rt[:, 1] > rt[:, 0])
        mt, rt = mt[ok], rt[ok]
        ticks_per_us = (mt[:, 8] - mt[:, 0]) / ((rt[:, 1] - rt[:, 0]) / 100.0)
        per_phase.append(np.diff(mt, axis=1) / ticks_per_us[:, None])
        base = rt[:, 0].min()
        timeline.append(((rt[:, 0] - base) / 100.0, (rt[:, 1] - base) / 100.0))
        ev.append(e0.elapsed_time(e1) * 1e3)
        if t == 2:
            idx = np.nonzero(ok)[0]
            xcd = (idx // 4) % 8  # 4 waves per workgroup, workgroups dealt round-robin over the 8 XCDs
            stream_us = (mt[:, 2] - mt[:, 1]) / ticks_per_us
            end_us = (rt[:, 1] - base) / 100.0
            xcd_rows = {}
            for x in range(8):
                m = xcd == x
                if not m.any():  # small batches leave XCDs without a stream
                    continue
                xcd_rows[x] = {"stream_p50": round(float(np.median(stream_us[m])), 1),
                               "end_p50": round(float(np.median(end_us[m])), 1),
                               "end_max": round(float(end_us[m].max()), 1)}
            slot = (idx % 4)
            slot_rows = {int(k): round(float(np.median(stream_us[slot == k])), 1) for k in range(4)
                         if (slot == k).any()}
            print(json.dumps({"per_xcd": xcd_rows, "stream_p50_by_wave_slot": slot_rows}), file=sys.stderr)
        if t == 2:
            print(f"valid rows {int(ok.sum())}; median clock {np.median(ticks_per_us):.1f} ticks/us", file=sys.stderr)
    d = np.concatenate(per_phase)
    out = {"lib": Path(a.lib).name, "event_us": round(float(np.median(ev)), 2), "phases_us": {}}
    for i, n in enumerate(NAMES):
        col = d[:, i]
        out["phases_us"][n] = {"mean": round(float(col.mean()), 2), "p50": round(float(np.median(col)), 2),
                               "p99": round(float(np.percentile(col, 99)), 2), "max": round(float(col.max()), 2)}
    st0, en0 = timeline[0]
    out["timeline_us"] = {"start": {q: round(float(np.percentile(st0, q)), 2) for q in (0, 10, 50, 90, 100)},
                          "end": {q: round(float(np.percentile(en0, q)), 2) for q in (0, 10, 50, 90, 100)},
                          "wave_duration": {q: round(float(np.percentile(en0 - st0, q)), 2) for q in (0, 10, 50, 90, 100)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
