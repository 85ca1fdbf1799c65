"""Phase attribution of the coder kernel: time the same launch with diagnostic early exits.

python tools/phase_timing.py [--lib path/to/variant.so] [--batch 4096] [--steps 30]
Prints one JSON line per phase: avg kernel ms measured with HIP events on the launch stream.
"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--topk", type=int, default=300)
    ap.add_argument("--stats", action="store_true", help="statistics build (EncodeSession(stats=True))")
    ap.add_argument("--full-only", action="store_true", help="time the full step only")
    a = ap.parse_args()
    if a.lib:
        os.environ["NSG_CODER_LIB"] = a.lib
    import numpy as np
    import torch

    from neuralsteganography_amd import _lib, synthetic
    from neuralsteganography_amd.coder import CoderContext, CoderParams, EncodeSession, row_stride

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
    sess = EncodeSession(ctx, bits, stats=a.stats)
    sess.enable_trace()
    phases = [("stream_no_cand", _lib.NS_STEP_DIAG_NO_CANDIDATES), ("stream_cand", _lib.NS_STEP_DIAG_STREAM_ONLY),
              ("stream_cand_rank", _lib.NS_STEP_DIAG_SKIP_CDF), ("full", 0)]
    if a.full_only:
        phases = phases[-1:]
    for name, fl in phases:
        for t in range(3):
            sess.step(pool[t % 4], diag_flags=fl)
        torch.cuda.synchronize()
        c0 = ctx.counters()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
        for t in range(a.steps):
            ev[t][0].record()
            sess.step(pool[t % 4], diag_flags=fl)
            ev[t][1].record()
        torch.cuda.synchronize()
        c1 = ctx.counters()
        ms = float(np.mean([x.elapsed_time(y) for x, y in ev]))
        gbs = B * (V * (2 if a.dtype == "f16" else 4)) / (ms / 1e3) / 1e9
        n = B * a.steps
        print(json.dumps({"lib": Path(_lib.LIB_PATH).name, "phase": name, "ms": round(ms, 4),
                          "GBps": round(gbs, 1), "exact_per_step": (c1[0] - c0[0]) / n,
                          "overflow_compactions_per_step": (c1[1] - c0[1]) / n,
                          "spec_miss_per_step": (c1[2] - c0[2]) / n}), flush=True)


if __name__ == "__main__":
    main()
