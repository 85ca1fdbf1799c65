"""Time the wide path (topk beyond the single-pass limit: the api default precision 16 / topk 50,000) per kernel
with HIP events around whole steps.  python tools/wide_timing.py [--lib variant.so] [--batch 4096]"""
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--topk", type=int, default=50000)
    ap.add_argument("--precision", type=int, default=16)
    ap.add_argument("--dtype", default="f32")
    a = ap.parse_args()
    if a.lib:
        os.environ["NSG_CODER_LIB"] = a.lib
    import numpy as np
    import torch

    from neuralsteganography_amd import _lib, synthetic
    from neuralsteganography_amd.coder import CoderContext, CoderParams, EncodeSession, row_stride

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
    for t in range(3):
        sess.step(pool[t % 3])
    torch.cuda.synchronize()
    c0 = ctx.counters()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    for t in range(a.steps):
        ev[t][0].record()
        sess.step(pool[t % 3])
        ev[t][1].record()
    torch.cuda.synchronize()
    ms = float(np.mean([x.elapsed_time(y) for x, y in ev]))
    sess.raise_errors()
    c1 = ctx.counters()
    print(json.dumps({"lib": Path(_lib.LIB_PATH).name, "batch": B, "topk": a.topk, "precision": a.precision, "dtype": a.dtype,
                      "counters": [x - y for x, y in zip(c1, c0)],
                      "ms_per_step": round(ms, 4), "tokens": int(sess.fields()["ntokens"].sum()),
                      "exact_sum_steps": ctx.counters()[0] - c0[0], "stream_steps": B * a.steps}), flush=True)


if __name__ == "__main__":
    main()
