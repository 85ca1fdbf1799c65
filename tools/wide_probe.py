"""Time the wide path (api default quality: precision 16, topk 50,000, temp 1.0) at B streams on resident
3*N(0,1) logits, one JSON line per dtype.  NSG_WIDE_V2=0/1 (read once per process) picks the one-pass kernel or
the stream + tail kernels.  Usage: python tools/wide_probe.py [--batch 4096] [--steps 20] [--dtype f32 f16]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--vocab", type=int, default=50257)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--dtype", nargs="+", default=["f32", "f16"])
    ap.add_argument("--decode", action="store_true", help="also time the decode of the encoded tokens")
    args = ap.parse_args()
    import torch

    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.coder import CoderContext, CoderParams, EncodeSession, row_stride

    dev = torch.device("cuda:0")
    V, B = args.vocab, args.batch
    for dt in args.dtype:
        params = CoderParams(vocab=V, precision=16, temp=1.0, topk=50000, dtype=dt)
        ctx = CoderContext(params, max_batch=B)
        ld = row_stride(V, dt)
        tdt = torch.float32 if dt == "f32" else torch.float16
        g = torch.Generator(device=dev)
        pool = []
        for i in range(3):
            g.manual_seed(1000 + i)
            pool.append((3.0 * torch.randn((B, ld), generator=g, device=dev)).to(tdt))
        sess = EncodeSession(ctx, [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 1024)) for s in range(B)])
        for t in range(args.warmup):
            sess.step(pool[t % 3])
        c0 = ctx.counters()
        nt0 = int(sess.fields()["ntokens"].astype("int64").sum())
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.time()
        s.record()
        for t in range(args.steps):
            sess.step(pool[t % 3])
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / args.steps
        sess.raise_errors()
        c1 = ctx.counters()
        ntok = int(sess.fields()["ntokens"].astype("int64").sum()) - nt0
        esz = 4 if dt == "f32" else 2
        alg = B * (V * esz + 76)
        print(json.dumps({"dtype": dt, "v2": os.environ.get("NSG_WIDE_V2"), "B": B, "ms_per_step": ms,
                          "frac": alg / (ms / 1e3) / 1e9 / 8000.0, "tokens": ntok,
                          "exact_per_tok": (c1[0] - c0[0]) / max(ntok, 1),
                          "sweeps_per_tok": (c1[1] - c0[1]) / max(ntok, 1),
                          "wall_s": time.time() - t0}), flush=True)
        del pool, sess, ctx
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
