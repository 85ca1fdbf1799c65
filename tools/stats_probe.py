"""Encode-step time with and without the on-device statistics (EncodeSession(stats=True): the avg_NLL / avg_KL /
words_per_bit / avg_Hq that code_base.encode_arithmetic returns), HIP-event timed on resident 3*N(0,1) rows.
usage: python tools/stats_probe.py [--batch 4096 1] [--dtype f16 f32] [--topk 300] [--steps 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[4096, 1])
    ap.add_argument("--dtype", nargs="+", default=["f16", "f32"])
    ap.add_argument("--topk", type=int, default=300)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch

    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.coder import CoderContext, CoderParams, EncodeSession, row_stride

    V = 50257
    for dt in a.dtype:
        for B in a.batch:
            params = CoderParams(vocab=V, precision=26, temp=0.9, topk=a.topk, dtype=dt)
            ld = row_stride(V, dt)
            g = torch.Generator(device="cuda")
            pool = []
            for i in range(3):
                g.manual_seed(i)
                pool.append((3.0 * torch.randn((B, ld), generator=g, device="cuda")).to(params.torch_dtype))
            rec = {"dtype": dt, "batch": B, "topk": a.topk}
            for stats in (False, True):
                ctx = CoderContext(params, max_batch=B)
                bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 1024)) for s in range(B)]
                sess = EncodeSession(ctx, bits, stats=stats)
                for t in range(3):
                    sess.step(pool[t % 3])
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for t in range(a.steps):
                    sess.step(pool[t % 3])
                e1.record()
                torch.cuda.synchronize()
                rec["us_stats" if stats else "us_plain"] = e0.elapsed_time(e1) / a.steps * 1e3
                sess.raise_errors()
                del sess, ctx
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
