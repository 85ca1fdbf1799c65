"""One whole encode job on the product path (slot scheduler, paged KV, hipGraph-replayed steps), for rocprofv3:

    rocprofv3 --kernel-trace --stats -d OUT -o c3 -- python tools/c3_job_probe.py [--batch 4096] [--bytes 1024]

A short warm-up encode (a few steps: kernels, graph, coder context) and the page pool's warm-up come first; the
job itself then runs every stream from the 32-token context to its end, so a kernel-stats summary of the run
averages each kernel over cache lengths T0 .. T0 + the longest cover (C3: 32 .. ~1,055, mean ~544).  Prints one
JSON line (job seconds, lockstep steps, tokens, the warm-up's share of the launches)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--messages", type=int, default=0, help="0: one message per slot")
    ap.add_argument("--bytes", type=int, default=1024)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--kv", default="fp16")
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--topk", type=int, default=300)
    args = ap.parse_args()
    import torch

    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    B = args.batch
    lm = HipArithmeticLM(random_gpt2(args.model, seed=1234), None, logits_dtype="f16", max_batch=B, kv_dtype=args.kv,
                         attention_window=args.window, logit_scale=args.scale)
    q = {"temp": 0.9, "precision": 26, "topk": args.topk}
    ctx = [lm.vocab - 1] + list(synthetic.DEFAULT_CONTEXT[1:])
    lm.encode_batch([[1, 0, 1, 1] * 8] * B, ctx, quality=q)
    lm.lm.warm_pool(B=B)
    n = args.messages or B
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, args.bytes)) for s in range(n)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    toks = lm.encode_batch(bits, ctx, quality=q, slots=B)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = max(map(len, toks))
    ntok = sum(map(len, toks))
    print(json.dumps({"batch": B, "messages": n, "bytes": args.bytes, "kv": args.kv, "window": args.window,
                      "scale": args.scale, "seconds": dt, "longest_cover": steps, "tokens": ntok,
                      "tok_per_s": ntok / dt, "schedule": lm.last_schedule,
                      "cache_lengths": f"{len(ctx)} .. {len(ctx) + steps}"}), flush=True)


if __name__ == "__main__":
    main()
