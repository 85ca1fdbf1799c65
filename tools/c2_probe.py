"""C2 probe: GPT-2-small (random-init, fp16) + coder at B streams (default 1) encoding a 1 KiB payload from the
32-token context, hipGraph-replayed token loop; prints ms per token step.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split of the step."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--bytes", type=int, default=1024)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--kv", default="fp16", choices=["fp16", "fp8"])
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--topk", type=int, default=300)
    args = ap.parse_args()
    import torch

    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    B = args.batch
    lm = HipArithmeticLM(random_gpt2(args.model, seed=1234), None, logits_dtype="f16", max_batch=B,
                         kv_dtype=args.kv, attention_window=args.window)
    q = {"temp": 0.9, "precision": 26, "topk": args.topk}
    ctx = synthetic.DEFAULT_CONTEXT
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, args.bytes)) for s in range(B)]
    graphs = False if args.eager else None
    lm.encode_batch([b[:64] for b in bits], ctx, quality=q, graphs=graphs)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    toks = lm.encode_batch(bits, ctx, quality=q, graphs=graphs)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = max(map(len, toks))
    print(json.dumps({"batch": B, "model": args.model, "steps": steps, "seconds": dt,
                      "ms_per_step": 1e3 * dt / steps, "graphs": not args.eager,
                      "kv": args.kv, "window": args.window, "cover_tokens_per_s": sum(map(len, toks)) / dt}), flush=True)


if __name__ == "__main__":
    main()
