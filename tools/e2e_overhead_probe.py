"""Where the timed end-to-end encode spends wall time outside the steady token steps: the shared-context prefill,
the first step + hipGraph capture, the host checks (sess.fields, every 16 steps), and the replays.  Wraps those
calls with device-synchronised timers (the wrapping itself adds a sync per check).
usage: python tools/e2e_overhead_probe.py [--batch 4096] [--kv fp16] [--window 0] [--bytes 1024]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--bytes", type=int, default=1024)
    ap.add_argument("--kv", default="fp16")
    ap.add_argument("--window", type=int, default=0)
    args = ap.parse_args()
    import torch

    from neuralsteganography_amd import coder as coder_mod
    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.lm import arithmetic as A
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    B = args.batch
    lm = A.HipArithmeticLM(random_gpt2("gpt2", seed=1234), None, logits_dtype="f16", max_batch=B, kv_dtype=args.kv,
                           attention_window=args.window)
    q = {"temp": 0.9, "precision": 26, "topk": 300}
    ctx = [lm.vocab - 1] + list(synthetic.DEFAULT_CONTEXT[1:])
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, args.bytes)) for s in range(B)]
    lm.encode_batch([b[:64] for b in bits], ctx, quality=q)
    lm.lm.prefill(ctx, B, 2 * max(len(b) for b in bits) + 64)  # as bench.py: the full-size cache once
    lm.lm.k_cache = lm.lm.v_cache = None
    torch.cuda.synchronize()
    acc = {}

    def wrap(obj, name, key):
        f = getattr(obj, name)

        def g(*a, **k):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = f(*a, **k)
            torch.cuda.synchronize()
            acc[key] = acc.get(key, 0.0) + time.perf_counter() - t
            acc[key + "_n"] = acc.get(key + "_n", 0) + 1
            return r
        setattr(obj, name, g)

    wrap(lm.lm, "prefill", "prefill")
    wrap(A._StepGraph, "__init__", "first_step_and_capture")
    wrap(coder_mod.EncodeSession, "fields", "fields")
    marks = []
    f0 = coder_mod.EncodeSession.fields

    def fields_marked(self):
        r = f0(self)
        marks.append(time.perf_counter())
        return r
    coder_mod.EncodeSession.fields = fields_marked
    wrap(coder_mod.EncodeSession, "ensure_history", "ensure_history")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    toks = lm.encode_batch(bits, ctx, quality=q)
    torch.cuda.synchronize()
    acc["total"] = time.perf_counter() - t0
    acc["steps"] = max(map(len, toks))
    acc["ms_per_16_steps"] = [round(1e3 * (b - a), 2) for a, b in zip(marks, marks[1:])]
    print(json.dumps(acc), flush=True)


if __name__ == "__main__":
    main()
