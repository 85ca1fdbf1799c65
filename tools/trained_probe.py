"""bits/token of GPT-2-small random-init with the head scaled (trained-entropy rows): B streams x N bytes per
scale.  usage: python tools/trained_probe.py [--batch 64] [--bytes 128] [--scales 2,4,6,8]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--bytes", type=int, default=128)
    ap.add_argument("--scales", default="2,4,6,8")
    a = ap.parse_args()
    import torch

    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    m = random_gpt2("gpt2", seed=1234)
    q = {"temp": 0.9, "precision": 26, "topk": 300}
    for sc in [float(x) for x in a.scales.split(",")]:
        lm = HipArithmeticLM(m, None, logits_dtype="f16", max_batch=a.batch, logit_scale=sc)
        ctx = [lm.vocab - 1] + list(synthetic.DEFAULT_CONTEXT[1:])
        bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, a.bytes)) for s in range(a.batch)]
        t0 = time.perf_counter()
        toks = lm.encode_batch(bits, ctx, quality=q)
        dt = time.perf_counter() - t0
        ntok = sum(map(len, toks))
        print(json.dumps({"scale": sc, "bits_per_token": 8 * a.bytes * a.batch / ntok, "max_tokens": max(map(len, toks)),
                          "seconds": dt}), flush=True)
        del lm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
