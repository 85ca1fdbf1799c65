"""Throughput of the Fraction coder kernel (row a12) against its CPU restatement (fractions.Fraction, the
reference's own arithmetic): B messages of zero bytes (the payloads this coder can carry) over
per-step float64 distributions of V tokens, encoded then decoded in lockstep; the restatement encodes a
sample of the same messages on one core.  Prints one JSON line.
usage: python tools/frac_probe.py [--batch 4096] [--vocab 16] [--bytes 8] [--sample 16]"""

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--vocab", type=int, default=16)
    ap.add_argument("--bytes", type=int, default=8)
    ap.add_argument("--sample", type=int, default=16)
    ap.add_argument("--steps", type=int, default=64, help="distributions per message")
    args = ap.parse_args()

    import torch

    from neuralsteganography_amd.codec import fraction as F
    from oracle import fraction_coder as fc

    rng = np.random.default_rng(0)
    base = rng.random((97, args.vocab))
    base /= base.sum(axis=1, keepdims=True)
    streams = [[base[(b + t) % 97] for t in range(args.steps)] for b in range(args.batch)]
    payloads = [bytes(args.bytes)] * args.batch
    F.encode_bits_batch(payloads[:8], [iter(s) for s in streams[:8]], [{} for _ in range(8)])  # warm-up
    torch.cuda.synchronize()
    states = [{} for _ in range(args.batch)]
    t0 = time.perf_counter()
    toks = F.encode_bits_batch(payloads, [iter(s) for s in streams], states)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    dec = F.decode_bits_batch(toks, [iter(s) for s in streams], [dict(s) for s in states])
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ntok = sum(len(t) for t in toks)
    steps = max(len(t) for t in toks)
    c0 = time.perf_counter()
    for b in range(args.sample):
        want, _ = fc.encode(payloads[b], streams[b])
        assert want == toks[b]
    c1 = time.perf_counter()
    ctok = sum(len(t) for t in toks[:args.sample])
    print(json.dumps({
        "probe": "fraction_coder", "batch": args.batch, "vocab": args.vocab, "payload_bytes": args.bytes,
        "lockstep_steps": steps, "tokens": ntok, "encode_s": t1 - t0, "decode_s": t2 - t1,
        "encode_tokens_per_s": ntok / (t1 - t0), "decode_tokens_per_s": ntok / (t2 - t1),
        "encode_payload_bits_per_s": 8 * args.bytes * args.batch / (t1 - t0),
        "roundtrip_exact_fraction": sum(d == p for d, p in zip(dec, payloads)) / args.batch,
        "cpu_restatement": {"tokens": ctok, "seconds": c1 - c0, "tokens_per_s": ctok / (c1 - c0), "cores": 1,
                            "kind": "port (fractions.Fraction, the reference's arithmetic)"},
        "note": "host-inclusive: per step the host gathers B rows from the ProbDist iterables (Python) and "
                "launches one kernel; kernel time from rocprofv3 frac_step_kernel"}), flush=True)


if __name__ == "__main__":
    main()
