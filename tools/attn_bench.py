"""The decode-attention microbenchmark of bench.py (roofline_attention) alone, for rocprofv3 passes.
usage: python tools/attn_bench.py [--batch 4096] [--L 544] [--steps 20] [--T0 32]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--L", type=int, default=544)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--T0", type=int, default=32, help="shared context positions (stored once)")
    a = ap.parse_args()
    import torch

    import bench

    args = argparse.Namespace(e2e_batch=a.batch)
    dev = torch.device("cuda", 0)
    rec = bench.attention_bench(args, 0, 1, dev, L=a.L, steps=a.steps, T0=a.T0)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
