"""Run bench.py's C5 quality-guard leg alone (one GPU) and print its JSON."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench

    args = argparse.Namespace(precision=26)
    out = bench.c5_guard(args, 0, 1, torch.device("cuda", 0))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
