#!/bin/bash
# Small-batch A/B of the two single-pass coder forms (one wave per stream vs the split workgroup-per-stream form):
# tools/split_ab.sh OUTDIR "phase_timing args" B1 B2 ...   (each run under its own time limit; stops at a failure)
set -e
out=$1; args=$2; shift 2
mkdir -p "$out"
for b in "$@"; do
    NSG_SPLIT_MAX_B=0 timeout -k 10 120 python tools/phase_timing.py --batch "$b" $args > "$out/wave_b$b.jsonl" 2>&1
    NSG_SPLIT_MAX_B=1000000 timeout -k 10 120 python tools/phase_timing.py --batch "$b" $args > "$out/split_b$b.jsonl" 2>&1
done
