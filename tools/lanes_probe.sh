#!/bin/bash
# Decode-step lanes A/B (BatchedGPT2.decode_lanes): the C3 step (fp16 KV) and the opt-in step (fp8 KV, window 256) at
# B = 4,096 after 512 steps (cache length ~544), one / two lanes, alternating / free attention order, graph replays
# (and eager launches with --eager as the second argument).
# usage: tools/lanes_probe.sh OUT.jsonl [--eager]
set -e
out=$1
for kv in "--kv fp16" "--kv fp8 --window 256"; do
  for lanes in "--lanes 1" "--lanes 2 --order alternate" "--lanes 2 --order free"; do
    timeout -k 10 240 python tools/replay_probe.py $kv $lanes --skip 512 --reps 32 --blocks 2 $2 >> "$out"
  done
done
