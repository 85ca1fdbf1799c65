#!/bin/bash
# Decode-step lanes with the attention on its own (optionally CU-masked) stream, eager launches, B = 4,096 after 512
# steps: opt-in (fp8 KV, window 256) and C3 (fp16) steps.  usage: tools/lanes_split_probe.sh OUT.jsonl
set -e
out=$1
for kv in "--kv fp8 --window 256" "--kv fp16"; do
  for lanes in "--lanes 1" "--lanes 2 --order split" "--lanes 2 --order split --cu-split 0.5" \
               "--lanes 2 --order split --cu-split 0.625" "--lanes 2 --order split --cu-split 0.75"; do
    timeout -k 10 240 python tools/replay_probe.py $kv $lanes --skip 512 --reps 32 --blocks 2 --eager >> "$out"
  done
done
