#!/bin/bash
# The paged attention probe over the shapes that matter (dense chunk planes vs layer-major pages), one JSON line each:
# tools/attn_probe_set.sh OUT.jsonl
set -e
out=$1
for args in "--L 160" "--L 544" "--L 900" "--L 544 --kv fp8 --window 256" "--B 1 --L 544"; do
  timeout -k 10 120 python tools/paged_attn_probe.py $args --only ac --steps 50 >> "$out"
done
