#!/bin/bash
# Paged attention row sums by DPP moves (base) vs ds_bpermute (variant nodpp): probe set, alternating twice.
# usage: tools/dpp_ab.sh OUT.txt [VARIANT]
set -e
out=$1
for k in 1 2; do
  for v in base ${2:-nodpp}; do
    if [ $v = base ]; then unset NSG_CODER_LIB; else export NSG_CODER_LIB=neuralsteganography_amd/_build/variants/$v.so; fi
    for args in "--B 4096 --L 160" "--B 4096 --L 544" "--B 4096 --L 900" "--B 4096 --L 544 --kv fp8 --window 256" "--B 4096 --L 544 --kv fp8" "--B 1 --L 544"; do
      echo -n "$v $args " >> "$out"
      timeout -k 10 120 python tools/paged_attn_probe.py $args --only c --steps 50 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_ms']*1000,2), 'us', round(d['GBps']))" >> "$out"
    done
  done
done
