#!/bin/bash
# fp8 pages with the register double buffer in multi-pair workgroups (NSG_ATT_DB8) vs the base library: the paged
# attention alone (fp8, window 256 and unbounded) and the opt-in decode step.  usage: tools/db8_ab.sh OUT.txt
set -e
out=$1
for v in base db8 db8w4 base db8; do
  if [ $v = base ]; then unset NSG_CODER_LIB; else export NSG_CODER_LIB=neuralsteganography_amd/_build/variants/$v.so; fi
  for args in "--B 4096 --L 544 --kv fp8 --window 256" "--B 4096 --L 544 --kv fp8" "--B 4096 --L 160 --kv fp8"; do
    echo -n "$v $args " >> "$out"
    timeout -k 10 120 python tools/paged_attn_probe.py $args --only c --steps 50 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_ms']*1000,2), 'us', round(d['GBps']))" >> "$out"
  done
done
for v in base db8; do
  if [ $v = base ]; then unset NSG_CODER_LIB; else export NSG_CODER_LIB=neuralsteganography_amd/_build/variants/$v.so; fi
  echo -n "$v optin-step " >> "$out"
  timeout -k 10 240 python tools/replay_probe.py --kv fp8 --window 256 --skip 512 --reps 32 --blocks 2 >> "$out"
done
