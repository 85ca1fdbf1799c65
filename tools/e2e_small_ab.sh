#!/bin/bash
# Small-batch end-to-end A/B of library variants: VARIANTS="cur name ..." bash tools/e2e_small_ab.sh
set -e
for v in ${VARIANTS:-cur}; do
  if [ $v = cur ]; then unset NSG_CODER_LIB; else export NSG_CODER_LIB=neuralsteganography_amd/_build/variants/$v.so; fi
  for b in ${BATCHES:-1 64}; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-wide --no-pcie --no-cpu-baseline --optin-window 0 \
        --e2e-batch $b --e2e-payload-bytes ${PAYLOAD:-256} > gpurun_out/e2e_${v}_b$b.json 2>/dev/null
    python -c "
import json;d=json.loads(open('gpurun_out/e2e_${v}_b$b.json').read().strip().splitlines()[-1])
e=d['end_to_end'];print('$v B=$b', round(e['cover_tokens_per_s']), round(e['ms_per_step'],4), e['lockstep_steps'])"
  done
done
