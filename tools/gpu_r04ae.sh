#!/bin/bash
# round 4: small-batch attention with the pair's q / k / v loads hoisted before the cache-length read -- LM kernel
# tests, C2 A/B
set -o pipefail
o=gpurun_out/r04ae; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_lm_kernels.py -x -q --timeout 300 --timeout-method thread > $o/pytest_lm.log 2>&1 || { tail -30 $o/pytest_lm.log; exit 1; }
tail -1 $o/pytest_lm.log
for rep in 1 2 3; do
for v in base noqpre; do
  if [ $v = base ]; then lib=""; else lib=$GRAFT_REPO_ROOT/neuralsteganography_amd/_build/variants/$v.so; fi
  echo -n "{\"variant\": \"$v\", \"r\": $rep, \"probe\": " >> $o/c2_ab.jsonl
  NSG_CODER_LIB=$lib timeout -k 10 200 python -u tools/c2_probe.py >> $o/c2_ab.jsonl 2>> $o/c2_ab.err || exit $?
  sed -i '$ s/$/}/' $o/c2_ab.jsonl
done
done
python -c "
import json
for l in open('$o/c2_ab.jsonl'): d=json.loads(l); print(d['variant'], d['r'], round(d['probe']['ms_per_step'],4))"
