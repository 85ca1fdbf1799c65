#!/bin/bash
# round 4: attention K/V load policy A/B (mid-job C3 step, HIP events)
set -o pipefail
o=gpurun_out/r04y; mkdir -p $o
for rep in 1 2; do
for v in base attplain; do
  if [ $v = base ]; then lib=""; else lib=$GRAFT_REPO_ROOT/neuralsteganography_amd/_build/variants/$v.so; fi
  echo -n "{\"variant\": \"$v\", \"r\": $rep, \"probe\": " >> $o/ab.jsonl
  NSG_CODER_LIB=$lib timeout -k 10 200 python -u tools/replay_probe.py --skip 300 --reps 32 >> $o/ab.jsonl 2>> $o/ab.err || exit $?
  sed -i '$ s/$/}/' $o/ab.jsonl
done
done
cat $o/ab.jsonl
