#!/bin/bash
# round 4: cross-workgroup small-batch attention + one-wave direct GEMMs: LM kernel tests, C2 A/B, C2 trace
set -o pipefail
mkdir -p gpurun_out/r04o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lm_kernels.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04o/pytest_lm.log 2>&1 || { tail -30 gpurun_out/r04o/pytest_lm.log; exit 1; }
tail -3 gpurun_out/r04o/pytest_lm.log
for rep in 1 2; do
for v in base noxwg nw4; do
  if [ $v = base ]; then lib=""; else lib=$GRAFT_REPO_ROOT/neuralsteganography_amd/_build/variants/$v.so; fi
  echo -n "{\"variant\": \"$v\", \"r\": $rep, \"probe\": " >> gpurun_out/r04o/c2_ab.jsonl
  NSG_CODER_LIB=$lib timeout -k 10 200 python -u tools/c2_probe.py >> gpurun_out/r04o/c2_ab.jsonl 2>> gpurun_out/r04o/c2_ab.err || exit $?
  sed -i '$ s/$/}/' gpurun_out/r04o/c2_ab.jsonl
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04o/prof -o c2 -- python3 tools/c2_probe.py \
  > gpurun_out/r04o/prof.log 2>&1 || exit $?
cat gpurun_out/r04o/c2_ab.jsonl
