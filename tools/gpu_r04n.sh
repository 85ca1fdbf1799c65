#!/bin/bash
# round 4: Fraction coder throughput (+ kernel trace); C2 (B = 1) A/B of the direct-GEMM workgroup size and the
# attention prefetch depth
set -o pipefail
mkdir -p gpurun_out/r04n
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/frac_probe.py --batch 4096 --vocab 16 --bytes 32 --sample 16 \
  > gpurun_out/r04n/frac_v16.jsonl 2> gpurun_out/r04n/frac_v16.err || exit $?
timeout -k 10 300 python -u tools/frac_probe.py --batch 1024 --vocab 256 --bytes 8 --sample 1 \
  > gpurun_out/r04n/frac_v256.jsonl 2> gpurun_out/r04n/frac_v256.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04n/prof -o frac -- \
  python3 tools/frac_probe.py --batch 4096 --vocab 16 --bytes 32 --sample 2 > gpurun_out/r04n/prof.log 2>&1 || exit $?
for rep in 1 2; do
for v in base nw1 nw2 pf3 pf4 nw1pf4 nw2pf4; do
  if [ $v = base ]; then lib=""; else lib=$GRAFT_REPO_ROOT/neuralsteganography_amd/_build/variants/$v.so; fi
  echo -n "{\"variant\": \"$v\", \"r\": $rep, \"probe\": " >> gpurun_out/r04n/c2_ab.jsonl
  NSG_CODER_LIB=$lib timeout -k 10 200 python -u tools/c2_probe.py >> gpurun_out/r04n/c2_ab.jsonl 2>> gpurun_out/r04n/c2_ab.err || exit $?
  sed -i '$ s/$/}/' gpurun_out/r04n/c2_ab.jsonl
done
done
cat gpurun_out/r04n/frac_v16.jsonl gpurun_out/r04n/frac_v256.jsonl gpurun_out/r04n/c2_ab.jsonl
