#!/bin/bash
# round 4: Fraction coder throughput vs its CPU restatement, with a kernel trace
set -o pipefail
mkdir -p gpurun_out/r04m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/frac_probe.py --batch 4096 --vocab 16 --bytes 32 --sample 16 \
  > gpurun_out/r04m/probe_v16.jsonl 2> gpurun_out/r04m/probe_v16.err &&
timeout -k 10 300 python -u tools/frac_probe.py --batch 1024 --vocab 256 --bytes 8 --sample 1 \
  > gpurun_out/r04m/probe_v256.jsonl 2> gpurun_out/r04m/probe_v256.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04m/prof -o frac -- \
  python3 tools/frac_probe.py --batch 4096 --vocab 16 --bytes 32 --sample 2 > gpurun_out/r04m/prof.log 2>&1
rc=$?
cat gpurun_out/r04m/probe_v16.jsonl gpurun_out/r04m/probe_v256.jsonl
exit $rc
