#!/bin/bash
# round 4: every GEMM tile configuration on the decode-step shapes (B = 4096 gpt2, B = 1024 gpt2-medium)
set -o pipefail
o=gpurun_out/r04aa; mkdir -p $o
timeout -k 10 400 python -u tools/lm_probe.py --batch 4096 --lens 512 --configs --no-step > $o/b4096.jsonl 2> $o/b4096.err || exit $?
timeout -k 10 400 python -u tools/lm_probe.py --batch 1024 --model gpt2-medium --lens 512 --configs --no-step > $o/b1024m.jsonl 2> $o/b1024m.err
rc=$?
wc -l $o/*.jsonl
exit $rc
