#!/bin/bash
# round 4: PMC of GPT-2's c_fc at B = 4096 on the 192- and 256-wide ping-pong panels
set -o pipefail
o=gpurun_out/r04ai; mkdir -p $o
bash tools/gemm_pmc.sh $o 4096 3072 768 gelu 18 || exit $?
bash tools/gemm_pmc.sh $o 4096 3072 768 gelu 17 || exit $?
cat $o/time_*.txt
