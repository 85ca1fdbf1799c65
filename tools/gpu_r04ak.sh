#!/bin/bash
# round 4: kernel trace of the C2 step (B = 1) on the final library
set -o pipefail
o=gpurun_out/r04ak; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 tools/c2_probe.py > $o/prof.log 2>&1
rc=$?
grep -h ms_per_step $o/prof.log
exit $rc
