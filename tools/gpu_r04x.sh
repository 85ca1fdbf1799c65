#!/bin/bash
# round 4: decode attention bandwidth mid-job (C3, cache length ~330-400)
set -o pipefail
o=gpurun_out/r04x; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python tools/replay_probe.py --skip 300 --reps 32 > $o/prof.log 2>&1
rc=$?
tail -2 $o/prof.log
exit $rc
