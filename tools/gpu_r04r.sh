#!/bin/bash
# round 4: where the opt-in step (fp8 KV + 256-position window, B = 4096) spends its time
set -o pipefail
o=gpurun_out/r04r; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c2_probe.py --batch 4096 --kv fp8 --window 256 > $o/optin.json 2> $o/optin.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python tools/c2_probe.py --batch 4096 --kv fp8 --window 256 > $o/prof.log 2>&1
rc=$?
cat $o/optin.json
exit $rc
