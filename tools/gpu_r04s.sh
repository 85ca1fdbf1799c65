#!/bin/bash
# round 4: timed-region overheads of the end-to-end encode (prefill, first step + capture, host checks)
set -o pipefail
o=gpurun_out/r04s; mkdir -p $o
timeout -k 10 300 python -u tools/e2e_overhead_probe.py > $o/c3.json 2> $o/c3.err || exit $?
timeout -k 10 300 python -u tools/e2e_overhead_probe.py --kv fp8 --window 256 > $o/optin.json 2> $o/optin.err || exit $?
cat $o/c3.json $o/optin.json
