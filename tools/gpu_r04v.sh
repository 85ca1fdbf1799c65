#!/bin/bash
set -o pipefail
o=gpurun_out/r04v; mkdir -p $o
timeout -k 10 300 python -u tools/e2e_overhead_probe.py --kv fp8 --window 256 > $o/optin.json 2> $o/optin.err || exit $?
cat $o/optin.json
