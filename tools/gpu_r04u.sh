#!/bin/bash
# round 4: sustained replay of the opt-in step (clock under load?)
set -o pipefail
o=gpurun_out/r04u; mkdir -p $o
timeout -k 10 300 python -u tools/replay_probe.py --kv fp8 --window 256 --skip 260 --reps 50 --blocks 20 > $o/optin.json 2> $o/optin.err || exit $?
cat $o/optin.json
