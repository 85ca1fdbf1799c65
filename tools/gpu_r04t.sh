#!/bin/bash
# round 4: host cost of a graph replay vs the step's GPU time (C3 and the opt-in mode)
set -o pipefail
o=gpurun_out/r04t; mkdir -p $o
timeout -k 10 300 python -u tools/replay_probe.py > $o/c3.json 2> $o/c3.err || exit $?
timeout -k 10 300 python -u tools/replay_probe.py --kv fp8 --window 256 > $o/optin.json 2> $o/optin.err || exit $?
cat $o/c3.json $o/optin.json
