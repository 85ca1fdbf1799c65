#!/bin/bash
# round 4: host-side list conversion fix -- overhead probe (opt-in, C3) + the north-star round-trip tests
set -o pipefail
o=gpurun_out/r04w; mkdir -p $o
timeout -k 10 300 python -u tools/e2e_overhead_probe.py --kv fp8 --window 256 > $o/optin.json 2> $o/optin.err || exit $?
timeout -k 10 300 python -u tools/e2e_overhead_probe.py > $o/c3.json 2> $o/c3.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_northstar.py tests/test_gpu_parity.py -x -v --timeout 600 --timeout-method thread > $o/pytest.log 2>&1
rc=$?
tail -3 $o/pytest.log
python -c "
import json
for f in ['optin','c3']:
    d=json.load(open('$o/'+f+'.json')); print(f, d['total'], d['steps'], sum(d['ms_per_16_steps'])/1e3)"
exit $rc
