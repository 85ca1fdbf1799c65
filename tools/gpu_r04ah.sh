#!/bin/bash
# round 4: auto PP192/PP256 -- LM kernel tests, probe, full default bench line
set -o pipefail
o=gpurun_out/r04ah; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_lm_kernels.py tests/test_gpu_northstar.py -x -q --timeout 600 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 400 python -u tools/lm_probe.py --batch 4096 --lens 512 --no-step > $o/b4096.jsonl 2> $o/b4096.err || exit $?
timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err
rc=$?
python -c "
import json
for l in open('$o/b4096.jsonl'):
    d=json.loads(l)
    if 'gemm' in d: print(d['gemm'], round(d['tflops_native']), round(d['tflops_torch']))
d=json.load(open('$o/bench.json')); print('C3', d['value'], d['ms_per_step'], d['cover_tokens_per_s'], d['roundtrip_exact_fraction'])
for k in ('end_to_end_c4','end_to_end_c5','end_to_end_optin','end_to_end_c2'): print(k, d[k]['cover_tokens_per_s'], d[k]['ms_per_step'], d[k].get('roundtrip_exact_fraction'))"
exit $rc
