#!/bin/bash
# round 4: 192-wide ping-pong GEMM tiles (one tile per CU for GPT-2's c_fc at B = 4096) -- tests + config sweep
set -o pipefail
o=gpurun_out/r04ag; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_lm_kernels.py -x -q --timeout 300 --timeout-method thread > $o/pytest_lm.log 2>&1 || { tail -30 $o/pytest_lm.log; exit 1; }
tail -1 $o/pytest_lm.log
timeout -k 10 400 python -u tools/lm_probe.py --batch 4096 --lens 512 --configs --no-step > $o/b4096.jsonl 2> $o/b4096.err || exit $?
timeout -k 10 400 python -u tools/lm_probe.py --batch 1024 --model gpt2-medium --lens 512 --configs --no-step > $o/b1024m.jsonl 2> $o/b1024m.err
rc=$?
python -c "
import json
for f in ['b4096','b1024m']:
    for l in open('$o/'+f+'.jsonl'):
        d=json.loads(l)
        if 'tflops_by_config' in d:
            c=d['tflops_by_config']; print(f, d['gemm'], 'pp256', c.get('17'), 'pp192', c.get('18'), 'best', max(c, key=lambda k: c[k]), round(max(c.values())), 'torch', round(d['tflops_torch']))"
exit $rc
