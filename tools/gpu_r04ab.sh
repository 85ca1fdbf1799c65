#!/bin/bash
# round 4: auto GEMM configuration retune (C5 shapes) -- LM kernel tests, probe, C5 leg
set -o pipefail
o=gpurun_out/r04ab; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_lm_kernels.py -x -q --timeout 300 --timeout-method thread > $o/pytest_lm.log 2>&1 || { tail -30 $o/pytest_lm.log; exit 1; }
tail -1 $o/pytest_lm.log
timeout -k 10 400 python -u tools/lm_probe.py --batch 1024 --model gpt2-medium --lens 512 --no-step > $o/b1024m.jsonl 2> $o/b1024m.err || exit $?
timeout -k 10 600 python -u bench.py --no-c2 --no-c4 --no-c5-guard --no-wide --no-f16-coder --no-fraction --optin-window 0 --no-cpu-baseline --no-pcie > $o/bench.json 2> $o/bench.err
rc=$?
python -c "
import json; d=json.load(open('$o/bench.json')); print('C3', d['value'], d['ms_per_step']); c=d['end_to_end_c5']; print('C5', c['cover_tokens_per_s'], c['ms_per_step'], c.get('roundtrip_exact_fraction'))"
exit $rc
