#!/bin/bash
# round 4: last check of the shipped library -- LM kernels, Fraction coder, parity subset, smoke
set -o pipefail
o=gpurun_out/r04af; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_lm_kernels.py tests/test_gpu_fraction.py tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
rc=$?
tail -1 $o/smoke.log
exit $rc
