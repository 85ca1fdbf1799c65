#!/bin/bash
# round 4: last library rebuild -- Fraction coder tests + smoke
set -o pipefail
o=gpurun_out/r04al; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_fraction.py tests/test_gpu_lm_kernels.py -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
rc=$?
tail -1 $o/smoke.log
exit $rc
