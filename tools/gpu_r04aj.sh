#!/bin/bash
# round 4: the whole GPU suite and smoke on the final library (192-wide GEMM panels)
set -o pipefail
o=gpurun_out/r04aj; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
rc=$?
tail -1 $o/smoke.log
exit $rc
