#!/bin/bash
# round 4 final pass, part 2 (library 0.16): the whole GPU suite, then smoke
set -o pipefail
o=gpurun_out/r04q; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
tail -3 $o/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
rc=$?
tail -3 $o/smoke.log
exit $rc
