#!/bin/bash
# round 4 final pass (library 0.16 + host-side fixes): the whole GPU suite, smoke, then the default bench line
set -o pipefail
o=gpurun_out/${TAG:-r04z}; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
tail -2 $o/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
tail -1 $o/smoke.log
timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err
rc=$?
tail -c 300 $o/bench.json
exit $rc
