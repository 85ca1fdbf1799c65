#!/bin/bash
# round 4: Fraction coder kernel parity (row a12)
set -o pipefail
mkdir -p gpurun_out/r04l
timeout -k 10 400 python -u -m pytest tests/test_gpu_fraction.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r04l/pytest_fraction.log 2>&1
rc=$?
tail -5 gpurun_out/r04l/pytest_fraction.log
exit $rc
