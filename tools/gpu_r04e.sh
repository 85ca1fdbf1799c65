# round 4: wide v2 (mean-pivot flushes, 16-bit ids, LDS-resident tail values, LDS-sort list kernel)
set -o pipefail
o=gpurun_out/r04e; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "wide or g4 or g5 or 50000 or 60000 or 2000 or masked or non_finite" > $o/pytest_parity.log 2>&1 || exit $?
NSG_WIDE_V2=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/wide -o run --output-format csv -- python tools/wide_probe.py --steps 10 > $o/wide.log 2>&1 || exit $?
NSG_WIDE_V2=1 timeout -k 10 120 python -u tools/wide_probe.py > $o/probe_v2.jsonl 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/c2prof -o run --output-format csv -- python tools/c2_probe.py > $o/c2.log 2>&1
