# round 4: wave-per-stream wide step (NSG_WIDE_V2=2): parity, timing, kernel split; C5 guard leg + f16/topk-300 PMC
set -o pipefail
o=gpurun_out/r04j; mkdir -p $o
NSG_WIDE_V2=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "wide or g4 or g5 or 50000 or 60000 or 2000 or masked or non_finite" > $o/pytest_parity_v3.log 2>&1 || exit $?
NSG_WIDE_V2=2 timeout -k 10 120 python -u tools/wide_probe.py > $o/probe_v3.jsonl 2>&1 || exit $?
NSG_WIDE_V2=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/wide -o run --output-format csv -- python tools/wide_probe.py --steps 10 > $o/wide.log 2>&1 || exit $?
