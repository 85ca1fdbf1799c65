# round 4: wide path v2 (stream + tail kernels) parity and timing, then the new parity tests of round 4
set -o pipefail
o=gpurun_out/r04b; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  > $o/pytest_parity.log 2>&1 || exit $?
NSG_WIDE_V2=1 timeout -k 10 120 python -u tools/wide_probe.py > $o/probe_v2.jsonl 2>&1 || exit $?
NSG_WIDE_V2=0 timeout -k 10 120 python -u tools/wide_probe.py > $o/probe_v1.jsonl 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_rank_coder.py tests/test_gpu_lm_kernels.py \
  tests/test_gpu_guard.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "rank or provider or crypto or queries or generic or seq_attention or native_prefill or invariant or scorer or max_context or cover" \
  > $o/pytest_new.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/c2prof -o run --output-format csv -- python tools/c2_probe.py > $o/c2.log 2>&1
