# round 4: wide v2 kernel split (rocprofv3), the rest of the new parity tests, the C2 step's kernel trace
set -o pipefail
o=gpurun_out/r04c; mkdir -p $o
NSG_WIDE_V2=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/wide -o run --output-format csv -- python tools/wide_probe.py --dtype f32 --steps 10 > $o/wide.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_rank_coder.py tests/test_gpu_lm_kernels.py \
  tests/test_gpu_guard.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "rank or provider or crypto or queries or generic or seq_attention or native_prefill or invariant or scorer or max_context or cover or ln_gemm" \
  > $o/pytest_new.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/c2prof -o run --output-format csv -- python tools/c2_probe.py > $o/c2.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_northstar.py -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "c4 or c2" > $o/pytest_ns.log 2>&1
