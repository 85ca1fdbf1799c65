# round 4, first GPU pass: new parity tests (masked rows, provider rows at float64, max_context, native sequence
# forward, guard invariance), then the C4 / C2 north-star round trips
set -o pipefail
o=gpurun_out/r04a; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_rank_coder.py tests/test_gpu_parity.py tests/test_gpu_lm_kernels.py \
  tests/test_gpu_guard.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "masked or non_finite or rank or provider or crypto or queries or generic or seq_attention or native_prefill or invariant or scorer or max_context or cover" \
  > $o/pytest_new.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_northstar.py -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "c4 or c2" > $o/pytest_ns.log 2>&1
