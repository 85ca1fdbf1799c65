set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_northstar.py -k c5 tests/test_gpu_guard.py tests/test_gpu_rank_coder.py tests/test_gpu_code_base_compat.py tests/test_gpu_provider.py > gpurun_out/r03b/tests.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err
