set -o pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_northstar.py::test_c5_like_gpt2_medium_topk100_guard_on_1024_secrets tests/test_gpu_guard.py tests/test_gpu_rank_coder.py tests/test_gpu_code_base_compat.py tests/test_gpu_provider.py > gpurun_out/r03c/tests.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r03c/bench.json 2> gpurun_out/r03c/bench.err
