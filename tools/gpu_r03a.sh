set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_northstar.py > gpurun_out/r03a/northstar.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
