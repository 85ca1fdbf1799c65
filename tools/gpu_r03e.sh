set -o pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 300 python -u tools/bpe_debug.py > gpurun_out/r03e/bpe_debug.log 2>&1 ; \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "wide or stepwise or golden" > gpurun_out/r03e/parity.log 2>&1 && \
timeout -k 10 300 python tools/wide_timing.py --steps 10 > gpurun_out/r03e/wide.jsonl 2>&1 && \
timeout -k 10 300 python tools/wide_timing.py --steps 10 --dtype f16 >> gpurun_out/r03e/wide.jsonl 2>&1
