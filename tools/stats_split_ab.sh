#!/bin/bash
# Statistics-build coder step (EncodeSession(stats=True), the code_base entry points) at B = 1 / 64 in both
# single-pass forms, then the GPU tests that check the statistics.  Run on the GPU box from the repo root.
set -e
for b in 1 64; do
  NSG_SPLIT_MAX_B=0 timeout -k 10 120 python tools/phase_timing.py --batch $b --stats --full-only > gpurun_out/stats_wave_b$b.jsonl 2>&1
  timeout -k 10 120 python tools/phase_timing.py --batch $b --stats --full-only > gpurun_out/stats_split_b$b.jsonl 2>&1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampler_stats.py tests/test_gpu_code_base_compat.py tests/test_gpu_provider.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_stats_split.log 2>&1
