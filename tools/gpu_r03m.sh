# rank coder tail of the suite + LM kernel tests after the GELU change, then the GEMM probe at B = 4096
set -o pipefail
o=gpurun_out/r03m; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_rank_coder.py tests/test_gpu_sampler_stats.py tests/test_gpu_lm_kernels.py -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 && \
timeout -k 10 300 python tools/lm_probe.py --batch 4096 --configs --no-step --lens 64 > $o/lmprobe_b4096.jsonl 2> $o/lmprobe.err
