# LM kernel tests + GEMM probe (all configurations) at B = 4096 and 1024
set -o pipefail  # usage: tools/gpu_r03n.sh TAG
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_lm_kernels.py -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 && \
timeout -k 10 300 python tools/lm_probe.py --batch 4096 --configs --no-step --lens 64 > $o/lmprobe_b4096.jsonl 2> $o/lmprobe.err && \
timeout -k 10 300 python tools/lm_probe.py --batch 1024 --model gpt2-medium --configs --no-step --lens 64 > $o/lmprobe_b1024_medium.jsonl 2>> $o/lmprobe.err
