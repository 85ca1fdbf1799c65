set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03i
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "wide or stepwise or golden" > $o/parity.log 2>&1 && \
for lib in libnsgcoder.so variants/opdiag1.so variants/op2cu.so variants/op2cu_diag1.so; do
  timeout -k 10 300 python tools/wide_timing.py --steps 10 --lib neuralsteganography_amd/_build/$lib >> $o/wide.jsonl 2>/dev/null || exit 1
  timeout -k 10 300 python tools/wide_timing.py --steps 10 --dtype f16 --lib neuralsteganography_amd/_build/$lib >> $o/wide.jsonl 2>/dev/null || exit 1
done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python tools/wide_timing.py --steps 10 > $o/trace.log 2>&1 && \
find $o/trace -name '*kernel_stats.csv' -exec cp {} $o/wide_kernel_stats.csv \; && \
NSG_CODER_LIB=neuralsteganography_amd/_build/variants/op2cu.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace2 -o run --output-format csv -- python tools/wide_timing.py --steps 10 --lib neuralsteganography_amd/_build/variants/op2cu.so > $o/trace2.log 2>&1 && \
find $o/trace2 -name '*kernel_stats.csv' -exec cp {} $o/wide_kernel_stats_2cu.csv \;
