# wide-path phases (diagnostic early exits) + single-pass coder phases (fp32 topk 300, fp16 topk 100)
set -o pipefail
o=gpurun_out/r03q; mkdir -p $o
for lib in libnsgcoder.so variants/opdiag1.so variants/scandiag3.so variants/scandiag4.so; do
  timeout -k 10 300 python tools/wide_timing.py --steps 10 --lib neuralsteganography_amd/_build/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
  timeout -k 10 300 python tools/wide_timing.py --steps 10 --dtype f16 --lib neuralsteganography_amd/_build/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
done
timeout -k 10 300 python tools/phase_timing.py --dtype f16 --topk 100 > $o/phases_f16.jsonl 2>>$o/err.log && \
timeout -k 10 300 python tools/phase_timing.py > $o/phases_f32.jsonl 2>>$o/err.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python tools/wide_timing.py --steps 10 > $o/trace.log 2>&1 && \
find $o/trace -name '*kernel_stats.csv' -exec cp {} $o/wide_kernel_stats.csv \;
