set -o pipefail
o=gpurun_out/r03j
mkdir -p $o
for lib in libnsgcoder.so variants/opdiag1.so variants/op_d3.so variants/op_d4.so variants/op_w8.so; do
  timeout -k 10 300 python tools/wide_timing.py --steps 10 --lib neuralsteganography_amd/_build/$lib >> $o/wide.jsonl 2>/dev/null || exit 1
  timeout -k 10 300 python tools/wide_timing.py --steps 10 --dtype f16 --lib neuralsteganography_amd/_build/$lib >> $o/wide.jsonl 2>/dev/null || exit 1
done
