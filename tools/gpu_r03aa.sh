# split wide step (stream kernel + tail kernel) A/B and parity
set -o pipefail
o=gpurun_out/r03aa; mkdir -p $o
V=neuralsteganography_amd/_build
NSG_CODER_LIB=$V/variants/s1_ns.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "wide or golden or stepwise or non_finite" > $o/parity_s1_ns.log 2>&1 || exit 1
for lib in variants/base.so variants/s1_ns.so variants/s1_sorted.so variants/s1_ns_w6.so variants/base.so variants/s1_ns.so; do
  timeout -k 10 200 python tools/wide_timing.py --steps 10 --lib $V/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
  timeout -k 10 200 python tools/wide_timing.py --steps 10 --dtype f16 --lib $V/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
done
export TMPDIR=/tmp
NSG_CODER_LIB=$V/variants/s1_ns.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python tools/wide_timing.py --steps 10 --lib $V/variants/s1_ns.so > $o/trace.log 2>&1
true
