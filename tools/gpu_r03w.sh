# sort-free wide tail (noinline) vs sorted tail: timing + stamps + wide parity
set -o pipefail
o=gpurun_out/r03w; mkdir -p $o
V=neuralsteganography_amd/_build
for lib in libnsgcoder.so variants/sorted.so libnsgcoder.so; do
  timeout -k 10 200 python tools/wide_timing.py --steps 10 --lib $V/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
  timeout -k 10 200 python tools/wide_timing.py --steps 10 --dtype f16 --lib $V/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
done
timeout -k 10 200 python tools/stamp_wide.py --lib $V/variants/wstamps.so > $o/stamps_f32.json 2>>$o/err.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "wide or golden or stepwise or non_finite" > $o/parity.log 2>&1
