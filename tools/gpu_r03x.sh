# wide path A/B: sort-free vs sorted tail, per-tile vs group appends, 512- vs 256-thread workgroups
set -o pipefail
o=gpurun_out/r03x; mkdir -p $o
V=neuralsteganography_amd/_build
for lib in libnsgcoder.so variants/sorted.so variants/v_ns.so variants/v_s.so variants/v_ns256.so variants/v_s256.so; do
  timeout -k 10 200 python tools/wide_timing.py --steps 10 --lib $V/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
  timeout -k 10 200 python tools/wide_timing.py --steps 10 --dtype f16 --lib $V/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
done
for lib in v_ns256 v_ns; do
  NSG_CODER_LIB=$V/variants/$lib.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "wide or golden or stepwise or non_finite" > $o/parity_$lib.log 2>&1
done
