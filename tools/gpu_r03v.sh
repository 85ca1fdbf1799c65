# sort-free wide tail: parity (wide / stepwise / golden / northstar C5), timing A/B vs the sorted tail, stamps
set -o pipefail
o=gpurun_out/r03v; mkdir -p $o
V=neuralsteganography_amd/_build
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_code_base_compat.py tests/test_gpu_sampler_stats.py > $o/parity.log 2>&1 || exit 1
for lib in libnsgcoder.so variants/sorted.so libnsgcoder.so; do
  timeout -k 10 200 python tools/wide_timing.py --steps 10 --lib $V/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
  timeout -k 10 200 python tools/wide_timing.py --steps 10 --dtype f16 --lib $V/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
done
timeout -k 10 200 python tools/stamp_wide.py --lib $V/variants/wstamps.so > $o/stamps_f32.json 2>>$o/err.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_northstar.py > $o/northstar.log 2>&1
