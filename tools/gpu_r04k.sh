# round 4: set-bit append A/B for the single-pass coder (variant library vs default), parity with the variant
set -o pipefail
o=gpurun_out/r04k; mkdir -p $o
V=neuralsteganography_amd/_build/variants/setbit.so
NSG_CODER_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "golden or stepwise or finish or masked or sample_tie or overflow or miss" > $o/pytest_setbit.log 2>&1 || exit $?
C="--no-cpu-baseline --no-e2e --no-wide --no-pcie --no-f16-coder"
for rep in 1 2; do
for cfg in "--dtype f32 --topk 300" "--dtype f16 --topk 300" "--dtype f16 --topk 100"; do
  timeout -k 10 120 python bench.py $C $cfg > $o/base_$rep.$(echo $cfg | tr -d ' -').json 2>/dev/null || exit $?
  NSG_CODER_LIB=$V timeout -k 10 120 python bench.py $C $cfg > $o/setbit_$rep.$(echo $cfg | tr -d ' -').json 2>/dev/null || exit $?
done
done
