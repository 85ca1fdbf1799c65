# round 4: coder append A/B -- set-bit appends (all dtypes) and packed fp16 groups, variant libraries vs default
set -o pipefail
o=gpurun_out/r04k; mkdir -p $o
VD=neuralsteganography_amd/_build/variants
for v in setbit f16n; do
  NSG_CODER_LIB=$VD/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "golden or stepwise or finish or masked or sample_tie or overflow or miss" > $o/pytest_$v.log 2>&1 || exit $?
done
C="--no-cpu-baseline --no-e2e --no-wide --no-pcie --no-f16-coder"
for rep in 1 2; do
for cfg in "--dtype f32 --topk 300" "--dtype f16 --topk 300" "--dtype f16 --topk 100"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 120 python bench.py $C $cfg > $o/base_$rep.$tag.json 2>/dev/null || exit $?
  NSG_CODER_LIB=$VD/setbit.so timeout -k 10 120 python bench.py $C $cfg > $o/setbit_$rep.$tag.json 2>/dev/null || exit $?
  case $cfg in *f16*) NSG_CODER_LIB=$VD/f16n.so timeout -k 10 120 python bench.py $C $cfg > $o/f16n_$rep.$tag.json 2>/dev/null || exit $? ;; esac
done
done
