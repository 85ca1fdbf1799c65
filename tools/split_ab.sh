set -e
mkdir -p gpurun_out/r06l
for v in base rows128 rows64; do
  if [ $v = base ]; then unset NSG_CODER_LIB; else export NSG_CODER_LIB=neuralsteganography_amd/_build/variants/$v.so; fi
  for args in "--B 1 --L 544" "--B 1 --L 160" "--B 1 --L 1000" "--B 4096 --L 544" "--B 4096 --L 160" "--B 4096 --L 900" "--B 4096 --L 544 --kv fp8 --window 256"; do
    echo -n "$v $args " >> gpurun_out/r06l/split.txt
    timeout -k 10 120 python tools/paged_attn_probe.py $args --only c --steps 50 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_ms']*1000,2), 'us', round(d['GBps']))" >> gpurun_out/r06l/split.txt
  done
done
