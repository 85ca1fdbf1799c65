set -e
for v in ${VARIANTS:-cur}; do
  if [ $v = cur ]; then unset NSG_CODER_LIB; else export NSG_CODER_LIB=neuralsteganography_amd/_build/variants/$v.so; fi
  for kv in fp8 fp16; do
    timeout -k 10 200 python tools/lm_probe.py --attn-only --kv $kv --lens 64,128,256,384,512,1024 --reps 20 --no-step > gpurun_out/attn_${v}_$kv.jsonl 2>&1
  done
done
unset NSG_CODER_LIB
for f in gpurun_out/attn_*.jsonl; do echo $f; grep attention $f | python -c "
import sys,json
print(' '.join(f\"L{d['attention_L']}:{d['GBs']/1000:.2f}\" for d in map(json.loads,sys.stdin)))"; done
