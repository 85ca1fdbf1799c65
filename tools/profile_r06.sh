#!/bin/bash
# Round-6 measurement pass (run on the GPU box from the repo root; every GPU step under its own time limit, stops at
# the first failure):
#   1. rocprofv3 --kernel-trace --stats of the coder legs (fp32 + fp16 coder, topk 300)    -> $out/coder_trace
#   2. FETCH_SIZE / WRITE_SIZE passes of the fp16 coder (the headline roofline's kernel)    -> pmc_traffic_f16.json
#   3. the same for the paged decode attention at L = 544 (tools/attn_bench.py)             -> pmc_traffic_attn.json
#   4. the same for the wide path's one-pass kernel (api default quality)                   -> pmc_traffic_wide.json
# usage: tools/profile_r06.sh OUT_DIR
set -e
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
ver=$(python -c 'from neuralsteganography_amd import _lib; print(_lib.version())')
echo "library: $ver" > "$out/version.txt"
coder="bench.py --no-cpu-baseline --no-e2e --no-wide --no-pcie --no-fraction"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/coder_trace" -o run --output-format csv -- \
    python $coder > "$out/coder_trace.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d "$out/pmc_f16_$c" -o run --output-format csv -- \
      python $coder --dtype f16 --no-f16-coder --steps 20 --warmup 2 > "$out/pmc_f16_$c.log" 2>&1
done
python tools/pmc_traffic.py "$(find "$out/pmc_f16_FETCH_SIZE" -name '*counter_collection.csv' -print -quit)" \
    "$(find "$out/pmc_f16_WRITE_SIZE" -name '*counter_collection.csv' -print -quit)" "$out/pmc_traffic_f16.json" \
    --version "$ver" --dtype f16 --topk 300 --batch 4096 > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/attn_trace" -o run --output-format csv -- \
    python tools/attn_bench.py --L 544 > "$out/attn_trace.log" 2>&1
alg=$(python -c 'B,H,D,T0,L=4096,12,64,32,544; print(B*H*(L+1-T0)*2*D*2 + H*T0*2*D*2 + B*3*H*D*2 + B*H*D*2)')
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d "$out/pmc_attn_$c" -o run --output-format csv -- \
      python tools/attn_bench.py --L 544 > "$out/pmc_attn_$c.log" 2>&1
done
python tools/pmc_traffic.py "$(find "$out/pmc_attn_FETCH_SIZE" -name '*counter_collection.csv' -print -quit)" \
    "$(find "$out/pmc_attn_WRITE_SIZE" -name '*counter_collection.csv' -print -quit)" "$out/pmc_traffic_attn.json" \
    --version "$ver" --kernel paged_attn_kernel --L 544 --alg-bytes "$alg" --dtype f16 > /dev/null
wide="bench.py --no-cpu-baseline --no-e2e --no-pcie --no-fraction --no-f16-coder --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/wide_trace" -o run --output-format csv -- \
    python $wide > "$out/wide_trace.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d "$out/pmc_wide_$c" -o run --output-format csv -- \
      python $wide > "$out/pmc_wide_$c.log" 2>&1
done
python tools/pmc_traffic.py "$(find "$out/pmc_wide_FETCH_SIZE" -name '*counter_collection.csv' -print -quit)" \
    "$(find "$out/pmc_wide_WRITE_SIZE" -name '*counter_collection.csv' -print -quit)" "$out/pmc_traffic_wide.json" \
    --version "$ver" --kernel wide_onepass_kernel --dtype f32 --topk 50000 > /dev/null
echo "profile_r06 done"
