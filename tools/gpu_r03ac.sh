# coder A/B: ring depth / occupancy (2 rounds of waves at B = 4096 so the second round's streams overlap the
# first round's tails), then a kernel trace of a short C3 end-to-end run (256-byte payloads) for the round
set -o pipefail
o=gpurun_out/r03ac; mkdir -p $o
V=neuralsteganography_amd/_build
for lib in libnsgcoder.so variants/pf8w2.so variants/pf8w3.so libnsgcoder.so variants/pf8w2.so; do
  timeout -k 10 200 python tools/phase_timing.py --full-only --lib $V/$lib >> $o/coder.jsonl 2>>$o/err.log || exit 1
  timeout -k 10 200 python tools/phase_timing.py --full-only --dtype f16 --topk 100 --lib $V/$lib >> $o/coder.jsonl 2>>$o/err.log || exit 1
done
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/e2e -o run --output-format csv -- python bench.py --no-cpu-baseline --no-wide --no-pcie --no-c2 --no-c4 --optin-window 0 --no-decode --e2e-payload-bytes 256 --steps 5 --warmup 2 > $o/e2e.log 2>&1
true
