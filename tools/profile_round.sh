#!/bin/bash
# Measurement pass for one round tag (run on the GPU box from the repo root):
#   1. bench.py default line (with cpu_baseline)             -> gpurun_out/prof_TAG/bench.json
#   2. rocprofv3 --kernel-trace --stats of the coder leg       -> gpurun_out/prof_TAG/trace/
#   3. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE)    -> gpurun_out/prof_TAG/pmc_*/
#   4. tools/pmc_traffic.py                                  -> gpurun_out/prof_TAG/pmc_traffic.json
# usage: tools/profile_round.sh TAG [bench args...]   (every GPU step under its own time limit; stops at
# the first failure)
set -e
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
ver=$(python -c 'from neuralsteganography_amd import _lib; print(_lib.version())')
echo "library: $ver" > "$out/version.txt"
timeout -k 10 300 python bench.py "$@" > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-e2e --no-wide --no-pcie "$@" > "$out/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$out/pmc_fetch" -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-e2e --no-wide --no-pcie --steps 20 --warmup 2 "$@" > "$out/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$out/pmc_write" -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-e2e --no-wide --no-pcie --steps 20 --warmup 2 "$@" > "$out/pmc_write.log" 2>&1
fetch=$(find "$out/pmc_fetch" -name '*counter_collection.csv' -print -quit)
write=$(find "$out/pmc_write" -name '*counter_collection.csv' -print -quit)
python tools/pmc_traffic.py "$fetch" "$write" "$out/pmc_traffic.json" --version "$ver"
cp "$fetch" "$out/pmc_fetch_size.csv"
cp "$write" "$out/pmc_write_size.csv"
find "$out/trace" -name '*kernel_stats.csv' -exec cp {} "$out/kernel_stats.csv" \;
echo "profile_round $tag done"
