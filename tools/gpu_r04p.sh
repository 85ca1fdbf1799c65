#!/bin/bash
# round 4 final pass, part 1 (library 0.16): coder f32 / f16 (topk 300) kernel traces + PMC FETCH/WRITE records
# (written to profiles/ so the bench in this call reads them), then the default bench line
set -o pipefail
o=gpurun_out/r04p; mkdir -p $o
export TMPDIR=/tmp
ver=$(python -c 'from neuralsteganography_amd import _lib; print(_lib.version())')
echo "$ver" > $o/version.txt
C="--no-cpu-baseline --no-e2e --no-wide --no-pcie --no-f16-coder --no-fraction"
run() {  # tag, bench args
  local t=$1; shift
  mkdir -p $o/$t
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/$t/trace -o run --output-format csv -- python bench.py $C "$@" > $o/$t/trace.log 2>&1 || return $?
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $o/$t/pmc_fetch -o run --output-format csv -- python bench.py $C --steps 20 --warmup 2 "$@" > $o/$t/pmc_fetch.log 2>&1 || return $?
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $o/$t/pmc_write -o run --output-format csv -- python bench.py $C --steps 20 --warmup 2 "$@" > $o/$t/pmc_write.log 2>&1 || return $?
}
run f32 && run f16 --dtype f16 || exit $?
for t in f32 f16; do
  fc=$(find $o/$t/pmc_fetch -name '*counter_collection.csv' | head -1)
  wc=$(find $o/$t/pmc_write -name '*counter_collection.csv' | head -1)
  python tools/pmc_traffic.py "$fc" "$wc" profiles/pmc_traffic_r04b_$t.json --version "$ver" --dtype $t --topk 300 \
    > $o/pmc_$t.json || exit $?
  cp profiles/pmc_traffic_r04b_$t.json $o/
done
timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err
rc=$?
tail -c 1500 $o/bench.json
exit $rc
