# round 4 measurement pass (library 0.15): coder f32 (topk 300) and f16 (topk 100) kernel traces + PMC FETCH/WRITE,
# the wide path's kernel trace + PMC (one-pass default), and the C3 end-to-end kernel trace (native prefill)
set -o pipefail
o=gpurun_out/r04f; mkdir -p $o
export TMPDIR=/tmp
ver=$(python -c 'from neuralsteganography_amd import _lib; print(_lib.version())')
echo "$ver" > $o/version.txt
C="--no-cpu-baseline --no-e2e --no-wide --no-pcie --no-f16-coder"
run() {  # tag, bench args
  local t=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/$t/trace -o run --output-format csv -- python bench.py $C "$@" > $o/$t/trace.log 2>&1 || return $?
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $o/$t/pmc_fetch -o run --output-format csv -- python bench.py $C --steps 20 --warmup 2 "$@" > $o/$t/pmc_fetch.log 2>&1 || return $?
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $o/$t/pmc_write -o run --output-format csv -- python bench.py $C --steps 20 --warmup 2 "$@" > $o/$t/pmc_write.log 2>&1 || return $?
}
mkdir -p $o/f32 $o/f16
run f32 && run f16 --dtype f16 --topk 100 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/wide/trace -o run --output-format csv -- python tools/wide_probe.py --dtype f32 --steps 10 > $o/wide_trace.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $o/wide/pmc_fetch -o run --output-format csv -- python tools/wide_probe.py --dtype f32 --steps 10 > $o/wide_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $o/wide/pmc_write -o run --output-format csv -- python tools/wide_probe.py --dtype f32 --steps 10 > $o/wide_write.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/e2e -o run --output-format csv -- python bench.py --no-cpu-baseline --no-wide --no-pcie --no-c2 --no-c4 --no-c5 --no-c5-guard --no-f16-coder --optin-window 0 --no-decode --e2e-payload-bytes 256 --steps 5 --warmup 2 > $o/e2e.log 2>&1
