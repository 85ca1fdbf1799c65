# round 4: PMC + trace of the headline's coder (f16 rows, topk 300), the C5 guard leg alone, the C2 probe
set -o pipefail
o=gpurun_out/r04i; mkdir -p $o/f16k300
export TMPDIR=/tmp
C="--no-cpu-baseline --no-e2e --no-wide --no-pcie --no-f16-coder --dtype f16 --topk 300"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/f16k300/trace -o run --output-format csv -- python bench.py $C > $o/f16k300/trace.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $o/f16k300/pmc_fetch -o run --output-format csv -- python bench.py $C --steps 20 --warmup 2 > $o/f16k300/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $o/f16k300/pmc_write -o run --output-format csv -- python bench.py $C --steps 20 --warmup 2 > $o/f16k300/pmc_write.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/c5_guard_probe.py > $o/c5_guard.json 2> $o/c5_guard.err || exit $?
timeout -k 10 200 python -u tools/c2_probe.py > $o/c2.json 2>&1
