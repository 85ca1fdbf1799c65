# library 0.14: full GPU suite + smoke, then the fp16 coder (C5's configuration: topk 100) rocprof + PMC record
set -o pipefail
o=gpurun_out/r03y; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" > $o/status.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
A="--no-cpu-baseline --no-e2e --no-wide --no-pcie --dtype f16 --topk 100"
timeout -k 10 200 python bench.py $A > $o/bench_f16.json 2> $o/bench_f16.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/trace_f16 -o run --output-format csv -- python bench.py $A > $o/trace_f16.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $o/pmc_fetch_f16 -o run --output-format csv -- python bench.py $A --steps 20 --warmup 2 > $o/pmc_fetch_f16.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $o/pmc_write_f16 -o run --output-format csv -- python bench.py $A --steps 20 --warmup 2 > $o/pmc_write_f16.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_WAVES -d $o/pmc_sq_f16 -o run --output-format csv -- python bench.py $A --steps 20 --warmup 2 > $o/pmc_sq_f16.log 2>&1
true
