# full GPU suite + smoke + bench (one box): tools/gpu_full.sh TAG
set -o pipefail
o=gpurun_out/$1
mkdir -p $o
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $o/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" > $o/status.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && \
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err
