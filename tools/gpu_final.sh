# final validation of the round's tree: full GPU suite, smoke, default bench + the C5 share line
set -o pipefail
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" > $o/status.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && \
timeout -k 10 900 python bench.py --c5 > $o/bench.json 2> $o/bench.err
