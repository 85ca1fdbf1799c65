# round 4: the whole GPU suite on the current tree, then smoke
set -o pipefail
o=gpurun_out/r04g; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
