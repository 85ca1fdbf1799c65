#!/bin/bash
# Run the GPU test tier once under a time limit; fail if the HIP runtime reported a device fault.
# usage: tools/gpu_pytest.sh LOGFILE [extra pytest args]
log=$1; shift
timeout -k 10 600 python -m pytest tests -m gpu -x -q "$@" > "$log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$log"
if grep -q "HSA_STATUS_ERROR\|Memory access fault" "$log"; then echo "GPU FAULT reported" >> "$log"; exit 99; fi
exit $rc
