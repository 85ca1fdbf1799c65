#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group, kernel counters only) over tools/phase_timing.py,
# summarised per phase by tools/pmc_phases.py.  usage: tools/pmc_phases.sh TAG [phase_timing args]
set -e
tag=$1; shift
out=gpurun_out/pmcph_$tag
mkdir -p "$out"
export TMPDIR=/tmp
groups=("SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH"
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"
        "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA")
i=0
csvs=()
for g in "${groups[@]}"; do
    timeout -k 10 300 rocprofv3 --pmc $g -d "$out/g$i" -o run --output-format csv -- \
        python tools/phase_timing.py --steps 10 "$@" > "$out/g$i.log" 2>&1
    csvs+=("$(find "$out/g$i" -name '*counter_collection.csv' -print -quit)")
    i=$((i + 1))
done
python tools/pmc_phases.py --steps 10 "$out/pmc_phases.json" "${csvs[@]}" | tee "$out/summary.txt"
