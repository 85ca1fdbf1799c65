#!/bin/bash
# A/B phase timing of library variants on one box: tools/ab_phases.sh OUTDIR "phase_timing args" lib1 lib2 ...
# ("cur" = the in-tree build).  Each run under its own time limit; stops at the first failure.
set -e
out=$1; args=$2; shift 2
mkdir -p "$out"
for v in "$@"; do
    if [ "$v" = cur ]; then lib=""; else lib="--lib neuralsteganography_amd/_build/variants/$v.so"; fi
    timeout -k 10 150 python tools/phase_timing.py $lib $args > "$out/$v.jsonl" 2>&1
done
