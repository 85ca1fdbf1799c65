#!/bin/bash
# C2 (one stream) token time, base library vs a variant, alternating on one box: tools/c2_ab.sh VARIANT OUT.txt
set -e
v=$1; out=$2
for k in 1 2; do
  for lib in base $v; do
    if [ $lib = base ]; then unset NSG_CODER_LIB; else export NSG_CODER_LIB=neuralsteganography_amd/_build/variants/$lib.so; fi
    echo -n "$lib " >> "$out"
    timeout -k 10 120 python tools/c2_probe.py >> "$out"
  done
done
