#!/bin/bash
# Compile a tuning variant of the coder library: tools/build_variant.sh NAME [-DMACRO=VALUE ...]
# -> neuralsteganography_amd/_build/variants/NAME.so (same sources as __graft_entry__.build()).
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/neuralsteganography_amd/_build/variants"
c=$root/neuralsteganography_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-function \
    -I "$root/include" "$@" -o "$root/neuralsteganography_amd/_build/variants/$name.so" \
    "$c/nsg_coder.hip" "$c/nsg_wide.hip" "$c/nsg_attn.hip" "$c/nsg_score.hip" "$c/nsg_lm.hip" "$c/nsg_fraction.hip"
echo "built variants/$name.so $*"
