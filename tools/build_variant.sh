#!/bin/bash
# Compile a tuning variant of the coder library: tools/build_variant.sh NAME [-DMACRO=VALUE ...]
# -> neuralsteganography_amd/_build/variants/NAME.so (same sources as __graft_entry__.build(), one object per source
# compiled in parallel).
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/neuralsteganography_amd/_build/variants
mkdir -p "$out/obj_$name"
c=$root/neuralsteganography_amd/csrc
pids=()
for s in nsg_coder nsg_wide nsg_attn nsg_score nsg_lm nsg_fraction; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wno-unused-function \
      -I "$root/include" "$@" -c -o "$out/obj_$name/$s.o" "$c/$s.hip" 2>/dev/null &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/$name.so" "$out"/obj_$name/*.o
rm -rf "$out/obj_$name"
echo "built variants/$name.so $*"
