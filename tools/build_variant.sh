#!/bin/bash
# Compile a tuning variant of the coder library: tools/build_variant.sh NAME [-DMACRO=VALUE ...]
# -> neuralsteganography_amd/_build/variants/NAME.so (same sources as __graft_entry__.build(), one object per source
# compiled in parallel).  Each compile's messages go to obj_NAME/SOURCE.log, printed when that compile fails; the
# object directory is removed on every exit.
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/neuralsteganography_amd/_build/variants
obj=$out/obj_$name
mkdir -p "$obj"
trap 'rm -rf "$obj"' EXIT
c=$root/neuralsteganography_amd/csrc
srcs=(nsg_coder nsg_wide nsg_attn nsg_score nsg_lm nsg_fraction)
pids=()
for s in "${srcs[@]}"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wno-unused-function \
      -I "$root/include" "$@" -c -o "$obj/$s.o" "$c/$s.hip" > "$obj/$s.log" 2>&1 &
  pids+=($!)
done
failed=0
for i in "${!pids[@]}"; do
  if ! wait "${pids[$i]}"; then
    echo "build_variant: ${srcs[$i]}.hip failed:" >&2
    cat "$obj/${srcs[$i]}.log" >&2
    failed=1
  fi
done
[ "$failed" = 0 ] || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/$name.so" "$obj"/*.o
echo "built variants/$name.so $*"
