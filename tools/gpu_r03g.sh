set -o pipefail
o=gpurun_out/r03g
mkdir -p $o
for lib in variants/opdiag1.so variants/opdiag1_noapp.so variants/opdiag1_noapp_noupd.so variants/opdiag1_ring8.so variants/old_p1.so variants/old_p1_nt.so; do
  timeout -k 10 300 python tools/wide_timing.py --steps 10 --lib neuralsteganography_amd/_build/$lib >> $o/wide.jsonl 2>/dev/null || exit 1
  timeout -k 10 300 python tools/wide_timing.py --steps 10 --dtype f16 --lib neuralsteganography_amd/_build/$lib >> $o/wide.jsonl 2>/dev/null || exit 1
done
