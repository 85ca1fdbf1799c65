# wide-kernel stamp timeline (f32, f16) + C3 / opt-in end to end after the KV-cache sizing fix
set -o pipefail
o=gpurun_out/r03s; mkdir -p $o
timeout -k 10 200 python tools/stamp_wide.py --lib neuralsteganography_amd/_build/variants/wstamps.so > $o/stamps_f32.json 2>>$o/err.log && \
timeout -k 10 200 python tools/stamp_wide.py --lib neuralsteganography_amd/_build/variants/wstamps.so --dtype f16 > $o/stamps_f16.json 2>>$o/err.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-wide --no-c4 --no-c2 --no-cpu-baseline --no-pcie > $o/bench.json 2> $o/bench.err
