# round 4: the default bench line (every leg), as the driver runs it
set -o pipefail
o=gpurun_out/r04h; mkdir -p $o
timeout -k 10 1000 python bench.py > $o/bench.json 2> $o/bench.err || exit $?
NSG_CODER_LIB=neuralsteganography_amd/_build/variants/w4.so timeout -k 10 120 python -u tools/wide_probe.py > $o/probe_w4.jsonl 2>&1
