# tail-kernel stamps (split sort-free diagnostic build), then the round measurement pass
set -o pipefail
mkdir -p gpurun_out/r03ab
timeout -k 10 200 python tools/stamp_tail.py --lib neuralsteganography_amd/_build/variants/tstamps.so > gpurun_out/r03ab/tail_stamps.json 2> gpurun_out/r03ab/tail_stamps.err
bash tools/profile_round.sh r03z
