# A/B: tail s_setprio (wide one-pass kernel and single-pass coder), same box
set -o pipefail
o=gpurun_out/r03t; mkdir -p $o
V=neuralsteganography_amd/_build
for lib in libnsgcoder.so variants/prio1.so variants/prio3.so libnsgcoder.so; do
  timeout -k 10 200 python tools/wide_timing.py --steps 10 --lib $V/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
  timeout -k 10 200 python tools/wide_timing.py --steps 10 --dtype f16 --lib $V/$lib >> $o/wide.jsonl 2>>$o/err.log || exit 1
  timeout -k 10 200 python tools/phase_timing.py --full-only --lib $V/$lib >> $o/coder.jsonl 2>>$o/err.log || exit 1
  timeout -k 10 200 python tools/phase_timing.py --full-only --dtype f16 --topk 100 --lib $V/$lib >> $o/coder.jsonl 2>>$o/err.log || exit 1
done
timeout -k 10 200 python tools/stamp_wide.py --lib $V/variants/wstamps_p3.so > $o/stamps_p3_f32.json 2>>$o/err.log
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $o/counters_list.txt 2>&1
grep -E "SQC_ICACHE|SQ_IFETCH|SQ_WAIT_INST|SQ_INST_CYCLES|SQ_BUSY" $o/counters_list.txt | head -n 40 > $o/counters_icache.txt
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $o/pmc1 -o run --output-format csv -- python tools/wide_timing.py --steps 4 > $o/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES -d $o/pmc2 -o run --output-format csv -- python tools/wide_timing.py --steps 4 > $o/pmc2.log 2>&1
true
