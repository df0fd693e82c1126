#!/bin/bash
# Same-box A/B of library variants (tools/var/lib_<name>.so), alternating, bench only:
#   tools/var_ab.sh "EXTRA BENCH ARGS" base new
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ARGS=$1; shift
for i in 1 2; do
  for name in "$@"; do
    TTSHIP_LIB=tools/var/lib_$name.so timeout -k 10 150 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --f32-steps 0 --r1-steps 0 $ARGS \
      > gpurun_out/ab_$name$i.json 2> gpurun_out/ab_$name$i.err || { echo "$name failed"; tail -3 gpurun_out/ab_$name$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$name$i.json')); print('$name$i', d['ms_per_step'], d['decoder_step_us'], d['tacotron2_ms'], d['vocoder_ms'], d['roofline']['launches'])"
  done
done
