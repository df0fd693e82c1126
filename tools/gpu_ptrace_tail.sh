#!/bin/bash
# Persistent-decoder phase traces of one bench step: the MT = 2 launch (steps 100..107) and the
# MT = 1 tail launch (steps 340..347), tools/ptrace.py summaries.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for cfg in "0 100" "1 340"; do
  set -- $cfg
  TTSHIP_LIB=$PWD/tools/var/lib_trace.so TTS_PTRACE=gpurun_out/pt$1.bin TTS_PTRACE_LAUNCH=$1 TTS_PTRACE_T0=$2 timeout -k 10 150 python bench.py --steps 1 --warmup 1 \
    --no-cpu-baseline --f32-steps 0 --r1-steps 0 > /dev/null 2>gpurun_out/pt$1.err || exit 1
  echo "== launch $1 from step $2"; python tools/ptrace.py gpurun_out/pt$1.bin | head -12
done
