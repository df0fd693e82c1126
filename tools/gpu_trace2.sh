#!/bin/bash
# phase traces of both persistent launches (MT = 2, then MT = 1) of the C2 bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for li in 0 1; do
  t0=40; [ $li = 1 ] && t0=340
  TTSHIP_LIB=$PWD/tools/var/lib_trace.so TTS_PTRACE=gpurun_out/t_pt$li.bin TTS_PTRACE_LAUNCH=$li TTS_PTRACE_T0=$t0 timeout -k 10 120 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > /dev/null 2>gpurun_out/t_pt$li.err || exit 1
  python3 tools/ptrace.py gpurun_out/t_pt$li.bin > gpurun_out/t_ptrace$li.txt && echo "== launch $li" && head -16 gpurun_out/t_ptrace$li.txt
done
