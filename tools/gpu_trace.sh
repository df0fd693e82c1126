#!/bin/bash
# persistent decoder phase trace (TTS_PTRACE) of one bench step, summarised by tools/ptrace.py
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TTSHIP_LIB=$PWD/tools/var/lib_trace.so TTS_PTRACE=gpurun_out/pt.bin timeout -k 10 150 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --f32-steps 0 --r1-steps 0 > gpurun_out/pt.json 2>gpurun_out/pt.err &&
python tools/ptrace.py gpurun_out/pt.bin > gpurun_out/pt.txt 2>&1
rc=$?
cat gpurun_out/pt.txt
exit $rc
