#!/bin/bash
# GPU tests, one bench line without the CPU baseline, and the persistent decoder phase trace
# (TTS_PTRACE, tools/ptrace.py) of one bench step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --f32-steps 0 > gpurun_out/b.json 2>gpurun_out/b.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/b.json')); print(d['ms_per_step'], d['decoder_step_us'], d['roofline']['launches'])"
TTSHIP_LIB=$PWD/tools/var/lib_trace.so TTS_PTRACE=gpurun_out/pt.bin timeout -k 10 150 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --f32-steps 0 > /dev/null 2>gpurun_out/pt.err && python tools/ptrace.py gpurun_out/pt.bin | head -14
