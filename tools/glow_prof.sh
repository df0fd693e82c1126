#!/bin/bash
# Glow-TTS throughput + kernel-trace profile -> gpurun_out/glow.json, gpurun_out/glowprof
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/glow_bench.py --cpu-utts 4 > gpurun_out/glow.json 2> gpurun_out/glow.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/glowprof -o run --output-format csv -- python3 tools/glow_bench.py --steps 3 --warmup 1 > gpurun_out/glowprof.log 2>&1
ls gpurun_out/glowprof/run_kernel_stats.csv > /dev/null
