#!/bin/bash
# ParallelWaveGAN throughput + kernel-trace profile -> gpurun_out/pwgan.json, gpurun_out/pwprof
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/pwgan_bench.py --cpu-frames 20 > gpurun_out/pwgan.json 2> gpurun_out/pwgan.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pwprof -o run --output-format csv -- python3 tools/pwgan_bench.py --steps 2 --warmup 1 > gpurun_out/pwprof.log 2>&1
ls gpurun_out/pwprof/run_kernel_stats.csv > /dev/null
