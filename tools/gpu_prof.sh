#!/bin/bash
# kernel-trace profile of a short bench run -> gpurun_out/prof (the tool segfaults at process exit
# after writing its outputs; that is expected and the last step here)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
ls gpurun_out/prof/run_kernel_stats.csv > /dev/null
