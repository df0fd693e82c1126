#!/bin/bash
# taco/postnet parity tests, then a kernel-trace profile of a short bench run (gpurun_out/qprof)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/qprof
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "${TESTS:-postnet or tacotron2 or c5}" > gpurun_out/qprof_t.log 2>&1 || { tail -30 gpurun_out/qprof_t.log; exit 1; }
tail -2 gpurun_out/qprof_t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/qprof.log 2>&1
ls gpurun_out/qprof/run_kernel_stats.csv > /dev/null && tail -1 gpurun_out/qprof.log | cut -c1-300
