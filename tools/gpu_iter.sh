#!/bin/bash
# Iteration check: every GPU test, one bench line (no CPU baseline), a kernel-trace profile.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b.json 2>gpurun_out/b.err
rc=$?; tail -1 gpurun_out/b.json | cut -c1-700; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
