#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile. Each GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
exec 3>&1  # step markers go to the script's stdout, not into the per-step logs
step() { local name=$1; shift; echo "== $name" >&3; "$@"; local rc=$?; echo "== $name rc=$rc" >&3; return $rc; }
step tests timeout -k 10 800 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
step smoke timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
step bench timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 &&
step prof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/prof.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log; tail -2 gpurun_out/smoke.log; tail -2 gpurun_out/bench.log
exit $rc
