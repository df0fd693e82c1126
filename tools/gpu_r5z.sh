#!/bin/bash
# Round 5, last tree: full GPU tests, smoke, bench line, kernel-trace stats
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/z_tests.log 2>&1 || { tail -40 gpurun_out/z_tests.log; exit 1; }
tail -1 gpurun_out/z_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/z_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/z_bench.json 2> gpurun_out/z_bench.err || exit 1
cut -c1-300 gpurun_out/z_bench.json
rm -rf gpurun_out/z_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/z_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/z_prof.log 2>&1 || exit 1
