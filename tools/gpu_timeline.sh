#!/bin/bash
# kernel + memory-copy trace of a short bench run, then the GPU timeline of its last step
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tl -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/tl.log 2>&1 &&
kt=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1) && mc=$(find gpurun_out/tl -name "*memory_copy_trace.csv" | head -1) &&
python tools/timeline.py "$kt" $mc > gpurun_out/timeline.txt 2>&1
rc=$?
tail -5 gpurun_out/timeline.txt
exit $rc
