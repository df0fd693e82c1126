#!/bin/bash
# Calibrates FETCH_SIZE / WRITE_SIZE for the decoder's hand-off access pattern:
# tools/stream_bench moves a KNOWN byte count (every one of 256 workgroups reads the same 192 KB
# block with 16-byte sc1 loads per iteration, 200 iterations per dispatch; mode 0 rewrites the
# block between passes as the decoder's producers do, mode 4 does not, mode 5 uses plain loads),
# so counter bytes / algorithmic bytes is the factor for exactly this pattern. One counter per pass.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_sf gpurun_out/pmc_sw
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_sf -o run --output-format csv -- tools/stream_bench 200 > gpurun_out/pmc_sf.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_sw -o run --output-format csv -- tools/stream_bench 200 > gpurun_out/pmc_sw.log 2>&1 &&
python3 tools/pmc_stream_cal.py gpurun_out/pmc_sf gpurun_out/pmc_sw 200 gpurun_out/stream_pmc_cal.json
