#!/bin/bash
# HBM traffic of the decoder's K4 launch from PMC counters: FETCH_SIZE and WRITE_SIZE in separate
# passes (they do not fit one TCC pass on gfx950), kernel trace only beside them. The summary
# (tools/pmc_summary.py) doubles FETCH_SIZE (gfx950 reports half the bytes of 16-B-per-lane reads,
# MI355X_MICROARCH.md §HBM) and writes profiles/k4_pmc.json.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --kernel-iters 20 > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --kernel-iters 20 > gpurun_out/pmc_write.log 2>&1 &&
python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/k4_pmc.json  # copy into profiles/ here
