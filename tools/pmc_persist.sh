#!/bin/bash
# HBM traffic of the persistent decoder's MT = 2 launch from PMC counters: FETCH_SIZE and WRITE_SIZE
# in separate passes (they do not fit one TCC pass on gfx950), kernel trace only beside them.
# tools/pmc_summary.py doubles FETCH_SIZE (MI355X_MICROARCH.md §HBM) and writes the summary.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --f32-steps 0 --r1-steps 0 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1
ls gpurun_out/pmc_fetch > /dev/null &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --f32-steps 0 --r1-steps 0 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/persist_pmc.json "persist_decoder_kernel<2, 8>"
