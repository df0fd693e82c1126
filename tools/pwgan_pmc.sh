#!/bin/bash
# PMC passes over one ParallelWaveGAN call on the LJ batch (tools/pwgan_bench.py): one rocprofv3 run
# per counter group, summarised per kernel by tools/pmc_kernels.py into gpurun_out/pwgan_pmc.txt
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0"
run() {
  local tag=$1; shift
  rm -rf gpurun_out/ppmc_$tag
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/ppmc_$tag -o run --output-format csv -- python3 tools/pwgan_bench.py $ARGS > gpurun_out/ppmc_$tag.log 2>&1
}
run 1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES &&
run 2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES &&
run 3 FETCH_SIZE &&
run 4 WRITE_SIZE
rc=$?
python3 tools/pmc_kernels.py gpurun_out/ppmc_1 gpurun_out/ppmc_2 gpurun_out/ppmc_3 gpurun_out/ppmc_4 > gpurun_out/pwgan_pmc.txt 2>&1
exit $rc
