#!/bin/bash
# PMC passes over the split-f16 conv kernel at the C2 shapes (tools/cx3_bench prof): one rocprofv3
# run per counter group, each under its own time limit; summaries in gpurun_out/cx3_pmc*.txt.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
BIN=${1:-./tools/cx3_bench}
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/cx3_pmc1 -o run --output-format csv -- $BIN prof > gpurun_out/cx3_pmc1.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU --kernel-trace -d gpurun_out/cx3_pmc2 -o run --output-format csv -- $BIN prof > gpurun_out/cx3_pmc2.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/cx3_pmc3 -o run --output-format csv -- $BIN prof > gpurun_out/cx3_pmc3.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/cx3_pmc4 -o run --output-format csv -- $BIN prof > gpurun_out/cx3_pmc4.log 2>&1
rc=$?
python3 tools/pmc_kernels.py gpurun_out/cx3_pmc1 gpurun_out/cx3_pmc2 gpurun_out/cx3_pmc3 gpurun_out/cx3_pmc4 > gpurun_out/cx3_pmc.txt 2>&1
exit $rc
