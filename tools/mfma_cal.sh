#!/bin/bash
# MFMA counter calibration (tools/mfma_cal.hip): the same SQ counter pass as tools/pmc_bench.sh
# plus the MFMA instruction counters and GRBM_GUI_ACTIVE, over kernels of known MFMA count and duty.
# Output: gpurun_out/mfma_cal.txt (tools/pmc_kernels.py summary of both passes + the tool's own lines).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
BIN=./tools/mfma_cal
rm -rf gpurun_out/cal_1 gpurun_out/cal_2
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-trace -d gpurun_out/cal_1 -o run --output-format csv -- $BIN > gpurun_out/cal_1.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \
  --kernel-trace -d gpurun_out/cal_2 -o run --output-format csv -- $BIN > gpurun_out/cal_2.log 2>&1
rc=$?
{ grep '^{' gpurun_out/cal_1.log; python3 tools/pmc_kernels.py gpurun_out/cal_1 gpurun_out/cal_2; } > gpurun_out/mfma_cal.txt 2>&1
exit $rc
