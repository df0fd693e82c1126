#!/bin/bash
# PMC passes over the split-f16 ResidualStack kernel (tools/rbx3_bench, profiling mode): one
# rocprofv3 run per counter group, each under its own time limit; results in gpurun_out/rbx3_pmc*.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${1:-192}
timeout -k 5 60 rocprofv3 -L > gpurun_out/rocprof_list.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/rbx3_pmc1 -o run --output-format csv -- ./tools/rbx3_bench $C > gpurun_out/rbx3_pmc1.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/rbx3_pmc2 -o run --output-format csv -- ./tools/rbx3_bench $C > gpurun_out/rbx3_pmc2.log 2>&1
rc=$?
grep -o "SQ_[A-Z_0-9]*" gpurun_out/rocprof_list.txt | sort -u > gpurun_out/sq_counters.txt
exit $rc
