#!/bin/bash
# PMC passes over one short bench.py run (every kernel of the C2 batch): one rocprofv3 run per
# counter group, each under its own time limit; per-kernel-class summary (tools/pmc_kernels.py:
# wave-cycle split, MfmaUtil (MFMA_BUSY over GRBM_GUI_ACTIVE x SIMDs, calibrated by tools/mfma_cal.sh),
# issued MFMA counts, LDS conflicts, HBM bytes with FETCH_SIZE x2) in gpurun_out/bench_pmc.txt.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0"
run() {
  local tag=$1; shift
  rm -rf gpurun_out/bpmc_$tag
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/bpmc_$tag -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/bpmc_$tag.log 2>&1
}
run 1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE &&
run 2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES &&
run 3 FETCH_SIZE &&
run 4 WRITE_SIZE &&
run 5 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAVES
rc=$?
python3 tools/pmc_kernels.py gpurun_out/bpmc_1 gpurun_out/bpmc_2 gpurun_out/bpmc_3 gpurun_out/bpmc_4 gpurun_out/bpmc_5 > gpurun_out/bench_pmc.txt 2>&1
exit $rc
