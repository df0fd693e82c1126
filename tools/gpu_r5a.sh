#!/bin/bash
# Round 5, call A: GPU tests on the LDS-layout decoder, same-box A/B against the old layout
# (tools/var/lib_old.so), decoder LDS-conflict PMC for both, phase trace, MFMA counter calibration.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
exec 3>&1
step() { local name=$1; shift; echo "== $name $(date +%T)" >&3; "$@"; local rc=$?; echo "== $name rc=$rc" >&3; return $rc; }
bl() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['decoder_step_us'], d['tacotron2_ms'], d['vocoder_ms'], d['roofline']['launches'])" $1; }
step tests timeout -k 10 400 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/a_tests.log 2>&1 || { tail -30 gpurun_out/a_tests.log; exit 1; }
tail -2 gpurun_out/a_tests.log
for i in 1 2 3; do
  for v in old new; do
    lib=$PWD/tts_amd/libttship.so; [ $v = old ] && lib=$PWD/tools/var/lib_old.so
    TTSHIP_LIB=$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/a_ab_$v.json 2>/dev/null || exit 1
    echo "$v run $i: $(bl gpurun_out/a_ab_$v.json)"
  done
done
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0"
for v in old new; do
  lib=$PWD/tts_amd/libttship.so; [ $v = old ] && lib=$PWD/tools/var/lib_old.so
  rm -rf gpurun_out/a_pmc_$v
  TTSHIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES \
    --kernel-trace -d gpurun_out/a_pmc_$v -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/a_pmc_$v.log 2>&1 || exit 1
  echo "PMC $v:"; python3 tools/pmc_kernels.py gpurun_out/a_pmc_$v | grep persist_decoder
done
TTSHIP_LIB=$PWD/tools/var/lib_trace.so TTS_PTRACE=gpurun_out/a_pt.bin timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > /dev/null 2>gpurun_out/a_pt.err && python3 tools/ptrace.py gpurun_out/a_pt.bin > gpurun_out/a_ptrace.txt; cat gpurun_out/a_ptrace.txt | head -8
step cal ./tools/mfma_cal.sh; cat gpurun_out/mfma_cal.txt
