#!/bin/bash
# decoder GPU tests, then the process-to-process spread with the calibrated barrier blocks
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "tacotron2 or decoder or encoder or bilstm or bench_workload or synthesizer" > gpurun_out/p_tests.log 2>&1 || { tail -30 gpurun_out/p_tests.log; exit 1; }
tail -1 gpurun_out/p_tests.log
bash tools/gpu_var.sh 6 TTS_DIAG_XCC=1 2>&1 | grep -v "launch 1\|addresses"
bash tools/gpu_var.sh 3 TTS_BAR_CALIBRATE=0 2>&1 | grep "^run"
