#!/bin/bash
# BiLSTM layouts A/B: for each (row groups, tiles per workgroup) the encoder parity tests, then the
# persistent LSTM kernel's average duration over a short bench run under rocprofv3
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/lstm_ab.txt
: > $out
for cfg in "2 1" "4 2" "2 2" "1 2" "2 1"; do
  set -- $cfg
  echo "== RG=$1 TPW=$2" | tee -a $out
  TTS_LSTM_RG=$1 TTS_LSTM_TPW=$2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "encoder_matches or encoder_row_groups or ge2e" >> $out 2>&1 || exit 1
  rm -rf gpurun_out/lab
  TTS_LSTM_RG=$1 TTS_LSTM_TPW=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/lab -o run --output-format csv -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/lab.log 2>&1 || exit 1
  grep -h "lstm_persist" $(find gpurun_out/lab -name "*kernel_stats.csv") | cut -c1-200 >> $out
done
cat $out
