#!/bin/bash
# PWGAN residual-block kernels: persistent weight-resident (default) vs the per-tile ring kernel
# (TTS_PWGAN_TILE=1): parity tests under both, bit-identity of a full LJ-batch call, timings
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/pw_ab.txt
: > $out
for v in 0 1; do
  echo "== TTS_PWGAN_TILE=$v" >> $out
  TTS_PWGAN_TILE=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "pwgan or c4_glow" >> $out 2>&1 || { cat $out; exit 1; }
done
for v in 0 1; do
  echo "== TTS_PWGAN_TILE=$v" >> $out
  TTS_PWGAN_TILE=$v timeout -k 10 200 python tools/pwgan_bench.py --steps 3 --dump gpurun_out/pw_$v.npy >> $out 2>&1 || { cat $out; exit 1; }
done
python -c "import numpy as np; a=np.load('gpurun_out/pw_0.npy'); b=np.load('gpurun_out/pw_1.npy'); print('bit-identical', np.array_equal(a,b), float(np.abs(a-b).max()))" >> $out 2>&1
rm -f gpurun_out/pw_*.npy
cat $out
