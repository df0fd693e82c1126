#!/bin/bash
# PWGAN residual-block kernels: persistent weight-resident with 8 waves (default, TTS_PWGAN_TILE=0)
# or 4 waves (=2), and the per-tile ring kernel (=1): parity tests, timings and bit-identity of a
# full LJ-batch call across the three
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/pw_ab.txt
: > $out
for v in 0 2; do
  echo "== tests TTS_PWGAN_TILE=$v" >> $out
  TTS_PWGAN_TILE=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "pwgan or c4_glow" >> $out 2>&1 || { cat $out; exit 1; }
done
for v in 0 2 1 0; do
  echo "== bench TTS_PWGAN_TILE=$v" >> $out
  TTS_PWGAN_TILE=$v timeout -k 10 200 python tools/pwgan_bench.py --steps 3 --dump gpurun_out/pw_$v.npy >> $out 2>&1 || { cat $out; exit 1; }
done
python -c "
import numpy as np
a, b, c = (np.load(f'gpurun_out/pw_{v}.npy') for v in (0, 2, 1))
print('bit-identical 8-wave == 4-wave', np.array_equal(a, b), '4-wave == per-tile', np.array_equal(b, c))" >> $out 2>&1
rm -f gpurun_out/pw_*.npy
cat $out
