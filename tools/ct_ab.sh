#!/bin/bash
# fused ConvTranspose + C = 48 stack (TTS_CT_FUSE) A/B: vocoder parity tests, bit-identity of the
# C2 batch's waveforms between the two modes, kernel times under rocprofv3
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/ct_ab.txt
: > $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "mbmelgan or melgan or c2 or synthesizer_mean_var" >> $out 2>&1 || { cat $out; exit 1; }
TTS_CT_FUSE=0 timeout -k 10 200 python tools/voc_dump.py gpurun_out/w0.npy --bench >> $out 2>&1 &&
TTS_CT_FUSE=1 timeout -k 10 200 python tools/voc_dump.py gpurun_out/w1.npy --bench >> $out 2>&1 &&
python -c "import numpy as np; a=np.load('gpurun_out/w0.npy'); b=np.load('gpurun_out/w1.npy'); print('bit-identical', np.array_equal(a,b), 'max diff', float(np.abs(a-b).max()))" >> $out 2>&1 || { cat $out; exit 1; }
rm -f gpurun_out/w0.npy gpurun_out/w1.npy
for f in 0 1 0 1; do
  rm -rf gpurun_out/ctp
  TTS_CT_FUSE=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ctp -o run --output-format csv -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/ctp.log 2>&1 || { cat $out; exit 1; }
  echo "== TTS_CT_FUSE=$f" >> $out
  grep -h -E "resstack_x3|conv_x3_kernel<3, 4, 2, 2" $(find gpurun_out/ctp -name "*kernel_stats.csv") | cut -c1-160 >> $out
done
cat $out
