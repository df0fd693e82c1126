#!/bin/bash
# same-box A/B of two builds of the library: tts_amd/libttship_ab.so (A, the previous code) against
# tts_amd/libttship.so (B); CMD is the benchmark command (default: the batch-64 PWGAN call, with a
# waveform dump compared for bit identity)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do
  for v in A B; do
    lib=tts_amd/libttship.so; [ $v = A ] && lib=tts_amd/libttship_ab.so
    TTSHIP_LIB=$PWD/$lib timeout -k 10 200 python3 tools/pwgan_bench.py --steps 3 --batch 64 --dump gpurun_out/lib_ab_$v.npy > gpurun_out/lib_ab_$v.$i.json 2>gpurun_out/lib_ab.err || exit 1
    echo "$v run $i: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_call'])" gpurun_out/lib_ab_$v.$i.json)"
  done
done
python3 -c "
import numpy as np
a, b = np.load('gpurun_out/lib_ab_A.npy'), np.load('gpurun_out/lib_ab_B.npy')
print('bit-identical', np.array_equal(a, b))"
rm -f gpurun_out/lib_ab_*.npy
