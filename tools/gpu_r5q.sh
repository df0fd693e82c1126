#!/bin/bash
# Round-5 check of the pre-split BiLSTM hand-off: the encoder / decoder / GE2E GPU tests of the
# in-tree library, then the BiLSTM and decoder kernel times (rocprofv3 stats) against
# tools/var/lib_lstmold.so (the same tree with the fp32 BiLSTM hand-off).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "tacotron2 or decoder or encoder or bilstm or ge2e or bench_workload or synthesizer" > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
for i in 1 2; do
  for v in lstmold new; do
    lib=$PWD/tts_amd/libttship.so; [ $v != new ] && lib=$PWD/tools/var/lib_$v.so
    rm -rf gpurun_out/q_prof
    TTSHIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/q_prof.log 2>&1 || exit 1
    f=$(find gpurun_out/q_prof -name "*kernel_stats.csv" | head -1)
    echo "$v run $i: $(grep -E 'lstm_persist|persist_decoder_kernel<2' $f | awk -F'",' '{print $2}' | cut -d, -f1,3 | tr '\n' ' ')"
  done
done
