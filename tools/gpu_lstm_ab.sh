#!/bin/bash
# Same-box A/B of the BiLSTM kernel time (rocprofv3 kernel-trace stats over a short bench run) for
# tools/var/lib_<v>.so variants against the in-tree library; then the barrier microbenchmark.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in "$@" new; do
    lib=$PWD/tts_amd/libttship.so; [ $v != new ] && lib=$PWD/tools/var/lib_$v.so
    rm -rf gpurun_out/l_prof
    TTSHIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/l_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/l_prof.log 2>&1 || exit 1
    f=$(find gpurun_out/l_prof -name "*kernel_stats.csv" | head -1)
    echo "$v run $i: $(grep -E 'lstm_persist|persist_decoder_kernel<2' $f | awk -F'",' '{print $2}' | cut -d, -f1,3 | tr '\n' ' ')"
  done
done
timeout -k 10 90 tools/bar_bench 4000
