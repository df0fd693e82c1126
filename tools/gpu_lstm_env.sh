#!/bin/bash
# BiLSTM kernel time (rocprofv3 kernel stats of a short bench run) with and without an environment
# switch, same box: tools/gpu_lstm_env.sh <rounds> VAR=value
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rounds=$1; shift
for i in $(seq 1 $rounds); do
  for v in default env; do
    rm -rf gpurun_out/le_prof
    if [ $v = env ]; then pre="env $*"; else pre=""; fi
    $pre timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/le_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/le_prof.log 2>&1 || exit 1
    f=$(find gpurun_out/le_prof -name "*kernel_stats.csv" | head -1)
    echo "$v run $i: $(python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'lstm_persist' in r['Name'] or 'persist_decoder' in r['Name']: print(r['Name'][:40], round(float(r['AverageNs'])/1000, 1), 'us', end='; ')
" $f)"
  done
done
