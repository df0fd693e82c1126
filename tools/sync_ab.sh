#!/bin/bash
# A/B of the host wait (TTS_SPIN_SYNC=0: blocking hipStreamSynchronize, 1: polled marker event) on one box
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1; do
    TTS_SPIN_SYNC=$v timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sync_ab_$v.$i.json 2> gpurun_out/sync_ab_$v.$i.err || exit 1
    echo "spin=$v run=$i $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'])" gpurun_out/sync_ab_$v.$i.json)"
  done
done
