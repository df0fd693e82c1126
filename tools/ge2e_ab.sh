#!/bin/bash
# GE2E layer pipeline: parity tests, then C5 with TTS_GE2E_PIPE=0 (per-layer launches) / 1, same box
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "ge2e or c5 or speaker" > gpurun_out/ge2e_t.log 2>&1 || { tail -30 gpurun_out/ge2e_t.log; exit 1; }
tail -3 gpurun_out/ge2e_t.log
for i in 1 2; do
  for v in 0 1; do
    TTS_GE2E_PIPE=$v timeout -k 10 200 python3 tools/c5_bench.py --steps 10 --warmup 2 > gpurun_out/ge2e_ab_$v.$i.json 2>gpurun_out/ge2e_ab.err || exit 1
    echo "pipe=$v run=$i $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['ge2e_ms'], d['value'])" gpurun_out/ge2e_ab_$v.$i.json)"
  done
done
