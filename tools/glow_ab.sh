#!/bin/bash
# Glow-TTS parity tests, then batch-64 timings (tools/glow_bench.py) on this box
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "glow or c4" > gpurun_out/glow_t.log 2>&1 || { tail -30 gpurun_out/glow_t.log; exit 1; }
tail -1 gpurun_out/glow_t.log
for i in 1 2; do
  timeout -k 10 200 python3 tools/glow_bench.py --steps 10 --warmup 2 --batch 64 > gpurun_out/glow_ab.$i.json 2> gpurun_out/glow_ab.err || exit 1
  cat gpurun_out/glow_ab.$i.json
done
