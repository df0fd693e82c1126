#!/bin/bash
# Vocoder-stream A/B (profiles/r06/v27_voc_stream.txt): vocoder GPU tests, overlap check, bench
# with TTS_VOC_STREAM=0 / 1 alternating. Run from the repo root under gpurun.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 200 --timeout-method thread -k "concurrent or fused or mbmelgan or pqmf or synthesizer" > gpurun_out/o1_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/o1_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/o1_tests.log
timeout -k 10 200 python -u tools/ovl_debug2.py 10 > gpurun_out/o1_dbg.log 2>&1 || { echo DBG_FAIL; tail -20 gpurun_out/o1_dbg.log; exit 1; }
grep -c "nan 0, differ 0" gpurun_out/o1_dbg.log; grep -v "nan 0, differ 0" gpurun_out/o1_dbg.log | tail -5
for i in 1 2; do
  for v in 0 1; do
    TTS_VOC_STREAM=$v timeout -k 10 200 python bench.py --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/o1_b$v$i.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/o1_b$v$i.log; exit 1; }
    echo "VOC_STREAM=$v: $(tail -1 gpurun_out/o1_b$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["sync_call_ms_per_step"], d["two_call_ms_per_step"], d["host_ms_per_step"])')"
  done
done
