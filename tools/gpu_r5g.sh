#!/bin/bash
# GE2E pipeline with the pre-split h hand-off: GE2E / C5 / encoder GPU tests, then C5 bench against
# tools/var/lib_ge2eold.so (fp32 hand-off), same box
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "ge2e or c5 or speaker or encoder or bilstm" > gpurun_out/g_tests.log 2>&1 || { tail -30 gpurun_out/g_tests.log; exit 1; }
tail -1 gpurun_out/g_tests.log
for i in 1 2 3; do
  for v in ge2eold new; do
    lib=$PWD/tts_amd/libttship.so; [ $v != new ] && lib=$PWD/tools/var/lib_$v.so
    TTSHIP_LIB=$lib timeout -k 10 200 python3 tools/c5_bench.py --steps 10 --warmup 2 > gpurun_out/g_ab_$v.json 2>gpurun_out/g_ab.err || exit 1
    echo "$v run $i: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['ge2e_ms'], d['value'])" gpurun_out/g_ab_$v.json)"
  done
done
