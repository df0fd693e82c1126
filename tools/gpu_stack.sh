#!/bin/bash
# Vocoder-side check of one change: the vocoder GPU tests, a bench A/B (ENV_A vs default,
# alternating) and a kernel-trace profile of the default. Each GPU step has its own time limit.
#   bash tools/gpu_stack.sh "TTS_STACK_FUSE=0"
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
A=$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "mbmelgan or fullband or bench_workload or c5" > gpurun_out/vt.log 2>&1; rc=$?
tail -3 gpurun_out/vt.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for tag in A B; do
    envs=$([ $tag = A ] && echo "$A" || echo "")
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --f32-steps 0 --r1-steps 0 --steps 10 > gpurun_out/ab_${tag}$i.json 2>gpurun_out/ab_${tag}$i.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${tag}$i.json')); print('$tag$i', d['ms_per_step'], d['decoder_step_us'], d['tacotron2_ms'], d['vocoder_ms'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/sprof.log 2>&1 &&
python tools/kstats.py gpurun_out/sprof/run_kernel_stats.csv 25
