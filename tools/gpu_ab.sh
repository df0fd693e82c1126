#!/bin/bash
# GPU tests, then an A/B of the bench on the same box: ENV_A vs ENV_B (environment assignments),
# alternating, each run under its own time limit; then the decoder phase trace of the B setting.
#   bash tools/gpu_ab.sh "TTS_ALIGN_IN_P4=1" ""
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
A=$1; B=$2
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
tail -3 gpurun_out/t.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for tag in A B; do
    envs=$([ $tag = A ] && echo "$A" || echo "$B")
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --f32-steps 0 --r1-steps 0 --steps 10 > gpurun_out/ab_${tag}$i.json 2>gpurun_out/ab_${tag}$i.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${tag}$i.json')); print('$tag$i', d['ms_per_step'], d['decoder_step_us'], d['tacotron2_ms'], d['vocoder_ms'], d['roofline']['launches'])"
  done
done
env $B TTS_PTRACE=gpurun_out/pt.bin timeout -k 10 150 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --f32-steps 0 --r1-steps 0 > /dev/null 2>gpurun_out/pt.err &&
python tools/ptrace.py gpurun_out/pt.bin
