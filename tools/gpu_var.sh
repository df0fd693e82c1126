#!/bin/bash
# Process-to-process spread of the decoder step on one box: the C2 bench run N times, each in a
# fresh process (tools/gpu_var.sh N [env assignments for every run])
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
n=$1; shift
for i in $(seq 1 $n); do
  env "$@" timeout -k 10 200 python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/var_$i.json 2>gpurun_out/var_$i.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('run', sys.argv[2], d['ms_per_step'], d['decoder_step_us'], d['vocoder_ms'], d['roofline']['launches'])" gpurun_out/var_$i.json $i
  grep TTS_DIAG gpurun_out/var_$i.err | tail -3 || true
done
