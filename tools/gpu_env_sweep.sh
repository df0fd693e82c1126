#!/bin/bash
# Same-box sweep of environment switches on the C2 bench: tools/gpu_env_sweep.sh <rounds> "A=1" "B=2 C=3" ...
# Each round runs the default, then every configuration; prints ms_per_step, decoder step, tacotron2, vocoder.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rounds=$1; shift
bl() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['decoder_step_us'], d['tacotron2_ms'], d['vocoder_ms'])" $1; }
for i in $(seq 1 $rounds); do
  timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/sw.json 2>/dev/null || exit 1
  echo "default run $i: $(bl gpurun_out/sw.json)"
  for c in "$@"; do
    env $c timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/sw.json 2>/dev/null || exit 1
    echo "[$c] run $i: $(bl gpurun_out/sw.json)"
  done
done
