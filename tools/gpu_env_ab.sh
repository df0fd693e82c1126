#!/bin/bash
# Same-box A/B of an environment switch on the C2 bench: tools/gpu_env_ab.sh <rounds> VAR=value ...
# (each round runs the bench with the assignments, then without them)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rounds=$1; shift
bl() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['decoder_step_us'], d['tacotron2_ms'], d['vocoder_ms'])" $1; }
for i in $(seq 1 $rounds); do
  env "$@" timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/env_a.json 2>/dev/null || exit 1
  echo "env run $i: $(bl gpurun_out/env_a.json)"
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/env_b.json 2>/dev/null || exit 1
  echo "default run $i: $(bl gpurun_out/env_b.json)"
done
