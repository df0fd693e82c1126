#!/bin/bash
# GPU side of tools/build_variants.sh: bench + phase trace for each named variant.
#   tools/var_run.sh h0 h1 ...   -> gpurun_out/var_<name>.{json,txt}
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for name in "$@"; do
  TTSHIP_LIB=tools/var/lib_$name.so timeout -k 10 120 python bench.py --steps 4 --warmup 1 --no-cpu-baseline \
    > gpurun_out/var_$name.json 2> gpurun_out/var_$name.err || { echo "$name bench failed"; tail -5 gpurun_out/var_$name.err; exit 1; }
  TTSHIP_LIB=tools/var/lib_$name.so TTS_PTRACE=gpurun_out/pt_$name.bin timeout -k 10 120 python bench.py --steps 1 --warmup 0 \
    --no-cpu-baseline > /dev/null 2>> gpurun_out/var_$name.err || { echo "$name trace failed"; exit 1; }
  python tools/ptrace.py gpurun_out/pt_$name.bin > gpurun_out/var_$name.txt
  python - "$name" <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads(open(f"gpurun_out/var_{n}.json").read().strip().splitlines()[-1])
print(n, "value", d["value"], "ms", d["ms_per_step"], "dec_us", d["decoder_step_us"], "taco_ms", d["tacotron2_ms"], "voc_ms", d["vocoder_ms"])
PY
  head -7 gpurun_out/var_$name.txt
done
