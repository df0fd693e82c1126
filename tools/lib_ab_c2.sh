#!/bin/bash
# same-box A/B of tts_amd/libttship_ab.so (A) against tts_amd/libttship.so (B) on the C2 bench
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "tacotron2_matches or decoder_state or encoder" > gpurun_out/abc2_t.log 2>&1 || { tail -20 gpurun_out/abc2_t.log; exit 1; }
tail -1 gpurun_out/abc2_t.log
for i in 1 2 3; do
  for v in A B; do
    lib=tts_amd/libttship.so; [ $v = A ] && lib=tts_amd/libttship_ab.so
    TTSHIP_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/abc2_$v.json 2>/dev/null || exit 1
    echo "$v run $i: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['decoder_step_us'], d['tacotron2_ms'], d['vocoder_ms'])" gpurun_out/abc2_$v.json)"
  done
done
