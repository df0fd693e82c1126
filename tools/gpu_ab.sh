#!/bin/bash
# Same-box A/B of tools/ab/lib_<name>.so variants against the in-tree library on the C2 bench,
# after the decoder / encoder GPU tests of the in-tree library. Usage: tools/gpu_ab.sh <rounds> <name>...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rounds=$1; shift
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "${TESTK:-tacotron2 or decoder or encoder or bilstm or bench_workload or synthesizer}" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
bl() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['decoder_step_us'], d['tacotron2_ms'], d['vocoder_ms'], d['roofline']['launches'])" $1; }
for i in $(seq 1 $rounds); do
  for v in "$@" new; do
    lib=$PWD/tts_amd/libttship.so; [ $v != new ] && lib=$PWD/tools/ab/lib_$v.so
    TTSHIP_LIB=$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
    echo "$v run $i: $(bl gpurun_out/ab_$v.json)"
  done
done
if [ -f tools/var/lib_trace.so ]; then
  TTSHIP_LIB=$PWD/tools/var/lib_trace.so TTS_PTRACE=gpurun_out/ab_pt.bin timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > /dev/null 2>gpurun_out/ab_pt.err && python3 tools/ptrace.py gpurun_out/ab_pt.bin > gpurun_out/ab_ptrace.txt && head -14 gpurun_out/ab_ptrace.txt
fi
