#!/bin/bash
# Round 5, call C: full GPU tests, smoke, bench line, same-box A/B against tools/var/lib_<v>.so
# variants, the phase trace and the kernel-trace stats of the bench. Usage: tools/gpu_r5c.sh <variant>...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
exec 3>&1
step() { local name=$1; shift; echo "== $name $(date +%T)" >&3; "$@"; local rc=$?; echo "== $name rc=$rc" >&3; return $rc; }
step tests timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/c_tests.log 2>&1 || { tail -40 gpurun_out/c_tests.log; exit 1; }
tail -2 gpurun_out/c_tests.log
step smoke timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c_smoke.log 2>&1 || exit 1
step bench timeout -k 10 400 python3 bench.py > gpurun_out/c_bench.json 2> gpurun_out/c_bench.err || exit 1
cut -c1-400 gpurun_out/c_bench.json
bl() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['decoder_step_us'], d['tacotron2_ms'], d['vocoder_ms'], d['roofline']['launches'])" $1; }
for i in 1 2 3; do
  for v in "$@" new; do
    lib=$PWD/tts_amd/libttship.so; [ $v != new ] && lib=$PWD/tools/var/lib_$v.so
    TTSHIP_LIB=$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/c_ab_$v.json 2>/dev/null || exit 1
    echo "$v run $i: $(bl gpurun_out/c_ab_$v.json)"
  done
done
TTSHIP_LIB=$PWD/tools/var/lib_trace.so TTS_PTRACE=gpurun_out/c_pt.bin timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > /dev/null 2>gpurun_out/c_pt.err && python3 tools/ptrace.py gpurun_out/c_pt.bin > gpurun_out/c_ptrace.txt; head -12 gpurun_out/c_ptrace.txt
rm -rf gpurun_out/c_prof
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/c_prof.log 2>&1 || exit 1
f=$(find gpurun_out/c_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/c_kernel_stats.csv; head -12 gpurun_out/c_kernel_stats.csv | cut -c1-160
