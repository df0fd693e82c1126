#!/bin/bash
# Round 5, final: full GPU tests, smoke, bench line, kernel-trace stats, the calibrated PMC passes
# over the bench (tools/pmc_bench.sh) and the decoder's HBM traffic record (tools/pmc_persist.sh).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
exec 3>&1
step() { local name=$1; shift; echo "== $name $(date +%T)" >&3; "$@"; local rc=$?; echo "== $name rc=$rc" >&3; return $rc; }
step tests timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/h_tests.log 2>&1 || { tail -40 gpurun_out/h_tests.log; exit 1; }
tail -2 gpurun_out/h_tests.log; grep -E "C4 batch 64" gpurun_out/h_tests.log
step smoke timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/h_smoke.log 2>&1 || exit 1
step bench timeout -k 10 400 python3 bench.py > gpurun_out/h_bench.json 2> gpurun_out/h_bench.err || exit 1
cut -c1-400 gpurun_out/h_bench.json
TTSHIP_LIB=$PWD/tools/var/lib_trace.so TTS_PTRACE=gpurun_out/h_pt.bin timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > /dev/null 2>gpurun_out/h_pt.err && python3 tools/ptrace.py gpurun_out/h_pt.bin > gpurun_out/h_ptrace.txt; head -12 gpurun_out/h_ptrace.txt
rm -rf gpurun_out/h_prof
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/h_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --r1-steps 0 --f32-steps 0 > gpurun_out/h_prof.log 2>&1 || exit 1
step pmc ./tools/pmc_bench.sh || exit 1
grep -E "persist_decoder|resblock|resstack|conv_x3|lstm_persist|out_pqmf" gpurun_out/bench_pmc.txt | cut -c1-330
step persist_pmc ./tools/pmc_persist.sh
cat gpurun_out/persist_pmc.json
