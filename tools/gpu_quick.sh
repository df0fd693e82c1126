set -o pipefail
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "tacotron2 or smoke or encoder or synth" > gpurun_out/t.log 2>&1; rc=$?; tail -5 gpurun_out/t.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2>gpurun_out/b.err && tail -1 gpurun_out/b.json | cut -c1-600
TTSHIP_LIB=$PWD/tools/var/lib_trace.so TTS_PTRACE=gpurun_out/pt.bin timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2>>gpurun_out/b.err && python tools/ptrace.py gpurun_out/pt.bin
