#!/bin/bash
# Bottleneck probes of the split-f16 ResidualStack block kernel (resblock_x3.hip RB_NO_* builds of
# tools/rbx3_bench.hip, profiling mode per stage): which resource the C2 stages' time follows.
#   build (container): tools/rb_probe.sh build ; run (GPU box): tools/rb_probe.sh run
set -o pipefail
cd "$(dirname "$0")/.."
V="base:- nowload:-DRB_NO_WLOAD nolds:-DRB_NO_LDS nomfma:-DRB_NO_MFMA noxload:-DRB_NO_XLOAD"
if [ "$1" = build ]; then
  mkdir -p tools/ab
  for v in $V; do
    n=${v%%:*}; f=${v#*:}; [ "$f" = - ] && f=
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include $f tools/rbx3_bench.hip -o tools/ab/rbx3_$n &
  done
  wait
  ls -la tools/ab/rbx3_*
  exit 0
fi
mkdir -p gpurun_out
for v in $V; do
  n=${v%%:*}
  for C in 192 96 48; do
    timeout -k 5 60 rocprofv3 --kernel-trace --stats -d gpurun_out/rbp_${n}_$C -o run --output-format csv -- tools/ab/rbx3_$n $C > /dev/null 2>&1 || exit 1
    us=$(python3 -c "
import csv,glob,sys
f=glob.glob('gpurun_out/rbp_${n}_$C/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'resblock_x3_kernel' in r['Name']: print(round(float(r['AverageNs'])/1e3,1))")
    echo "probe $n C=$C: $us us per launch"
  done
done
