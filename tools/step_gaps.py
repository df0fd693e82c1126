"""Timeline of bench steps in a rocprofv3 kernel trace.

  python tools/step_gaps.py gpurun_out/prof/run_kernel_trace.csv [--all]
      the last headline step: per-kernel start, gap to the previous kernel's end and duration,
      then span vs busy time, and the idle time between the previous step's last kernel
      (out_pqmf) and this step's first (taco_setup)
  python tools/step_gaps.py <trace.csv> --steps
      one line per step (taco_setup to the next taco_setup): span, kernel-busy time and the idle
      time inside it, for every step of the run (bench.py's passes in order: warmup, pipelined
      warmup, the timed pipelined loop, the blocking and two-call loops, the stage split, ...)
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))

if "--steps" in sys.argv:
    setups = [i for i, r in enumerate(rows) if "taco_setup_kernel" in r["Kernel_Name"]]
    for n, (a, b) in enumerate(zip(setups, setups[1:] + [len(rows)])):
        s0 = int(rows[a]["Start_Timestamp"])
        end = s0
        busy = 0
        for r in rows[a:b]:  # union of the kernels' intervals
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if e > end:
                busy += e - max(s, end)
                end = e
        nxt = int(rows[b]["Start_Timestamp"]) if b < len(rows) else end
        print(f"step {n:2d}: span to the next step {(nxt - s0) / 1e3:9.1f} us, busy {busy / 1e3:9.1f} us, "
              f"idle {(nxt - s0 - busy) / 1e3:7.1f} us")
    sys.exit(0)

idx = [i for i, r in enumerate(rows) if "persist_decoder_kernel<2, 8>" in r["Kernel_Name"]]
i0 = idx[-1]
j = i0
while "taco_setup_kernel" not in rows[j]["Kernel_Name"]:
    j -= 1
k = i0
while k + 1 < len(rows) and "out_pqmf" not in rows[k]["Kernel_Name"]:
    k += 1
p = j - 1
while p > 0 and "out_pqmf" not in rows[p]["Kernel_Name"]:
    p -= 1
t0 = int(rows[j]["Start_Timestamp"])
prev = t0
busy = 0
show = "--all" in sys.argv
for r in rows[j:k + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    if show or s - prev > 2000 or e - s > 100000:
        print(f"{(s - t0) / 1e3:9.1f} gap={(s - prev) / 1e3:7.1f} dur={(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:70]}")
    prev = max(prev, e)
print(f"span {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle inside the step {(prev - t0 - busy) / 1e3:.1f} us")
if p > 0:
    print(f"previous step's out_pqmf end -> this step's taco_setup start: "
          f"{(t0 - int(rows[p]['End_Timestamp'])) / 1e3:.1f} us")
