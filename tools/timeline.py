"""Print the GPU timeline of a rocprofv3 kernel trace (and memory-copy trace, if given): every
kernel / copy in start order with its duration and the idle gap before it, for the last bench step
(the span between the last two persistent-decoder launches' predecessors is found by name).

    python tools/timeline.py <run_kernel_trace.csv> [<run_memory_copy_trace.csv>] [--all]
"""
import csv
import sys


def load(path, kind):
    out = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Operation") or kind
        if kind == "copy":
            name = "COPY " + (r.get("Operation") or "") + f" {r.get('Source_Agent_Id', '')}->{r.get('Destination_Agent_Id', '')}"
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    return out


def main(argv):
    show_all = "--all" in argv
    paths = [a for a in argv if not a.startswith("--")]
    ev = load(paths[0], "kernel")
    if len(paths) > 1:
        ev += load(paths[1], "copy")
    ev.sort()
    # one bench step starts at the embedding gather; print the last complete step
    starts = [i for i, e in enumerate(ev) if "embed_gather" in e[2]]
    if not show_all and len(starts) >= 2:
        ev = ev[starts[-2]:starts[-1]]
    elif not show_all and starts:
        ev = ev[starts[-1]:]
    t0 = ev[0][0]
    prev_end = t0
    busy = 0
    for s, e, n in ev:
        gap = s - prev_end
        busy += e - s
        print(f"{(s - t0) / 1e3:10.1f} us  +gap {gap / 1e3:8.1f}  dur {(e - s) / 1e3:9.1f}  {n[:100]}")
        prev_end = max(prev_end, e)
    span = prev_end - t0
    print(f"span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us, events {len(ev)}")


if __name__ == "__main__":
    main(sys.argv[1:])
