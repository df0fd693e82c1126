"""FETCH_SIZE / WRITE_SIZE per stream_bench dispatch against its known byte counts.

  pmc_stream_cal.py FETCH_DIR WRITE_DIR ITERS OUT.json

Algorithmic bytes per dispatch (tools/stream_bench.hip): loads 256 workgroups x 192 KB x ITERS
(modes 0, 1, 3, 4, 5, 6; mode 2 none); stores 256 x 48 x 16 B x ITERS (modes 0, 1, 3, 5, 6).
Counters are in KiB. Reported per mode: counter bytes / algorithmic bytes (raw, no doubling).
"""
import csv
import glob
import json
import os
import re
import sys

BLOCK = 192 * 1024
WG = 256


def per_mode(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            m = re.search(r"stream_kernel<(\d+)>", row.get("Kernel_Name", ""))
            if m and row.get("Counter_Name") == counter:
                vals.setdefault(int(m.group(1)), []).append(float(row["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    fd, wd, iters, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    fetch, write = per_mode(fd, "FETCH_SIZE"), per_mode(wd, "WRITE_SIZE")
    res = {"iters": iters, "load_bytes_per_dispatch": WG * BLOCK * iters,
           "store_bytes_per_dispatch": WG * 48 * 16 * iters, "modes": {}}
    for m in sorted(set(fetch) | set(write)):
        ld = 0 if m == 2 else WG * BLOCK * iters
        st = WG * 48 * 16 * iters if m in (0, 1, 3, 5, 6, 7, 8, 9) else 0
        e = {"fetch_bytes": fetch.get(m), "write_bytes": write.get(m)}
        if ld and fetch.get(m) is not None:
            e["fetch_over_load_bytes"] = round(fetch[m] / ld, 5)
            e["fetch_over_one_block_per_xcd"] = round(fetch[m] / (8 * BLOCK * iters), 4)
        if st and write.get(m) is not None:
            e["write_over_store_bytes"] = round(write[m] / st, 4)
        res["modes"][m] = e
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
