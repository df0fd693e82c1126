"""Per-launch HBM bytes of the decoder K4 kernel from two rocprofv3 --pmc passes.

K4 is the <1,4,MT> skinny kernel launched with 256 workgroups of 256 threads (grid 65536
threads); the projection launch uses the same instantiation with 1 + 5r + 256 workgroups, so the
grid size tells them apart. FETCH_SIZE is doubled (gfx950 tallies 128-B requests at 64 B,
MI355X_MICROARCH.md §HBM); both counters are in KiB.
"""
import csv
import glob
import json
import os
import sys


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = []
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            grid = int(row.get("Grid_Size", "0") or 0)
            if "skinny_kernel<1, 4," in name and grid == 256 * 256 and row.get("Counter_Name") == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit("no K4 dispatches found")
    f_kb = sum(fetch) / len(fetch)
    w_kb = sum(write) / len(write)
    out = {
        "kernel": "decoder K4 skinny_kernel<1,4,MT> (256 x 256 grid)",
        "dispatches": {"fetch": len(fetch), "write": len(write)},
        "fetch_size_kib_raw": f_kb,
        "write_size_kib": w_kb,
        "hbm_bytes_per_launch": int(2 * f_kb * 1024 + w_kb * 1024),
        "correction": "FETCH_SIZE x2 (gfx950 half-count of 16-B/lane reads); Infinity-Cache hits are counted",
    }
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
