"""Per-launch HBM bytes of one decoder kernel from two rocprofv3 --pmc passes.

  pmc_summary.py FETCH_DIR WRITE_DIR OUT.json [KERNEL_SUBSTRING]

Default kernel: the graph path's K4 (<1,4,MT> skinny kernel, 256 x 256 grid; the projection
launch uses the same instantiation with a different grid). With a substring (e.g.
"persist_decoder_kernel<2>") every dispatch whose name contains it is averaged. FETCH_SIZE is
doubled (gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md §HBM); both counters are in
KiB; Infinity-Cache (MALL) hits are counted.
"""
import csv
import glob
import json
import os
import sys


def load(d, counter, sub=None):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = []
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            grid = int(row.get("Grid_Size", "0") or 0)
            hit = (sub in name) if sub else ("skinny_kernel<1, 4," in name and grid == 256 * 256)
            if hit and row.get("Counter_Name") == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    sub = sys.argv[4] if len(sys.argv) > 4 else None
    fetch = load(sys.argv[1], "FETCH_SIZE", sub)
    write = load(sys.argv[2], "WRITE_SIZE", sub)
    if not fetch or not write:
        raise SystemExit("no matching dispatches found")
    f_kb = sum(fetch) / len(fetch)
    w_kb = sum(write) / len(write)
    out = {
        "kernel": sub or "decoder K4 skinny_kernel<1,4,MT> (256 x 256 grid)",
        "dispatches": {"fetch": len(fetch), "write": len(write)},
        "fetch_size_kib_raw": f_kb,
        "write_size_kib": w_kb,
        "hbm_bytes_per_launch": int(2 * f_kb * 1024 + w_kb * 1024),
        "correction": "FETCH_SIZE x2 (gfx950 half-count of 16-B/lane reads); Infinity-Cache hits are counted",
    }
    info = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tts_amd", "build_info.json")
    if os.path.exists(info):  # which build of the sources the counted library was
        b = json.load(open(info))
        out["library_sha256"], out["sources_sha256"] = b.get("library_sha256"), b.get("sources_sha256")
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
