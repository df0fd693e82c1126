"""Average rocprofv3 --pmc counters per (kernel, grid size) over one or more counter directories
and print one line per dispatch class: wave-cycle split (waiting / issue-stalled / active), MFMA
busy share, LDS and VALU instruction counts per wave, HBM bytes (FETCH_SIZE x2, gfx950).

  pmc_kernels.py DIR [DIR ...]
"""
import collections
import csv
import glob
import os
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            key = (row.get("Kernel_Name", "")[:60], int(row.get("Grid_Size", "0") or 0))
            vals[key][row["Counter_Name"]].append(float(row["Counter_Value"]))

for (name, grid), c in sorted(vals.items()):
    a = {k: sum(v) / len(v) for k, v in c.items()}
    out = [f"{name:60s} grid {grid:9d}"]
    wc = a.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in a:
                out.append(f"{k[3:]} {a[k] / wc:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in a and "SQ_BUSY_CYCLES" in a:
        out.append(f"MFMA_BUSY/BUSY {a['SQ_VALU_MFMA_BUSY_CYCLES'] / (a['SQ_BUSY_CYCLES'] * 4 * 4):.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in a and "GRBM_GUI_ACTIVE" in a and a["GRBM_GUI_ACTIVE"]:
        # MfmaUtil as rocprofiler-sdk defines it (sum of per-SIMD busy cycles over GUI-active cycles x
        # SIMDs); GRBM_GUI_ACTIVE is reported summed over the 8 XCDs, 1024 SIMDs on the chip
        out.append(f"MfmaUtil {a['SQ_VALU_MFMA_BUSY_CYCLES'] / (a['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
    # issued MFMA instructions from the MOPS counters (units of 512 FLOP): 16x16x32 f16 = 16384 FLOP,
    # 16x16x4 f32 = 2048 FLOP
    if "SQ_INSTS_VALU_MFMA_MOPS_F16" in a:
        out.append(f"f16 MFMA {a['SQ_INSTS_VALU_MFMA_MOPS_F16'] * 512 / 16384 / 1e6:.3f} M")
    if "SQ_INSTS_VALU_MFMA_MOPS_F32" in a:
        out.append(f"f32 MFMA {a['SQ_INSTS_VALU_MFMA_MOPS_F32'] * 512 / 2048 / 1e6:.3f} M")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
        out.append(f"MFMA_BUSY {a['SQ_VALU_MFMA_BUSY_CYCLES'] / 1e6:.3f} Mcyc")
    if "GRBM_GUI_ACTIVE" in a:
        out.append(f"GUI_ACTIVE {a['GRBM_GUI_ACTIVE'] / 8:.0f} cyc/XCD")
    w = a.get("SQ_WAVES")
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU"):
        if k in a and w:
            out.append(f"{k[9:]}/wave {a[k] / w:.0f}")
    if "SQ_LDS_BANK_CONFLICT" in a and "SQ_LDS_IDX_ACTIVE" in a and a["SQ_LDS_IDX_ACTIVE"]:
        out.append(f"LDS_conflict {a['SQ_LDS_BANK_CONFLICT'] / a['SQ_LDS_IDX_ACTIVE']:.2f}")
    if "FETCH_SIZE" in a:
        out.append(f"HBM rd {2 * a['FETCH_SIZE'] / 1024:.1f} MB wr {a.get('WRITE_SIZE', 0) / 1024:.1f} MB")
    if "SQ_WAVES" in a:
        out.append(f"waves {a['SQ_WAVES']:.0f}")
    print("  ".join(out))
