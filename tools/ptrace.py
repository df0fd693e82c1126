"""Summarise a persistent-decoder phase trace (TTS_PTRACE=<file>): [8 steps][10 stamps][256 WGs]
of s_memrealtime ticks (100 MHz). Stamp 2k = phase k starts (barrier released), 2k+1 = its work
ends (barrier entered); phases P1, P3, P4, P5, P6."""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64).astype(np.int64)
a = raw[:8 * 16 * 256].reshape(8, 16, 256)
at = raw[8 * 16 * 256:].reshape(8, 256, 8) if raw.size > 8 * 16 * 256 else None
names = ["P1 stop+prenet2", "P3 attLSTM+pq", "P4 attention", "P5 decLSTM", "P6 attpre+proj"]
rows = []
for s in range(7):  # the next step's stamp 0 closes the last barrier
    st = a[s]
    nxt = a[s + 1]
    r = []
    for k in range(5):
        start = st[2 * k].min()
        end = st[2 * k + 1]
        rel = (nxt[0] if k == 4 else st[2 * k + 2])
        r.append(((end.max() - start) / 100.0, np.median(end - st[2 * k]) / 100.0, (rel.min() - end.max()) / 100.0,
                  (rel.max() - rel.min()) / 100.0))
    rows.append(r)
rows = np.array(rows)  # steps x phase x 4
med = np.median(rows, axis=0)
print(f"{'phase':18s} {'last WG done':>12s} {'median WG':>10s} {'barrier':>8s} {'release skew':>12s}  (us)")
for k in range(5):
    print(f"{names[k]:18s} {med[k,0]:12.2f} {med[k,1]:10.2f} {med[k,2]:8.2f} {med[k,3]:12.2f}")
step = np.median([(a[s + 1][0].min() - a[s][0].min()) / 100.0 for s in range(7)])
print(f"step {step:.2f} us")
NATT = 64
for agg, lab in ((np.median, "median"), (np.max, "max")):
    sub = [np.median([agg((a[s][k][:NATT] - a[s][2][:NATT]).astype(float) / 100.0) for s in range(7)])
           for k in (13, 10, 11, 12, 3)]
    print(f"P3 inside attention_rnn workgroups ({lab} WG, us after release): staged %.2f, MFMA %.2f, cell %.2f, "
          "query partials %.2f, done %.2f" % tuple(sub))
sub = [np.median([(a[s][k][NATT:] - a[s][2][NATT:]).astype(float) / 100.0 for s in range(7)]) for k in (3,)]
print("P3 item workgroups (h_dec part + frames) done %.2f" % tuple(sub))

g14 = [np.median([(a[s][14] - a[s][4]).astype(float) / 100.0 for s in range(7) if a[s][14].min() > 0])
       for _ in (0,)] if a[:, 14].min() > 0 else None
if g14 is not None:
    print("P4 GEMM waves done (median WG, us after release): %.2f" % g14[0])

if a[:, 15, NATT:].min() > 0:  # item workgroups' P4 entry stamps (15: path taken, 14: first item call)
    s15 = np.median([np.median((a[s][15][NATT:] - a[s][4][NATT:]).astype(float) / 100.0) for s in range(7)])
    s14 = np.median([np.median((a[s][14][NATT:] - a[s][4][NATT:]).astype(float) / 100.0) for s in range(7)])
    print("P4 item workgroups after their own release (median, us): item path %.2f, first item call %.2f" % (s15, s14))
    if at is not None:
        own = []
        for s in range(3):
            for i in range(256 - NATT):
                if at[s][i][0] > 0:
                    own.append((at[s][i][0] - a[s][4][NATT + i]) / 100.0)
        print("P4 items: loads issued %.2f us after their own release (median)" % np.median(own))

if at is not None:
    # attention items: stamps 0 start (after loads), 1 query summed, 2 location conv, 3 energies,
    # 4 energy reduction, 5 partials published, 6 ticket, 7 combine done (last arriver only)
    labels = ["loads", "query", "locconv", "energy", "reduce", "publish", "ticket", "combine"]
    for s in range(3):
        p4start = a[s][4].min()
        items = [i for i in range(256) if at[s][i][0] > 0]
        if not items:
            continue
        d = np.array([[(at[s][i][k] - p4start) / 100.0 if at[s][i][k] > 0 else np.nan for k in range(8)]
                      for i in items])
        print(f"step {s}: {len(items)} items; stamp times after P4 release (us): median / max")
        print("  " + " ".join(f"{labels[k]}={np.nanmedian(d[:, k]):.2f}/{np.nanmax(d[:, k]):.2f}" for k in range(8)))
    # last arrivers: combine done (ctx written) -> their P4 work end (alignment pass + rest)
    IW0 = 64
    tails = []
    for s in range(7):
        for i in range(256 - IW0):
            if at[s][i][7] > 0:
                tails.append((a[s][5][IW0 + i] - at[s][i][7]) / 100.0)
    if tails:
        print("last arrivers: combine done -> P4 end (alignment pass): median %.2f max %.2f us" %
              (np.median(tails), np.max(tails)))
