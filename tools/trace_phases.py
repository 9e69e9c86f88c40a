#!/usr/bin/env python3
"""Per-phase kernel time of the last training iteration in a rocprofv3 kernel trace
(critic = from the critic's k_sample_dw to the actor's; actor = the rest)."""
import collections
import csv
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_train/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_sample_dw" in r["Kernel_Name"]]


def short(n):
    return n[:40] if n.startswith("Cijk") else re.sub(r"<.*", "", n)[:70]


for name, (a, b) in {"critic": (idx[-2], idx[-1]), "actor": (idx[-1], len(rows))}.items():
    agg = collections.OrderedDict()
    span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
    busy = 0.0
    for r in rows[a:b]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        busy += d
        c = agg.setdefault(short(r["Kernel_Name"]), [0, 0.0])
        c[0] += 1
        c[1] += d
    print(f"== {name}: {b - a} kernels, span {span:.1f} us, busy {busy:.1f} us")
    for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {t:8.1f} {n:4d}  {k}")
