#!/usr/bin/env python3
"""Timeline of the last training iteration in a rocprofv3 kernel trace of
tools/train_bench.py: every kernel from the iteration's first k_sample_dw (the
critic sample) to the end, with start offset, duration and queue, then the
per-kernel totals.

    python tools/iter_timeline.py [gpurun_out/prof_train/run_kernel_trace.csv]
"""
import collections
import csv
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_train/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
# the last iteration: from the first kernel after the Adam step that precedes its two
# forward rollouts (its samples were drawn at the end of the previous iteration)
fwd = [i for i, r in enumerate(rows) if re.search(r"k_rollout_nn(4|_x3)?<", r["Kernel_Name"])]
t_first = int(rows[fwd[-2]]["Start_Timestamp"])
adam = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"] and int(r["End_Timestamp"]) <= t_first]
a = adam[-1] + 1 if adam else fwd[-2]
t0 = int(rows[a]["Start_Timestamp"])
qkey = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)


def short(n):
    return n[:40] if n.startswith("Cijk") else re.sub(r"<.*", "", re.sub(r"^void ", "", n))[:60]


agg = collections.OrderedDict()
end = t0
for r in rows[a:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    end = max(end, e)
    d = (e - s) / 1e3
    q = r[qkey] if qkey else "-"
    if d > 5.0:
        print(f"{(s - t0) / 1e3:9.1f} {d:8.1f}  q{q:>3}  {short(r['Kernel_Name'])}")
    c = agg.setdefault(short(r["Kernel_Name"]), [0, 0.0])
    c[0] += 1
    c[1] += d
print(f"== iteration span {(end - t0) / 1e3:.1f} us, {len(rows) - a} kernels")
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {t:8.1f} {n:4d}  {k}")
