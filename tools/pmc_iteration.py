#!/usr/bin/env python3
"""HBM bytes of ONE lqr_d20 training iteration from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; MI355X_MICROARCH.md §HBM: KiB, FETCH_SIZE x2 on gfx950) over tools/train_bench.py:
the dispatches of the last iteration, found as tools/iter_timeline.py finds it (from the kernel
after the Adam step that precedes the last iteration's two forward rollouts), in dispatch order.

    python tools/pmc_iteration.py <fetch run_counter_collection.csv> <write ...csv> > out.json
"""
import collections
import csv
import json
import re
import sys


def per_dispatch(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"], float(r["Counter_Value"])) for r in rows]


def last_iteration(seq):
    names = [n for n, _ in seq]
    fwd = [i for i, n in enumerate(names) if re.search(r"k_rollout_nn(4|_x3)?<", n)]
    start = fwd[-2]
    adam = [i for i in range(start) if "k_adam" in names[i]]
    a = adam[-1] + 1 if adam else start
    return seq[a:]


def short(n):
    return re.sub(r"<.*", "", re.sub(r"^void ", "", n))[:60]


def main():
    f = last_iteration(per_dispatch(sys.argv[1], "FETCH_SIZE"))
    w = last_iteration(per_dispatch(sys.argv[2], "WRITE_SIZE"))
    by = collections.OrderedDict()
    for n, v in f:
        by.setdefault(short(n), [0.0, 0.0])[0] += v * 1024 * 2
    for n, v in w:
        by.setdefault(short(n), [0.0, 0.0])[1] += v * 1024
    tot_r = sum(v[0] for v in by.values())
    tot_w = sum(v[1] for v in by.values())
    out = {"dispatches": [len(f), len(w)], "hbm_read_bytes": tot_r, "hbm_write_bytes": tot_w,
           "hbm_bytes": tot_r + tot_w,
           "per_kernel_GB": {k: [round(v[0] / 1e9, 4), round(v[1] / 1e9, 4)] for k, v in
                             sorted(by.items(), key=lambda kv: -(kv[1][0] + kv[1][1]))},
           "note": "one lqr_d20 fp32 iteration at B = 2048 (tools/train_bench.py), read / written GB per kernel name; "
                   "FETCH_SIZE x2 (gfx950 counts half a wide read), counters in KiB"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
