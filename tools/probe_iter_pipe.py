#!/usr/bin/env python3
"""Pipelined lqr_d20 training iterations (bench.py's training variant: no synchronize between
iterations) for a kernel trace, and the steady-state analysis of that trace.

    rocprofv3 --kernel-trace -d gpurun_out/pipe -o run --output-format csv -- \\
        python3 tools/probe_iter_pipe.py --iters 20
    python3 tools/probe_iter_pipe.py --analyze gpurun_out/pipe/run_kernel_trace.csv

The analysis splits the trace at the critic's NN rollout (one per iteration, queue of the
critic) and prints, per iteration, its period (start to next start), the busy time of the
union of all queues, the idle gaps of that union above 5 us, and the kernels that end last."""
import argparse
import csv
import json
import os
import re
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(iters, warmup, batch):
    import torch
    from deeppde_actorcritic_amd import equation as peq
    from deeppde_actorcritic_amd import solver as psol
    from deeppde_actorcritic_amd.config import baseline_config
    cfg = baseline_config(iters, 10 ** 9, "float32", batch, batch, name="lqr_d20")
    sp = psol.ActorCriticSolver(cfg, peq.LQR(cfg.eqn_config), seed=1, sampler="device")
    N = cfg.eqn_config.num_time_interval_critic

    def iteration():
        dc, da = sp.sample_iteration(batch, N, N)
        sp.train_iteration(dc, da, batch)
        sp.prefetch_samples(batch, N, N)
    for _ in range(warmup):
        iteration()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        iteration()
    torch.cuda.synchronize()
    print(json.dumps({"ms_per_iter": (time.perf_counter() - t0) / iters * 1e3, "iters": iters, "batch": batch}))


def analyze(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # the critic's rollout without saves: k_rollout_nn_x3<..., false, false, false>
    starts = [int(r["Start_Timestamp"]) for r in rows
              if "k_rollout_nn_x3<" in r["Kernel_Name"] and "false, false, false" in r["Kernel_Name"]]
    per, busy, gaps = [], [], []
    for a, b in zip(starts[-11:], starts[-10:]):
        ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
              if a <= int(r["Start_Timestamp"]) < b]
        t, tot, g = a, 0, []
        for s, e, n in ks:  # union of intervals
            if s > t:
                if s - t > 5000:
                    g.append((round((t - a) / 1e3, 1), round((s - t) / 1e3, 1)))
                t = s
            if e > t:
                tot += e - t
                t = e
        per.append((b - a) / 1e3)
        busy.append(tot / 1e3)
        gaps.append(g)
    print(json.dumps({"period_us": [round(x, 1) for x in per], "median_period_us": statistics.median(per),
                      "busy_us": [round(x, 1) for x in busy], "gaps_over_5us": gaps}, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--analyze", default=None)
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        run(a.iters, a.warmup, a.batch)
