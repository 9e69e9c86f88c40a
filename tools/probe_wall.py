#!/usr/bin/env python3
"""Where the wall clock of bench.py's headline goes beyond the kernels: K back-to-back
launches of the cold-rotation rollout timed between synchronize pairs, in several forms,
10 repetitions each (median), next to the HIP event pair over the same launches.

    python tools/probe_wall.py [--steps 20]

  plain     bench.py's loop (event pair recorded inside the wall bracket)
  ev_out    the start event recorded before t0 (the wall bracket holds only the launches)
  spin      ev_out, then spin on the end event's query() before synchronize()
  graph     the K launches captured once as a HIP graph, one replay per timing
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    from deeppde_actorcritic_amd import _lib
    from deeppde_actorcritic_amd.equation import LQR
    lib = _lib.load()
    eqp = LQR(bench.lqr_config()).params()
    B, N, d, K = bench.B_PER_GPU, bench.HORIZON, bench.DIM, a.steps
    rs = bench.RolloutSets(lib, eqp, _lib.SCHEME_ADAPTIVE, torch.float32, B, N, d, 0, bench.N_SETS)
    launch = rs.launcher(bench.N_SETS)
    for i in range(10):
        launch(i)
    torch.cuda.synchronize()
    out = {}

    def timed(kind):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        if kind != "plain":
            s.record()
        t0 = time.perf_counter()
        if kind == "plain":
            s.record()
        if kind == "graph":
            g.replay()
        else:
            for i in range(K):
                launch(i)
        e.record()
        if kind == "spin":
            while not e.query():
                pass
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e6, s.elapsed_time(e) / K * 1e3

    # graph of the K launches on the capture stream
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    P = ctypes.c_void_p
    with torch.cuda.graph(g, stream=side):
        st = P(torch.cuda.current_stream().cuda_stream)
        for i in range(K):
            args = rs.args[i % bench.N_SETS][:-1] + (st,)
            rc = lib.dpac_rollout_fwd(*args)
            assert rc == 0, lib.dpac_last_error()
    for kind in ("plain", "ev_out", "spin", "graph"):
        w, ev = [], []
        for _ in range(a.reps):
            x, y = timed(kind)
            w.append(x)
            ev.append(y)
        out[kind] = {"wall_us_per_launch": statistics.median(w), "event_us_per_launch": statistics.median(ev),
                     "wall_all": [round(v, 2) for v in w]}
        print(kind, json.dumps(out[kind]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
