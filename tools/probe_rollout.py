#!/usr/bin/env python3
"""Probe the rollout kernel: per-launch time vs batch size / horizon / dtype.

    python tools/probe_rollout.py [--B 4096,8192,16384] [--N 200] [--reps 50]
Prints one JSON line per configuration (GPU only).
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", default="4096,8192,16384")
    ap.add_argument("--N", default="200")
    ap.add_argument("--d", type=int, default=20)
    ap.add_argument("--eqn", default="LQR")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--scheme", default="adaptive")
    ap.add_argument("--philox", action="store_true")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--sets", type=int, default=1, help="rotate over this many buffer sets (5: not MALL-resident)")
    a = ap.parse_args()
    from deeppde_actorcritic_amd import _lib, ops
    from deeppde_actorcritic_amd import equation as peq
    from tests.helpers import eqn_config
    lib = _lib.load()
    dt_ = torch.float32 if a.dtype == "f32" else torch.float64
    sch = _lib.SCHEME_ADAPTIVE if a.scheme == "adaptive" else _lib.SCHEME_NAIVE
    for N in [int(v) for v in a.N.split(",")]:
        cfg = eqn_config(a.eqn, a.d, T=0.2, N=N)
        eqp = getattr(peq, a.eqn)(cfg).params()
        for B in [int(v) for v in a.B.split(",")]:
            P = ctypes.c_void_p
            keep, argl = [], []
            for k in range(a.sets):
                x0, dw, _ = ops.sample(eqp, 0, B, N, seed=1 + k, dtype=dt_, device="cuda")
                x = torch.empty(N + 1, B, a.d, dtype=dt_, device="cuda")
                dt = torch.empty(B, N, dtype=dt_, device="cuda")
                coef = torch.empty(B, N, dtype=dt_, device="cuda")
                keep.append((x0, dw, x, dt, coef))
                argl.append((ctypes.byref(eqp), sch, _lib.F32 if dt_ == torch.float32 else _lib.F64, B, N, 0.2,
                             P(x0.data_ptr()), None if a.philox else P(dw.data_ptr()), 1, 0, 0, P(x.data_ptr()),
                             P(dt.data_ptr()), P(coef.data_ptr()), None, 0, None, None,
                             P(torch.cuda.current_stream().cuda_stream)))
            args = argl[0]
            for _ in range(5):
                lib.dpac_rollout_fwd(*args)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for i in range(a.reps):
                assert lib.dpac_rollout_fwd(*argl[i % a.sets]) == 0
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.reps
            esz = 4 if dt_ == torch.float32 else 8
            byts = B * N * ((a.d if not a.philox else 0) + a.d + 2) * esz
            print(json.dumps({"B": B, "N": N, "d": a.d, "eqn": a.eqn, "dtype": a.dtype, "philox": a.philox, "sets": a.sets,
                              "us": ms * 1e3, "ns_per_step": ms * 1e6 / N, "GBps": byts / ms / 1e6,
                              "traj_steps_per_s": B * N / ms * 1e3}), flush=True)


if __name__ == "__main__":
    main()
