#!/usr/bin/env python3
"""Time dpac_rollout_nn_fwd (fused NN-control rollout) on lqr_d20's actor shape (GPU only).

    python tools/probe_nn.py [--B 2048] [--N 100] [--dtype f32] [--hidden 200,200,200] [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", default="2048")
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--d", type=int, default=20)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--hidden", default="200,200,200")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--save", action="store_true")
    a = ap.parse_args()
    from deeppde_actorcritic_amd import _lib, ops
    from deeppde_actorcritic_amd import equation as peq
    from deeppde_actorcritic_amd import solver as psol
    from deeppde_actorcritic_amd.config import set_floatx
    from tests.helpers import full_config
    dt_ = torch.float32 if a.dtype == "f32" else torch.float64
    set_floatx("float32" if a.dtype == "f32" else "float64")
    hidden = tuple(int(h) for h in a.hidden.split(","))
    cfg = full_config("LQR", a.d, N=a.N, hidden=hidden)
    net = psol.DeepNN(cfg, "actor", torch.Generator().manual_seed(0), dt_, "cuda")
    eqp = peq.LQR(cfg.eqn_config).params()
    view = net.mlp_view()
    macs = sum(hidden[i] * hidden[i + 1] for i in range(len(hidden) - 1)) + a.d * hidden[0] + hidden[-1] * a.d
    for B in [int(v) for v in a.B.split(",")]:
        x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, a.N, seed=1, dtype=dt_, device="cuda")
        run = lambda: ops.rollout_nn(eqp, _lib.SCHEME_ADAPTIVE, x0, dw, 0.2, a.N, view, save=a.save)
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            run()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.reps
        print(json.dumps({"B": B, "N": a.N, "hidden": hidden, "dtype": a.dtype, "ms": ms,
                          "us_per_step": ms * 1e3 / a.N,
                          "mlp_TFLOPs": 2 * macs * B * a.N / (ms * 1e-3) / 1e12}), flush=True)


if __name__ == "__main__":
    main()
