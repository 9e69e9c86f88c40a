#!/usr/bin/env python3
"""Time the in-kernel Philox rollout (dpac_rollout_fwd with dw = NULL) and the device sampler at
the bench shape (LQR d = 20, B = 4096, N = 200, adaptive, analytic control), 5 rotating output
sets: HIP event pair over K launches.  One JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deeppde_actorcritic_amd import _lib, ops  # noqa: E402
from deeppde_actorcritic_amd.equation import LQR  # noqa: E402
import bench  # noqa: E402


def timed(fn, k=40, w=5):
    for i in range(w):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(k):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k * 1e3  # us


def main():
    torch.cuda.set_device(0)
    eqp = LQR(bench.lqr_config()).params()
    B, N, d = 4096, 200, 20
    sets = []
    for i in range(5):
        x0, _, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=7 + i, device="cuda", want_dw=False)
        sets.append(x0)
    us_philox = timed(lambda i: ops.rollout_analytic(eqp, _lib.SCHEME_ADAPTIVE, sets[i % 5], None, 0.2, N,
                                                     seed=99 + i))
    bufs = [(torch.empty(B, d, device="cuda"), torch.empty(N, B, d, device="cuda"), torch.empty(B, d, device="cuda"))
            for _ in range(5)]
    us_sample = timed(lambda i: ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=5 + i, device="cuda", out=bufs[i % 5]))
    print(json.dumps({"lib": _lib.LIB_PATH, "philox_rollout_us": us_philox,
                      "philox_traj_steps_per_s": B * N / (us_philox * 1e-6), "sample_us": us_sample,
                      "sample_GBps": (N + 2) * B * d * 4 / (us_sample * 1e-6) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
