#!/usr/bin/env python3
"""Multi-rank product path == single-process path (float64), on one GPU.

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tests/dp_equality.py --out gpurun_out/dp_equality.json

Each rank runs the PRODUCT solver with parallel.DataParallel over gloo (both ranks share
cuda:0; RCCL needs one GPU per rank): train_iteration with its HIP graphs, the critic step
split at the G network (V's all-reduce on the current stream, G's on the side stream that
runs G's backward), then the actor's all-reduce — solver.py:67-70 order, gradient sites
:88 and :95 of the reference.  Rank 0 then runs the same iterations in one process on the
whole batch (the device sampler is keyed by global trajectory index, so rank r's shard is
rows [off, off+cnt) of that batch) and compares every parameter; then train() end to end
(validation metrics reduced over ranks, the final arrays gathered in global order) against
the single-process train().  Cases: lqr_var_d20 (BASELINE configs[3]) and vdp_d20
(configs[4]) at d = 20 with TD1, lqr_var_d20 with TD2 (no G network: no split critic).
Writes one JSON object (max relative differences) and exits non-zero past 1e-12, or if a
train_iteration issues other than two gradient all-reduces (V's; the actor's with G's).
With --backend nccl every collective of that path runs on RCCL (the seed broadcast on a
device tensor, the gradient all-reduces on the current and the side stream, the metric
reductions, the device all-gather of the final arrays); a one-GPU box runs it as one rank.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TOL = 1e-12
CASES = [("lqr_var_d20", "TD1"), ("vdp_d20", "TD1"), ("lqr_var_d20", "TD2")]


def config(name, td, B, N=10, hidden=(48, 48), iters=2):
    from deeppde_actorcritic_amd.config import BASELINE_EQN_CONFIGS, munchify
    eqn = dict(BASELINE_EQN_CONFIGS[name], total_time_critic=0.2, total_time_actor=0.2,
               num_time_interval_critic=N, num_time_interval_actor=N)
    return munchify({
        "eqn_config": eqn,
        "net_config": {"num_hiddens_critic": list(hidden), "num_hiddens_actor": list(hidden),
                       "lr_values_critic": [1e-3, 1e-4, 1e-5], "lr_boundaries_critic": [30000, 40000],
                       "lr_values_actor": [1e-3, 1e-4, 1e-5], "lr_boundaries_actor": [30000, 40000],
                       "num_iterations": iters, "batch_size": B, "valid_size": B,
                       "logging_frequency": 1, "dtype": "float64", "verbose": False},
        "train_config": {"sample_type": "normal", "scheme": "adaptive", "TD_type": td,
                         "train": "actor-critic"},
    })


def make(cfg, par):
    from deeppde_actorcritic_amd import equation as peq
    from deeppde_actorcritic_amd import solver as psol
    bsde = getattr(peq, cfg.eqn_config.eqn_name)(cfg.eqn_config)
    return psol.ActorCriticSolver(cfg, bsde, seed=7, sampler="device", parallel=par)


def iterate(sp, B, N, k, counts=None):
    """k iterations of solver.train's loop body; counts (a list) receives the gradient
    all-reduces each train_iteration issued (two)."""
    for _ in range(k):
        dc, da = sp.sample_iteration(B, N, N)
        before = sp.par.grad_allreduces
        sp.train_iteration(dc, da, B)
        if counts is not None:
            counts.append(sp.par.grad_allreduces - before)
        sp.prefetch_samples(B, N, N)
    torch.cuda.synchronize()
    return [v.detach().cpu().clone() for v in sp.critic_variables() + sp.actor_variables()]


def rel(a, b):
    return max(float((x - y).abs().max() / (1 + y.abs().max())) for x, y in zip(a, b))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--batch", type=int, default=40)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--backend", default="gloo", choices=["gloo", "nccl"],
                    help="nccl (= RCCL): one rank per GPU, so on a one-GPU box a single rank")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dist.init_process_group(a.backend)
    from deeppde_actorcritic_amd.config import set_floatx
    from deeppde_actorcritic_amd.parallel import DataParallel
    set_floatx("float64")
    rank, world = dist.get_rank(), dist.get_world_size()
    res = {"world": world, "backend": "gloo (ranks share cuda:0)" if a.backend == "gloo" else
           f"nccl = RCCL, {world} rank(s), one GPU each", "tol": TOL, "cases": []}
    ok = True
    B, N = a.batch, 10
    for name, td in CASES:
        cfg = config(name, td, B, N)
        counts = []
        dp = iterate(make(cfg, DataParallel()), B, N, a.iters, counts)
        cfg2 = config(name, td, B, N)
        hist_dp = make(cfg2, DataParallel()).train()
        case = {"config": name, "TD": td, "batch": B, "N": N, "iterations": a.iters,
                "grad_allreduces_per_iteration": counts}
        if rank == 0:
            ref = iterate(make(config(name, td, B, N), None), B, N, a.iters)
            case["params_max_rel_diff"] = rel(dp, ref)
            hist_1 = make(config(name, td, B, N), None).train()
            h_dp, h_1 = np.asarray(hist_dp[0])[:, 1:8], np.asarray(hist_1[0])[:, 1:8]
            case["history_max_rel_diff"] = float(np.max(np.abs(h_dp - h_1) / (1 + np.abs(h_1))))
            outs = [float(np.max(np.abs(p - q))) for p, q in zip(hist_dp[1:], hist_1[1:])]
            case["final_arrays_rows"] = int(hist_dp[1].shape[0])
            case["final_arrays_max_abs_diff"] = max(outs)
            good = (case["params_max_rel_diff"] <= TOL and case["history_max_rel_diff"] <= TOL
                    and case["final_arrays_max_abs_diff"] <= TOL and case["final_arrays_rows"] == B
                    and counts == [2] * a.iters)
            case["ok"] = good
            ok = ok and good
            print(json.dumps(case), flush=True)
        res["cases"].append(case)
        dist.barrier()
    res["ok"] = ok
    if rank == 0 and a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    flag = torch.tensor([0 if ok else 1], device="cuda" if a.backend == "nccl" else "cpu")
    dist.broadcast(flag, 0)
    dist.destroy_process_group()
    sys.exit(int(flag.item()))


if __name__ == "__main__":
    main()
