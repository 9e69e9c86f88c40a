#!/usr/bin/env python3
"""Training-level parity on lqr_d20: err_value (solver.py:109-113) of the product
(GPU, fp32 and fp64) against the float64 CPU oracle, same initial weights and the
same host-sampled numpy stream (solver.py:36-71 run verbatim).

    python tests/train_check.py --iters 200 --log-freq 50 --runs gpu32,gpu64,oracle \
        --out gpurun_out/train_check.json

lqr_d20 is the reference's configs/lqr_d20.json (values restated below): d = c = 20,
N = 100, T = 0.2, 3x200 MLPs, batch = valid = 2048, adaptive scheme, TD1, normal
sampling, actor-critic.  --iters / --log-freq shorten the 50 000-iteration run.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from deeppde_actorcritic_amd import equation as peq  # noqa: E402
from deeppde_actorcritic_amd import solver as psol  # noqa: E402
from deeppde_actorcritic_amd.config import BASELINE_EQN_CONFIGS, baseline_config  # noqa: E402


EQN_CONFIGS = BASELINE_EQN_CONFIGS
lqr_d20 = baseline_config


COLS = ["step", "loss_critic", "loss_actor", "err_value", "err_value_infty", "err_control",
        "err_value_grad", "err_cost", "elapsed"]


def history_dict(h):
    h = np.asarray(h)[:-1]  # last row is the true-loss-actor record (solver.py:62)
    return {c: h[:, i].tolist() for i, c in enumerate(COLS)}


def heartbeat(period=60.0):
    """Print a line every `period` s so a long CPU-oracle run never looks hung."""
    import threading
    t0 = time.perf_counter()

    def beat():
        while True:
            time.sleep(period)
            print(f"... {time.perf_counter() - t0:.0f} s", flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--log-freq", type=int, default=50)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--valid", type=int, default=2048)
    ap.add_argument("--runs", default="gpu32,gpu64,oracle")
    ap.add_argument("--config", default="lqr_d20", choices=sorted(EQN_CONFIGS))
    ap.add_argument("--seed", type=int, default=11, help="weight-initialisation seed")
    ap.add_argument("--data-seed", type=int, default=123, help="np.random.seed before train()")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "train_check.json"))
    ap.add_argument("--graphs", type=int, default=1,
                    help="1: the production path (HIP graphs, split critic/actor steps on side streams)")
    ap.add_argument("--sampler", default="host", choices=["host", "device"],
                    help="host: the reference's numpy stream (needed for the oracle); device: Philox "
                         "drawn in float64 for every run and rounded to the run's dtype (long GPU runs)")
    ap.add_argument("--oracle-from", default=None,
                    help="reuse the oracle history of an earlier train_check JSON (same settings)")
    a = ap.parse_args()
    runs = a.runs.split(",")
    if a.sampler == "device":
        assert "oracle" not in runs and not a.oracle_from, "the oracle needs the host sampler's numpy stream"
    res = {"config": f"{a.config} (configs/{a.config}.json values)", "iters": a.iters, "log_freq": a.log_freq,
           "batch": a.batch, "valid": a.valid, "graphs": bool(a.graphs), "sampler": a.sampler, "runs": {}}
    init = None
    for run in runs:
        if run == "oracle":
            continue
        dtype = "float32" if run == "gpu32" else "float64"
        cfg = lqr_d20(a.iters, a.log_freq, dtype, a.batch, a.valid, a.config)
        bsde = getattr(peq, cfg.eqn_config.eqn_name)(cfg.eqn_config)
        sp = psol.ActorCriticSolver(cfg, bsde, seed=a.seed, sampler=a.sampler, graphs=bool(a.graphs))
        if a.sampler == "device":  # same Philox keys in every run; increments drawn in float64
            draw = bsde.sample_device

            def sample64(kind, n, N, key, off=0, dtype=None, out=None, _draw=draw, _dt=sp.dtype):
                b = _draw(kind, n, N, key, off, torch.float64)
                if out is None:
                    return type(b)(*(t.to(_dt) for t in b))
                for dst, src in zip(out, b):  # the solver's in-place prefetch (its idle graph set)
                    dst.copy_(src)
                return out
            bsde.sample_device = sample64
        if init is None:  # every run starts from the first run's weights, in float64
            init = {"critic": sp.model_critic.NN_value.export_params(),
                    "critic_grad": sp.model_critic.NN_value_grad.export_params(),
                    "actor": sp.model_actor.NN_control.export_params()}
        else:
            sp.model_critic.NN_value.load_params(init["critic"])
            sp.model_critic.NN_value_grad.load_params(init["critic_grad"])
            sp.model_actor.NN_control.load_params(init["actor"])
        np.random.seed(a.data_seed)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h = sp.train()[0]
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        res["runs"][run] = {"history": history_dict(h), "wall_s": wall, "dtype": dtype}
        print(json.dumps({"run": run, "wall_s": wall, "err_value": res["runs"][run]["history"]["err_value"]}),
              flush=True)
    if "oracle" in runs:
        from oracle import equations as oeq
        from oracle import solver as osol
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        cfg = lqr_d20(a.iters, a.log_freq, "float64", a.batch, a.valid, a.config)
        so = osol.ActorCriticSolver(cfg, oeq.make(cfg.eqn_config), params=init)
        np.random.seed(a.data_seed)
        t0 = time.perf_counter()
        h = so.train()
        wall = time.perf_counter() - t0
        res["runs"]["oracle"] = {"history": history_dict(h), "wall_s": wall, "dtype": "float64",
                                 "threads": torch.get_num_threads()}
        print(json.dumps({"run": "oracle", "wall_s": wall, "err_value": res["runs"]["oracle"]["history"]["err_value"]}),
              flush=True)
    if a.oracle_from:
        prev = json.load(open(a.oracle_from))
        assert (prev["iters"], prev["log_freq"], prev["batch"], prev["valid"]) == (a.iters, a.log_freq, a.batch, a.valid)
        assert prev["config"].split()[0] == a.config
        res["runs"]["oracle"] = dict(prev["runs"]["oracle"], source=a.oracle_from)
    if "oracle" in res["runs"]:
        ref = np.array(res["runs"]["oracle"]["history"]["err_value"])
        res["max_abs_err_value_diff_vs_oracle"] = {
            r: float(np.max(np.abs(np.array(v["history"]["err_value"]) - ref)))
            for r, v in res["runs"].items() if r != "oracle"}
        print(json.dumps(res["max_abs_err_value_diff_vs_oracle"]), flush=True)
    elif "gpu64" in res["runs"]:  # long runs: the fp64 product (5.6e-17 of the oracle) as the reference
        ref = np.array(res["runs"]["gpu64"]["history"]["err_value"])
        res["max_abs_err_value_diff_vs_gpu64"] = {
            r: float(np.max(np.abs(np.array(v["history"]["err_value"]) - ref)))
            for r, v in res["runs"].items() if r != "gpu64"}
        res["final_err_value"] = {r: v["history"]["err_value"][-1] for r, v in res["runs"].items()}
        print(json.dumps({k: res[k] for k in ("max_abs_err_value_diff_vs_gpu64", "final_err_value")}), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
