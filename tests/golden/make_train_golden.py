#!/usr/bin/env python3
"""Golden vectors for training at BASELINE sizes, from the float64 CPU oracle (test
infrastructure; run in the build container, not on the GPU box):

    python tests/golden/make_train_golden.py [--threads 8]        # lqr_d20, B = 4096, 6 its
    python tests/golden/make_train_golden.py --name ekn_d20 --batch 4096
    python tests/golden/make_train_golden.py --name lqr_var_d20 --batch 2048
    python tests/golden/make_train_golden.py --name vdp_d20 --batch 8192

-> tests/golden/train_<name>_B<batch>.npz: solver.py:36-71 run verbatim by the oracle for
the given iterations (logging every iteration) on the BASELINE config (d = 20, N = 100,
T = 0.2, 3x200 MLPs, TD1, adaptive, normal sampling, actor-critic; configs/*_d20.json)
with the given batch_size and valid_size 512, initial weights from the product's
initialiser (seed 11: the Keras initialisers drawn from torch.Generator().manual_seed(11)
in the order critic V, critic G, actor, which is what ActorCriticSolver(seed=11) draws)
and the reference's numpy sample stream after np.random.seed(123).  lqr_d20 is BASELINE
configs[1]; ekn_d20 configs[2] at its one-GPU batch; lqr_var_d20 at 2048 and vdp_d20 at
8192, the per-rank shards of configs[3] (16384 / 8) and configs[4] (65536 / 8).

Stored: the 9-column history, and per trainable tensor (critic V, critic G, actor, in
trainable_variables() order) its sum, sum of squares and first 16 entries after the
loop (solver.py:44-70 trains at every step, the last logged one included).  The oracle needs about
10 CPU-minutes per iteration at this size, too slow for a GPU test's time limit, so the
test (tests/test_gpu_training.py) compares against these vectors.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

SEED_PARAMS, SEED_NUMPY, ITERS, BATCH, VALID, NAME = 11, 123, 6, 4096, 512, "lqr_d20"


def config(name=NAME, iters=ITERS, batch=BATCH, valid=VALID):
    from deeppde_actorcritic_amd.config import baseline_config
    return baseline_config(iters, 1, "float64", batch, valid, name)


def summarize(tensors):
    out = []
    for t in tensors:
        t = torch.as_tensor(t, dtype=torch.float64).reshape(-1)
        out.append([float(t.sum()), float((t * t).sum())] + t[:16].tolist() + [0.0] * (16 - min(16, t.numel())))
    return np.array(out, dtype=np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--name", default=NAME)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--iters", type=int, default=ITERS)
    ap.add_argument("--valid", type=int, default=VALID)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    from oracle import equations as oeq
    from oracle import solver as osol
    cfg = config(a.name, a.iters, a.batch, a.valid)
    bo = oeq.make(cfg.eqn_config)
    gen = torch.Generator().manual_seed(SEED_PARAMS)
    params = {k: osol.init_params(osol.DeepNN(cfg, ac).sizes, gen)
              for k, ac in (("critic", "critic"), ("critic_grad", "critic_grad"), ("actor", "actor"))}
    so = osol.ActorCriticSolver(cfg, bo, params=params)
    np.random.seed(SEED_NUMPY)
    t0 = time.time()
    hist = so.train()
    print(f"oracle train: {time.time() - t0:.0f} s", flush=True)
    np.savez_compressed(os.path.join(HERE, f"train_{a.name}_B{a.batch}.npz"),
                        history=np.asarray(hist, dtype=np.float64),
                        params=summarize([v.detach() for v in so.critic_vars() + so.actor_vars()]),
                        meta=np.array([SEED_PARAMS, SEED_NUMPY, a.iters, a.batch, a.valid], dtype=np.int64),
                        name=np.array(a.name))


if __name__ == "__main__":
    main()
