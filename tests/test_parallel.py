"""CPU, world_size 2 over gloo: the data-parallel exchange (parallel.py).

The per-rank compute here is the ORACLE (test infrastructure) standing in for the
GPU path, so the test exercises exactly the distributed logic: shard ranges by
global trajectory index, one flattened gradient all-reduce, metric SUM / MAX —
and checks that the sharded result equals the unsharded one.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deeppde_actorcritic_amd.parallel import DataParallel, shard_range


def test_shard_range_covers_batch():
    for total in (1, 7, 4096, 16384, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert sum(c for _, c in spans) == total
            off = 0
            for o, c in spans:
                assert o == off
                off += c
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import equations as oeq
        from oracle import solver as osol
        from tests.helpers import full_config
        torch.set_num_threads(1)
        cfg = full_config("LQR", 5, N=6, batch=30, hidden=(8, 8), scheme="adaptive", td="TD1")
        eq = oeq.make(cfg.eqn_config)
        gen = torch.Generator().manual_seed(3)
        params = {k: osol.init_params(osol.DeepNN(cfg, ac).sizes, gen)
                  for k, ac in (("critic", "critic"), ("critic_grad", "critic_grad"), ("actor", "actor"))}
        so = osol.ActorCriticSolver(cfg, eq, params=params)
        np.random.seed(9)  # every rank draws the same global batch ...
        x0, dw, xb = eq.sample_normal(30, 6)
        par = DataParallel()
        off, cnt = par.shard(30)  # ... and keeps its shard of global trajectories
        shard = (x0[off:off + cnt], dw[off:off + cnt], xb[off:off + cnt])
        gc, _ = so.grad_critic(shard, False, False)
        ga, _ = so.grad_actor(shard, False, False, False)
        gc = par.allreduce_grads(gc, cnt, 30)
        ga = par.allreduce_grads(ga, cnt, 30)
        # metrics: sums and max over ranks
        x0t = torch.as_tensor(shard[0])
        with torch.no_grad():
            err = eq.V_true(x0t) - so.model_critic.NN_value(x0t)
        num = par.sum(torch.sum(err ** 2))
        mx = par.max(torch.max(torch.abs(err)))
        if rank == 0:
            q.put({"gc": [g.detach() if g is not None else None for g in gc],
                   "ga": [g.detach() for g in ga], "num": float(num), "max": float(mx)})
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gradients_equal_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # the unsharded reference
    from oracle import equations as oeq
    from oracle import solver as osol
    from tests.helpers import full_config
    cfg = full_config("LQR", 5, N=6, batch=30, hidden=(8, 8), scheme="adaptive", td="TD1")
    eq = oeq.make(cfg.eqn_config)
    gen = torch.Generator().manual_seed(3)
    params = {k: osol.init_params(osol.DeepNN(cfg, ac).sizes, gen)
              for k, ac in (("critic", "critic"), ("critic_grad", "critic_grad"), ("actor", "actor"))}
    so = osol.ActorCriticSolver(cfg, eq, params=params)
    np.random.seed(9)
    data = eq.sample_normal(30, 6)
    gc, _ = so.grad_critic(data, False, False)
    ga, _ = so.grad_actor(data, False, False, False)
    for a, b in zip(res["gc"] + res["ga"], gc + ga):
        assert torch.allclose(a, b, rtol=1e-12, atol=1e-13)
    x0t = torch.as_tensor(data[0])
    with torch.no_grad():
        err = eq.V_true(x0t) - so.model_critic.NN_value(x0t)
    assert abs(res["num"] - float(torch.sum(err ** 2))) < 1e-12 * (1 + float(torch.sum(err ** 2)))
    assert res["max"] == float(torch.max(torch.abs(err)))


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        par = DataParallel()
        total = 11  # ragged: shards of 4, 4, 3
        off, cnt = par.shard(total)
        rows = torch.arange(total * 3, dtype=torch.float64).view(total, 3)[off:off + cnt]
        got = par.gather_rows(rows, total)
        seed = par.broadcast_int(1000 + rank)  # every rank ends up with rank 0's value
        q.put((rank, got, seed))
    finally:
        dist.destroy_process_group()


def test_gloo_world3_gather_rows_and_seed_broadcast():
    """parallel.DataParallel.gather_rows (train()'s final validation arrays, solver.py:63-66,
    in global row order from ragged shards) and broadcast_int (one seed on every rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(3)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = torch.arange(33, dtype=torch.float64).view(11, 3)
    for rank, got, seed in res:
        assert torch.equal(got, full)
        assert seed == 1000


def _multi_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        par = DataParallel()
        gen = torch.Generator().manual_seed(100 + rank)
        a = [torch.randn(3, 4, generator=gen, dtype=torch.float64), None,
             torch.randn(5, generator=gen, dtype=torch.float64)]
        b = [torch.randn(7, generator=gen, dtype=torch.float64)]
        cnt_a, cnt_b = (3, 5) if rank == 0 else (2, 4)
        sep = (par.allreduce_grads([t.clone() if t is not None else None for t in a], cnt_a, 5),
               par.allreduce_grads([t.clone() for t in b], cnt_b, 9))
        n0 = par.grad_allreduces
        one = par.allreduce_grads_multi([(a, cnt_a, 5), (b, cnt_b, 9)])
        q.put((rank, sep, one, par.grad_allreduces - n0))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_allreduce_grads_multi_is_one_exchange():
    """allreduce_grads_multi (the actor's gradients and the critic's G half in one flattened
    all-reduce, solver.train_iteration) equals one allreduce_grads per part, each with its own
    shard weight count/total, and counts as ONE gradient all-reduce."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_multi_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, sep, one, n in res:
        assert n == 1
        for s_part, o_part in zip(sep, one):
            for s, o in zip(s_part, o_part):
                assert (s is None) == (o is None)
                if s is not None:
                    assert torch.equal(s, o)
