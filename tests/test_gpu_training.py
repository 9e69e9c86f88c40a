"""GPU: training (solver.py:36-71) at d = 20 against the float64 oracle.

* Joint actor-critic training of every BASELINE equation at d = 20 (VDP with c = 10) against
  the live oracle, small nets, both the eager path and the production path (HIP graphs, the
  critic step split at the G network, the actor's forward rollout on a side stream).
* the BASELINE configs at their batches (lqr_d20 and ekn_d20 at B = 4096, lqr_var_d20 at 2048,
  vdp_d20 at 8192; N = 100, 3x200 MLPs, TD1, adaptive) against the committed oracle vectors
  tests/golden/train_<config>_B<batch>.npz (made by tests/golden/make_train_golden.py in the
  build container: too slow for a GPU test's time limit).
Same initial weights (ActorCriticSolver(seed) draws the Keras initialisers from
torch.Generator().manual_seed(seed), which the oracle's init_params reproduces) and the same
numpy sample stream (sampler="host").  Tolerance: 1e-8 relative (float64; GEMM and reduction
re-association only).
"""
import glob
import os

import numpy as np
import pytest
import torch

from deeppde_actorcritic_amd import equation as peq
from deeppde_actorcritic_amd import solver as psol
from oracle import equations as oeq
from oracle import solver as osol
from tests.helpers import full_config, rel_close

pytestmark = pytest.mark.gpu
GOLDENS = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "train_*_B*.npz")))


def pair(cfg, seed, graphs):
    bp = getattr(peq, cfg.eqn_config.eqn_name)(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bp, seed=seed, sampler="host", graphs=graphs)
    params = {"critic": sp.model_critic.NN_value.export_params(),
              "critic_grad": sp.model_critic.NN_value_grad.export_params(),
              "actor": sp.model_actor.NN_control.export_params()}
    return sp, osol.ActorCriticSolver(cfg, oeq.make(cfg.eqn_config), params=params)


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("name", ["VDP", "LQR", "EKN", "LQR_var"])
def test_joint_training_d20_matches_oracle(name, graphs):
    cfg = full_config(name, 20, N=10, hidden=(32, 32), batch=48, valid=48, iters=3, log_freq=1,
                      train="actor-critic", td="TD1")
    sp, so = pair(cfg, 13, graphs)
    np.random.seed(77)
    hp = sp.train()
    np.random.seed(77)
    ho = so.train()
    assert hp[0].shape == ho.shape == (5, 9)
    assert rel_close(hp[0][:, 1:8], ho[:, 1:8], 1e-8)
    for vp, vo in zip(sp.critic_variables() + sp.actor_variables(), so.critic_vars() + so.actor_vars()):
        assert rel_close(vp.detach().cpu(), vo.detach(), 1e-8)


def summarize(tensors):
    out = []
    for t in tensors:
        t = t.detach().to("cpu", torch.float64).reshape(-1)
        out.append([float(t.sum()), float((t * t).sum())] + t[:16].tolist() + [0.0] * (16 - min(16, t.numel())))
    return np.array(out, dtype=np.float64)


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("path", GOLDENS, ids=[os.path.basename(p)[6:-4] for p in GOLDENS])
def test_baseline_batch_matches_oracle_vectors(path, graphs):
    """float64 training at the BASELINE configs' batches against the committed oracle vectors
    (lqr_d20 / ekn_d20 at 4096, lqr_var_d20 at 2048, vdp_d20 at 8192), 1e-8 relative."""
    from deeppde_actorcritic_amd.config import baseline_config
    g = np.load(path)
    name = str(g["name"]) if "name" in g.files else "lqr_d20"
    seed_params, seed_np, iters, batch, valid = (int(v) for v in g["meta"])
    cfg = baseline_config(iters, 1, "float64", batch, valid, name)
    bsde = getattr(peq, cfg.eqn_config.eqn_name)(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bsde, seed=seed_params, sampler="host", graphs=graphs)
    np.random.seed(seed_np)
    hist = sp.train()[0]
    ref = g["history"]
    assert hist.shape == ref.shape
    assert rel_close(hist[:, 1:8], ref[:, 1:8], 1e-8)
    got = summarize(sp.critic_variables() + sp.actor_variables())
    assert got.shape == g["params"].shape
    assert rel_close(got, g["params"], 1e-8)


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("name,d", [("LQR", 20), ("VDP", 4)])
def test_bounded_sampling_training_matches_oracle(name, d, graphs):
    """sample_type "bounded" (solver.py:26-27 -> equation.py:25-36: the 3-point increments
    +-sqrt(3) w.p. 1/6, 0 w.p. 2/3) end to end: the reference's numpy stream of
    sample_bounded feeds both sides; 3 iterations, logged after each, 1e-8 (float64)."""
    cfg = full_config(name, d, N=10, hidden=(32, 32), batch=48, valid=48, iters=3, log_freq=1,
                      train="actor-critic", td="TD1", sample="bounded")
    sp, so = pair(cfg, 19, graphs)
    np.random.seed(71)
    hp = sp.train()
    np.random.seed(71)
    ho = so.train()
    assert hp[0].shape == ho.shape == (5, 9)
    assert rel_close(hp[0][:, 1:8], ho[:, 1:8], 1e-8)
    for vp, vo in zip(sp.critic_variables() + sp.actor_variables(), so.critic_vars() + so.actor_vars()):
        assert rel_close(vp.detach().cpu(), vo.detach(), 1e-8)


def config0(dtype):
    """BASELINE configs[0]: the reference's configs/lqr_d5.json with TD2, the naive scheme and
    batch 256 (3 iterations, logged after each)."""
    from deeppde_actorcritic_amd.config import munchify
    from tests.helpers import SHIPPED_LQR_D5
    import copy
    c = copy.deepcopy(SHIPPED_LQR_D5)
    c["train_config"].update(TD_type="TD2", scheme="naive")
    c["net_config"].update(batch_size=256, num_iterations=3, logging_frequency=1, dtype=dtype,
                           verbose=False)
    return munchify(c)


@pytest.mark.parametrize("graphs", [False, True])
def test_baseline_config0_lqr_d5_td2_naive_b256_matches_oracle(graphs):
    """BASELINE configs[0] end to end (float64, the reference's dtype) against the live
    oracle: shipped nets (2x200), N = 50, T = 0.2, valid_size 1024; 1e-8."""
    cfg = config0("float64")
    sp, so = pair(cfg, 23, graphs)
    np.random.seed(29)
    hp = sp.train()
    np.random.seed(29)
    ho = so.train()
    assert hp[0].shape == ho.shape == (5, 9)
    assert rel_close(hp[0][:, 1:8], ho[:, 1:8], 1e-8)
    for vp, vo in zip(sp.critic_variables() + sp.actor_variables(), so.critic_vars() + so.actor_vars()):
        assert rel_close(vp.detach().cpu(), vo.detach(), 1e-8)
    assert sp.model_critic.td == 2  # TD2: G is never evaluated, its variables never move
    g0 = sp.model_critic.NN_value_grad.export_params()
    assert all(torch.equal(a, b) for a, b in zip(g0["W"], so.model_critic.NN_value_grad.params["W"]))


def test_baseline_config0_float32_matches_oracle():
    """configs[0] on the float32 production path (HIP graphs; B = 256 takes the 4-row MFMA
    rollout kernel) against the float64 oracle: |d err_value|, |d err_control| <= 1e-5 at every
    logged step (the fp32 tolerance of tests/test_gpu_fp32_production.py)."""
    cfg = config0("float32")
    sp, so = pair(cfg, 23, True)
    np.random.seed(29)
    hp = sp.train()[0]
    np.random.seed(29)
    ho = so.train()
    dv, dc = np.abs(hp[:-1, 3] - ho[:-1, 3]).max(), np.abs(hp[:-1, 5] - ho[:-1, 5]).max()
    print(f"\n[configs[0] fp32] max |d err_value| {dv:.2e}, |d err_control| {dc:.2e}")
    assert dv <= 1e-5 and dc <= 1e-5
    assert rel_close(hp[:, 1:3], ho[:, 1:3], 1e-4)


def test_gback_early_and_late_give_bitwise_equal_parameters(monkeypatch):
    """The critic's G-network backward launched right after the critic head (DPAC_GBACK=early:
    beside V's backward, V's Adam step, the actor's terminal V and then the BPTT) or after the
    BPTT is queued (late, the default) must give bitwise the same parameters: it shares no
    buffer with the work it overlaps (ops._workspace tags 0 / 1).  float32 production path
    (HIP graphs, split critic / actor steps, device sampler), lqr_d20 shape at B = 2048."""
    from deeppde_actorcritic_amd.config import baseline_config
    out = {}
    for mode in ("early", "late"):
        monkeypatch.setattr(psol, "GBACK", mode)
        cfg = baseline_config(4, 10 ** 9, "float32", 2048, 256, "lqr_d20")
        sp = psol.ActorCriticSolver(cfg, peq.LQR(cfg.eqn_config), seed=5, sampler="device")
        for _ in range(4):
            dc, da = sp.sample_iteration(2048, 100, 100)
            sp.train_iteration(dc, da, 2048)
            sp.prefetch_samples(2048, 100, 100)
        torch.cuda.synchronize()
        assert sp._critic_split_ok()
        out[mode] = [v.detach().cpu().clone() for v in sp.critic_variables() + sp.actor_variables()]
    for a, b in zip(out["early"], out["late"]):
        assert torch.equal(a, b)


def _production_params(monkeypatch, attr, value, iters=4, big=None):
    """The float32 production path (HIP graphs, split steps, device sampler, lqr_d20 at B = 2048)
    with psol.<attr> = value: the parameters after `iters` iterations of the loop solver.train
    and bench.py run (sample_iteration / train_iteration / prefetch_samples).  big: every
    network's first hidden BN scale times this factor (split-fp16 operands out of range)."""
    from deeppde_actorcritic_amd import ops
    from deeppde_actorcritic_amd.config import baseline_config
    monkeypatch.setattr(psol, attr, value)
    ops.x3_status_reset("cuda")
    cfg = baseline_config(iters, 10 ** 9, "float32", 2048, 256, "lqr_d20")
    sp = psol.ActorCriticSolver(cfg, peq.LQR(cfg.eqn_config), seed=5, sampler="device")
    if big:
        with torch.no_grad():
            for net in (sp.model_critic.NN_value, sp.model_critic.NN_value_grad, sp.model_actor.NN_control):
                net.bn_gamma[1].mul_(big)
    for _ in range(iters):
        dc, da = sp.sample_iteration(2048, 100, 100)
        sp.train_iteration(dc, da, 2048)
        sp.prefetch_samples(2048, 100, 100)
    torch.cuda.synchronize()
    assert sp._critic_split_ok()
    fell = ops.x3_fell_back("cuda")
    ops.x3_status_reset("cuda")
    return [v.detach().cpu().clone() for v in sp.critic_variables() + sp.actor_variables()], fell


def _bitwise(a, b):
    torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)


def test_graph_sets_one_and_two_give_bitwise_equal_parameters(monkeypatch):
    """DPAC_GRAPH_SETS=2 (prefetch_samples draws the next iteration's samples on a
    side stream straight into the idle graph set's static inputs, guarded by the event recorded
    after the last iteration that used the set) against 1 (one set, the samples copied in):
    bitwise the same parameters over 4 iterations, so no reader of a set's inputs (the side
    stream's forward replay, the G backward's dw rows) races the next draw."""
    p1, _ = _production_params(monkeypatch, "GRAPH_SETS", 1)
    p2, _ = _production_params(monkeypatch, "GRAPH_SETS", 2)
    for a, b in zip(p1, p2):
        assert torch.equal(a, b)


@pytest.mark.parametrize("big", [None, 2.0 ** 20])
def test_guard_deferred_and_inline_give_bitwise_equal_parameters(monkeypatch, big):
    """Round 6: the backward chains' range-guard fallbacks at the end of each
    chain's own graph (DPAC_GUARD_DEFER=1, the default) and as one redo graph after the actor's
    and G's chains join (join) against
    each fallback right behind its split-fp16 launch (0): bitwise the same parameters over 4
    iterations, in range (the fallbacks stay no-ops) and with every network's BN_1 times 2^20
    (the status word is set and the deferred fallbacks recompute the chains in exact f32)."""
    pi, fi = _production_params(monkeypatch, "GUARD_DEFER", False, big=big)
    pd, fd = _production_params(monkeypatch, "GUARD_DEFER", True, big=big)
    assert fi == fd == (big is not None)
    for a, b in zip(pi, pd):
        _bitwise(a, b)
    # DPAC_GUARD_DEFER=join: one redo graph after the chains join (the default ends each chain's
    # own graph with its fallbacks)
    monkeypatch.setattr(psol, "GUARD_DEFER_JOIN", True)
    pj, fj = _production_params(monkeypatch, "GUARD_DEFER", True, big=big)
    assert fj == fi
    for a, b in zip(pi, pj):
        _bitwise(a, b)
