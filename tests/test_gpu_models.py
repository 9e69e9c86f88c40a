"""GPU parity of the models and the training loop against the oracle (float64).

The product (libdpac kernels + PyTorch MLPs on the GPU) and the oracle
(torch-CPU restatement of solver.py/equation.py) start from the same weights and
the same host-sampled inputs; losses and gradients must agree to 1e-9 relative
(float64; the bound covers re-association inside GEMMs / reductions).
"""
import ctypes

import numpy as np
import pytest
import torch

from deeppde_actorcritic_amd import equation as peq
from deeppde_actorcritic_amd import solver as psol
from oracle import equations as oeq
from oracle import solver as osol
from tests.helpers import full_config, rel_close

pytestmark = pytest.mark.gpu
TOL = 1e-9


def pair(cfg, seed=0):
    bp = getattr(peq, cfg.eqn_config.eqn_name)(cfg.eqn_config)
    bo = oeq.make(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bp, seed=seed, sampler="host")
    params = {"critic": sp.model_critic.NN_value.export_params(),
              "critic_grad": sp.model_critic.NN_value_grad.export_params(),
              "actor": sp.model_actor.NN_control.export_params()}
    so = osol.ActorCriticSolver(cfg, bo, params=params)
    return sp, so


def grads_close(gp, go, tol=TOL):
    assert len(gp) == len(go)
    for a, b in zip(gp, go):
        if b is None:
            assert a is None or float(a.abs().max()) == 0.0
            continue
        assert a is not None
        assert rel_close(a.detach().cpu(), b.detach(), tol), float((a.detach().cpu() - b).abs().max())


CASES = [("LQR", 5, "adaptive", "TD1"), ("LQR", 20, "naive", "TD2"), ("VDP", 4, "adaptive", "TD1"),
         ("VDP", 10, "naive", "TD1"), ("EKN", 5, "adaptive", "TD1"), ("EKN", 5, "naive", "TD2"),
         ("LQR_var", 5, "adaptive", "TD1"), ("LQR_var", 10, "naive", "TD1")]


@pytest.mark.parametrize("name,d,scheme,td", CASES)
def test_critic_loss_and_gradients(name, d, scheme, td):
    cfg = full_config(name, d, N=12, batch=48, scheme=scheme, td=td)
    sp, so = pair(cfg)
    np.random.seed(4)
    data = so.sample(48, 12)
    for cheat in (False, True):
        gp = sp.grad_critic(data, False, cheat)
        go, lo = so.grad_critic(data, False, cheat)
        lp = sp.loss_critic(data, False, cheat)
        assert rel_close(float(lp), float(lo), TOL)
        grads_close(gp, go)


@pytest.mark.parametrize("name,d,scheme,td", CASES)
def test_actor_loss_and_gradients(name, d, scheme, td):
    """BPTT through the rollout: dpac_step_bwd + MLP autograd vs the oracle tape."""
    cfg = full_config(name, d, N=12, batch=48, scheme=scheme, td=td)
    sp, so = pair(cfg)
    np.random.seed(5)
    data = so.sample(48, 12)
    for cheat_value in (False, True):
        gp = sp.grad_actor(data, False, cheat_value, False)
        go, lo = so.grad_actor(data, False, cheat_value, False)
        lp = sp.loss_actor(data, False, cheat_value, False)
        assert rel_close(float(lp), float(lo), TOL)
        grads_close(gp, go)
    with torch.no_grad():  # analytic control and value (true_loss_actor, solver.py:42)
        lp = sp.loss_actor(data, False, True, True)
    lo = so.loss_actor(data, False, True, True)
    assert rel_close(float(lp), float(lo), TOL)


@pytest.mark.parametrize("name,d,train", [("LQR", 5, "actor-critic"), ("VDP", 4, "critic"),
                                          ("EKN", 5, "actor"), ("LQR_var", 5, "actor-critic")])
def test_training_iterations_match_oracle(name, d, train):
    """solver.py:36-71 end to end: same numpy stream, same weights, 3 iterations."""
    cfg = full_config(name, d, N=8, batch=32, valid=32, iters=3, log_freq=1, train=train)
    sp, so = pair(cfg, seed=11)
    np.random.seed(123)
    hp = sp.train()
    np.random.seed(123)
    ho = so.train()
    assert hp[0].shape == ho.shape == (5, 9)
    assert rel_close(hp[0][:, 1:8], ho[:, 1:8], 1e-8)
    for vp, vo in zip(sp.critic_variables() + sp.actor_variables(),
                      so.critic_vars() + so.actor_vars()):
        assert rel_close(vp.detach().cpu(), vo.detach(), 1e-8)
    x0, y, true_y, z, true_z, grad_y = hp[1:]
    assert x0.shape == (32, d) and y.shape == (32, 1) and true_y.shape == (32, 1)
    assert z.shape == true_z.shape == (32, cfg.eqn_config.control_dim) and grad_y.shape == (32, d)


def test_reference_layout_propagate_surface():
    """Equation.propagate_* keep the reference signature and layouts (equation.py:46, :73)."""
    cfg = full_config("LQR", 5, N=10)
    bp = peq.LQR(cfg.eqn_config)
    bo = oeq.LQR(cfg.eqn_config)
    np.random.seed(8)
    x0, dw, _ = bo.sample_normal(16, 10)
    from deeppde_actorcritic_amd.config import set_floatx
    set_floatx("float64")
    for name in ("propagate_naive", "propagate_adaptive"):
        xs, dt, coef = getattr(bp, name)(16, x0, dw, None, False, 0.2, 10, True)
        xr, dtr, cr = getattr(bo, name)(16, x0, dw, None, False, 0.2, 10, True)
        assert tuple(xs.shape) == (16, 5, 11) and tuple(dt.shape) == (16, 10)
        assert rel_close(xs.cpu(), xr, 1e-12) and rel_close(dt.cpu(), dtr, 1e-12)
        assert np.array_equal(coef.cpu().numpy(), cr.numpy())


@pytest.mark.parametrize("name,d,td", [("LQR", 20, "TD1"), ("EKN", 5, "TD2"), ("VDP", 4, "TD1")])
def test_hip_graph_steps_match_eager(name, d, td):
    """Training steps replayed from captured HIP graphs give the parameters of eager steps."""
    cfg = full_config(name, d, N=10, hidden=(32, 32), batch=64, valid=64, td=td)
    res = []
    for graphs in (False, True):
        bp = getattr(peq, name)(cfg.eqn_config)
        sp = psol.ActorCriticSolver(cfg, bp, seed=7, sampler="device", graphs=graphs)
        for _ in range(3):
            sp.train_step_critic(sp.sample(64, 10))
            sp.train_step_actor(sp.sample(64, 10))
        res.append([v.detach().cpu() for v in sp.critic_variables() + sp.actor_variables()])
    for a, b in zip(*res):
        assert rel_close(a, b, 1e-12)


@pytest.mark.parametrize("name,d,td,train,cheat", [("LQR", 20, "TD1", "actor-critic", False),
                                                  ("EKN", 5, "TD2", "actor-critic", False),
                                                  ("VDP", 4, "TD1", "actor-critic", False)])
def test_overlapped_iteration_matches_sequential(name, d, td, train, cheat):
    """train_iteration (the actor's forward rollout on a side stream during the critic
    step, its gradient from the saves afterwards) gives the parameters of sequential
    eager critic + actor steps (float64, 1e-12)."""
    cfg = full_config(name, d, N=10, hidden=(32, 32), batch=64, valid=64, td=td, train=train)
    res = []
    for overlap in (False, True):
        bp = getattr(peq, name)(cfg.eqn_config)
        sp = psol.ActorCriticSolver(cfg, bp, seed=7, sampler="device", graphs=overlap)
        for _ in range(3):
            dc = sp.sample(64, 10)
            da = sp.sample(64, 10)
            if overlap:
                sp.train_iteration(dc, da)
            else:
                sp.train_step_critic(dc)
                sp.train_step_actor(da)
        res.append([v.detach().cpu() for v in sp.critic_variables() + sp.actor_variables()])
    for a, b in zip(*res):
        assert rel_close(a, b, 1e-12)


def test_actor_grads_from_saves_match_tape():
    """actor_grads_from(actor_forward(batch)) equals grad_actor (autograd through the fused
    rollout) on the same batch, float64."""
    cfg = full_config("LQR", 20, N=12, hidden=(40, 40), batch=50, valid=50)
    sp = psol.ActorCriticSolver(cfg, peq.LQR(cfg.eqn_config), seed=3, sampler="device", graphs=False)
    data = sp.sample(50, 12)
    g_tape = sp.grad_actor(data, False, False, False)
    g_split = sp.actor_grads_from(sp.actor_forward(data))
    for a, b in zip(g_split, g_tape):
        assert rel_close(a.cpu(), b.cpu(), 1e-12)


@pytest.mark.parametrize("name,d", [("LQR", 20), ("VDP", 10), ("EKN", 5)])
def test_critic_split_grads_match_tape(name, d):
    """critic_front (V's gradients, dL/dG) + critic_G_back (G's gradients from the saves)
    equal grad_critic (autograd through the whole critic loss) on the same batch,
    float64."""
    cfg = full_config(name, d, N=12, hidden=(40, 40), batch=50, valid=50, td="TD1")
    bp = getattr(peq, name)(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bp, seed=3, sampler="device", graphs=False)
    data = sp.sample(50, 12)
    g_tape = sp.grad_critic(data, False, False)
    front = sp.critic_front(data)
    g_split = front[0] + sp.critic_G_back(front)
    assert len(g_split) == len(g_tape)
    for a, b in zip(g_split, g_tape):
        assert rel_close(a.cpu(), b.cpu(), 1e-12)


def test_sample_iteration_prefetch_keeps_the_sample_stream():
    """sample_iteration + prefetch_samples (the next iteration's pair drawn on a side stream)
    return the same batches, bit for bit, as drawing critic then actor samples in place."""
    cfg = full_config("LQR", 20, N=12, hidden=(16, 16), batch=64, valid=64)
    a = psol.ActorCriticSolver(cfg, peq.LQR(cfg.eqn_config), seed=5, sampler="device", graphs=False)
    b = psol.ActorCriticSolver(cfg, peq.LQR(cfg.eqn_config), seed=5, sampler="device", graphs=False)
    for _ in range(3):
        got = a.sample_iteration(64, 12, 12)
        a.prefetch_samples(64, 12, 12)
        ref = (b.sample(64, 12), b.sample(64, 12))
        for ga, rb in zip(got, ref):
            for x, y in zip(ga, rb):
                assert torch.equal(x, y)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_critic_loss_grad_kernel_matches_tensor_ops(dtype):
    """dpac_critic_loss_grad (the critic loss's gradient at V's outputs, solver.py:73-78,
    189-190) is bitwise the tensor expressions it replaces, including deltas past the Huber
    clip on both sides and a zero delta; and rejects malformed calls."""
    from deeppde_actorcritic_amd import _lib, ops
    B = 1000
    g = torch.Generator().manual_seed(3)
    V = (torch.randn(3 * B, 1, generator=g, dtype=torch.float64) * 40).to(dtype).cuda()
    y = (torch.randn(B, generator=g, dtype=torch.float64) * 40).to(dtype).cuda()
    disc = torch.rand(B, generator=g, dtype=torch.float64).to(dtype).cuda()
    zb = (torch.randn(B, 1, generator=g, dtype=torch.float64) * 40).to(dtype).cuda()
    V[0, 0], y[0], V[B, 0] = 1.0, 1.0, 0.0  # delta = 0 exactly
    g_out, neg_g = ops.critic_loss_grad(V, y, disc, zb, 100.0 / B, psol.DELTA_CLIP)
    Vv = V[:, 0]
    delta = Vv[:B] - y - Vv[B:2 * B] * disc
    delta_b = Vv[2 * B:] - zb[:, 0]
    gr = psol._huber_grad(delta) * (100.0 / B)
    ref = torch.cat([gr, -gr * disc, psol._huber_grad(delta_b) * (100.0 / B)]).unsqueeze(1)
    assert int((delta.abs() >= psol.DELTA_CLIP).sum()) > 10 and int((delta.abs() < psol.DELTA_CLIP).sum()) > 10
    assert torch.equal(g_out, ref) and torch.equal(neg_g, -gr)
    lib = _lib.load()
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    assert lib.dpac_critic_loss_grad(_lib.F32, 0, P(V), P(y), P(disc), P(zb), 1.0, 50.0, P(V), P(y),
                                     None) == _lib.DPAC_EINVAL
    assert lib.dpac_critic_loss_grad(_lib.F32, B, None, P(y), P(disc), P(zb), 1.0, 50.0, P(V), P(y),
                                     None) == _lib.DPAC_EINVAL
    assert lib.dpac_critic_loss_grad(_lib.F32, B, P(V), P(y), P(disc), P(zb), 1.0, 0.0, P(V), P(y),
                                     None) == _lib.DPAC_EINVAL
