"""GPU: a state dimension outside the main build (4, 5, 10, 20) through a dimension plugin.

The reference's Equation takes any `dim` (equation.py:7-11).  libdpac compiles its equation
kernels per dimension; `make ext EXT_DIMS=7` (run by __graft_entry__.build()) builds
libdpac_d7.so, whose instantiations register into libdpac's dispatch table when _lib.load()
loads it.  Checked at d = 7 against the float64 oracle: the rollout of both schemes for the
three equations that allow an odd dimension (VDP needs d = 2c), and joint actor-critic training
(solver.py:36-71), at the tolerances of the d = 20 tests (1e-12 paths, 1e-8 training).
DPAC_TEST_DIM=<d> runs the same checks at another dimension: without a prebuilt plugin the
first call builds it on demand (_lib.ensure_dim, round 6: a run-time state dimension).
"""
import os

import numpy as np
import pytest
import torch

from deeppde_actorcritic_amd import _lib, ops
from deeppde_actorcritic_amd import equation as peq
from deeppde_actorcritic_amd import solver as psol
from oracle import equations as oeq
from oracle import solver as osol
from tests.helpers import full_config, rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
D = int(os.environ.get("DPAC_TEST_DIM", "7"))


@pytest.mark.parametrize("scheme", ["adaptive", "naive"])
@pytest.mark.parametrize("name", ["LQR", "EKN", "LQR_var"])
def test_rollout_d7_matches_oracle(name, scheme):
    cfg = full_config(name, D, N=16, scheme=scheme)
    bp, bo = getattr(peq, name)(cfg.eqn_config), oeq.make(cfg.eqn_config)
    assert _lib.ensure_dim(bp.params())  # prebuilt (d = 7) or compiled on demand
    assert _lib.load().dpac_supported(bp.params()) == 1
    np.random.seed(3)
    B, N = 300, 16
    x0, dw, _ = bo.sample_normal(B, N)
    prop = bo.propagate_adaptive if scheme == "adaptive" else bo.propagate_naive
    xr, dtr, cr = prop(B, x0, dw, None, False, 0.2, N, True)
    x, dt, coef, *_ = ops.rollout_analytic(
        bp.params(), _lib.SCHEME_ADAPTIVE if scheme == "adaptive" else _lib.SCHEME_NAIVE,
        torch.as_tensor(x0, device=DEV), torch.as_tensor(dw, device=DEV).permute(2, 0, 1).contiguous(), 0.2, N)
    assert np.array_equal(coef.cpu().numpy(), cr.numpy())
    assert rel_close(x.permute(1, 2, 0).cpu().numpy(), xr.numpy(), 1e-12)
    assert rel_close(dt.cpu().numpy(), dtr.numpy(), 1e-12)


@pytest.mark.parametrize("graphs", [False, True])
def test_training_d7_matches_oracle(graphs):
    cfg = full_config("LQR", D, N=10, hidden=(32, 32), batch=48, valid=48, iters=3, log_freq=1,
                      train="actor-critic", td="TD1")
    bp = peq.LQR(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bp, seed=13, sampler="host", graphs=graphs)
    params = {"critic": sp.model_critic.NN_value.export_params(),
              "critic_grad": sp.model_critic.NN_value_grad.export_params(),
              "actor": sp.model_actor.NN_control.export_params()}
    so = osol.ActorCriticSolver(cfg, oeq.make(cfg.eqn_config), params=params)
    np.random.seed(77)
    hp = sp.train()
    np.random.seed(77)
    ho = so.train()
    assert hp[0].shape == ho.shape == (5, 9)
    assert rel_close(hp[0][:, 1:8], ho[:, 1:8], 1e-8)
    for vp, vo in zip(sp.critic_variables() + sp.actor_variables(), so.critic_vars() + so.actor_vars()):
        assert rel_close(vp.detach().cpu(), vo.detach(), 1e-8)
