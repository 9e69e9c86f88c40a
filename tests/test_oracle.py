"""CPU: the oracle against the golden fixtures and closed-form known answers."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import equations as oeq
from tests.helpers import eqn_config

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "sampler_*.npz"))))
def test_oracle_sampler_matches_reference_outputs(path):
    """Pins the oracle's sampler (and its RNG call order) bit-for-bit to the
    reference's own sample_normal / sample_bounded / sample0 (equation.py:13-44)."""
    g = np.load(path)
    cfg = eqn_config("LQR", int(g["dim"]), R=float(g["R"]))
    eq = oeq.LQR(cfg)
    B, N, seed = int(g["num_sample"]), int(g["N"]), int(g["seed"])
    for name in ("sample_normal", "sample_bounded", "sample0"):
        np.random.seed(seed)
        x0, dw, xb = getattr(eq, name)(B, N)
        assert np.array_equal(x0, g[f"{name}_x0"]), name
        assert np.array_equal(dw, g[f"{name}_dw"]), name
        assert np.array_equal(xb, g[f"{name}_x_bdry"]), name
    np.random.seed(seed)
    a = eq.sample_normal(B, N)
    b = eq.sample_normal(B, N)
    assert np.array_equal(a[0], g["seq_x0_1"]) and np.array_equal(b[1], g["seq_dw_2"])


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "sampler_*.npz"))))
def test_product_host_sampler_matches_reference_outputs(path):
    """The product's host samplers are the same stream (drop-in inputs)."""
    from deeppde_actorcritic_amd import equation as peq
    g = np.load(path)
    eq = peq.LQR(eqn_config("LQR", int(g["dim"]), R=float(g["R"])))
    B, N, seed = int(g["num_sample"]), int(g["N"]), int(g["seed"])
    for name in ("sample_normal", "sample_bounded", "sample0"):
        np.random.seed(seed)
        x0, dw, xb = getattr(eq, name)(B, N)
        assert np.array_equal(x0, g[f"{name}_x0"]) and np.array_equal(dw, g[f"{name}_dw"])
        assert np.array_equal(xb, g[f"{name}_x_bdry"])


def test_bounded_increments_distribution():
    """equation.py:31-32: values {-sqrt3, 0, sqrt3} with probabilities {1/6, 2/3, 1/6}."""
    g = np.load(os.path.join(GOLD, "sampler_d20_s2024.npz"))
    v = g["sample_bounded_dw"]
    assert set(np.unique(v)).issubset({-np.sqrt(3.0), 0.0, np.sqrt(3.0)})
    eq = oeq.LQR(eqn_config("LQR", 20))
    np.random.seed(3)
    _, dw, _ = eq.sample_bounded(2000, 10)
    p = [np.mean(dw == -np.sqrt(3.0)), np.mean(dw == 0), np.mean(dw == np.sqrt(3.0))]
    assert abs(p[0] - 1 / 6) < 0.01 and abs(p[1] - 2 / 3) < 0.01 and abs(p[2] - 1 / 6) < 0.01


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "rollout_*.npz"))))
def test_oracle_rollout_regression(path):
    g = np.load(path)
    cfg = eqn_config(str(g["eqn"]), int(g["dim"]), int(g["control_dim"]), float(g["T"]), int(g["N"]))
    eq = oeq.make(cfg)
    B, N, T = g["x0"].shape[0], int(g["N"]), float(g["T"])
    prop = eq.propagate_naive if str(g["scheme"]) == "naive" else eq.propagate_adaptive
    x, dt, coef = prop(B, g["x0"], g["dw"], None, False, T, N, True)
    np.testing.assert_array_equal(coef.numpy(), g["coef"])
    np.testing.assert_allclose(x.numpy(), g["x"], rtol=0, atol=1e-14)
    np.testing.assert_allclose(dt.numpy(), g["dt"], rtol=0, atol=1e-16)


def test_lqr_riccati_constant_kat():
    """equation.py:151: k = (sqrt(g^2 q^2 + 4 p q b^2) - q g) / b^2 / 2 = golden ratio - 1 at p=q=b=g=1."""
    eq = oeq.LQR(eqn_config("LQR", 20))
    assert abs(eq.k - 0.6180339887498949) < 1e-15
    eqv = oeq.LQR_var(eqn_config("LQR_var", 20))
    assert abs(eqv.k - (np.sqrt(5) - 1) / 2) < 1e-16


@pytest.mark.parametrize("name,d", [("LQR", 5), ("VDP", 4), ("EKN", 5), ("LQR_var", 5)])
def test_analytic_gradient_consistency(name, d):
    """V_grad_true is the gradient of V_true (equation.py: V_true / V_grad_true pairs)."""
    eq = oeq.make(eqn_config(name, d))
    torch.manual_seed(0)
    x = (torch.rand(16, d, dtype=torch.float64) - 0.5).requires_grad_(True)
    (g,) = torch.autograd.grad(eq.V_true(x).sum(), x)
    np.testing.assert_allclose(g.detach().numpy(), eq.V_grad_true(x).detach().numpy(), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("name,d", [("LQR", 5), ("VDP", 4), ("LQR_var", 5)])
def test_hjb_residual_vanishes_for_analytic_solution(name, d):
    """The analytic pair solves the HJB: w(x,u*) + <drift(x,u*), grad V> + tr(sigma sigma^T Hess V)/2 - gamma V = 0.
    Checked with autograd Hessians on random interior points (pins the coefficient functions)."""
    eq = oeq.make(eqn_config(name, d))
    torch.manual_seed(1)
    x = (torch.rand(8, d, dtype=torch.float64) - 0.5) * 0.8
    res = []
    for i in range(x.shape[0]):
        xi = x[i:i + 1].clone().requires_grad_(True)
        V = eq.V_true(xi)
        (gV,) = torch.autograd.grad(V.sum(), xi, create_graph=True)
        H = torch.stack([torch.autograd.grad(gV[0, j], xi, retain_graph=True)[0][0] for j in range(d)])
        u = eq.u_true(xi)
        s = eq.sigma(xi, u, 1)[0]
        val = (eq.w_tf(xi, u)[0, 0] + (eq.drift(xi, u) * gV).sum() + 0.5 * torch.trace(s @ s.T @ H)
               - eq.gamma * V[0, 0])
        res.append(float(val.detach()))
    assert np.max(np.abs(res)) < 1e-10, res


def test_adaptive_invariants():
    """SURVEY §4 invariants: recorded states stay inside the ball, coef in {0,1} non-increasing,
    adaptive dt >= 1e-4 * dt0."""
    cfg = eqn_config("LQR", 20, T=0.2, N=50)
    eq = oeq.LQR(cfg)
    np.random.seed(11)
    x0, dw, _ = eq.sample_normal(64, 50)
    x, dt, coef = eq.propagate_adaptive(64, x0, dw, None, False, 0.2, 50, True)
    assert torch.all(torch.sqrt(torch.sum(x ** 2, 1)) < 1.0)
    c = coef.numpy()
    assert set(np.unique(c)).issubset({0.0, 1.0})
    assert np.all(np.diff(c, axis=1) <= 0)
    assert np.all(dt.numpy() >= 0.2 / 50 * 1e-4 * (1 - 1e-12))
