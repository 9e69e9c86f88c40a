"""GPU parity: every libdpac kernel against the oracle (tests run through the C ABI).

Tolerances (stated per test):
  * float64 kernels vs the float64 oracle: |a-b| <= 1e-12 * (1 + |b|) elementwise, coef exact;
  * float32 kernels vs the float64 oracle: at most 0.1 % of trajectories may take a
    different exit decision (|x| = R flips); on the others
    |a-b| <= 2e-5 * (1 + |b|) for states and 1e-4 relative for accumulated costs.
"""
import glob
import os

import numpy as np
import pytest
import torch

from deeppde_actorcritic_amd import _lib, ops
from deeppde_actorcritic_amd import equation as peq
from oracle import equations as oeq
from tests.helpers import eqn_config, rel_close

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"
CASES = [("LQR", 5), ("LQR", 20), ("VDP", 4), ("VDP", 20), ("EKN", 5), ("EKN", 20), ("LQR_var", 5),
         ("LQR_var", 20)]
SCHEMES = {"naive": _lib.SCHEME_NAIVE, "adaptive": _lib.SCHEME_ADAPTIVE}


def pe(cfg):
    return getattr(peq, cfg.eqn_name)(cfg)


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.asarray(a), dtype=dtype, device=DEV)


def native_dw(dw, dtype=torch.float64):
    return dev(dw, dtype).permute(2, 0, 1).contiguous()


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "rollout_*.npz"))))
def test_rollout_matches_golden_fp64(path):
    g = np.load(path)
    cfg = eqn_config(str(g["eqn"]), int(g["dim"]), int(g["control_dim"]), float(g["T"]), int(g["N"]))
    eqp = pe(cfg).params()
    sch = SCHEMES[str(g["scheme"])]
    x0, dw = dev(g["x0"]), native_dw(g["dw"])
    N, T = int(g["N"]), float(g["T"])
    for order, key in ((_lib.COST_CRITIC, "y_critic"), (_lib.COST_ACTOR, "y_actor")):
        x, dt, coef, u, y, disc = ops.rollout_analytic(eqp, sch, x0, dw, T, N, want_u=True, cost_order=order)
        np.testing.assert_array_equal(coef.cpu().numpy(), g["coef"])
        assert rel_close(x.permute(1, 2, 0).cpu(), g["x"], 1e-12)
        assert rel_close(dt.cpu(), g["dt"], 1e-12)
        assert rel_close(y.cpu(), g[key], 1e-12)
        assert rel_close(disc.cpu(), g["disc"], 1e-12)


@pytest.mark.parametrize("name,d", CASES)
@pytest.mark.parametrize("scheme", ["naive", "adaptive"])
@pytest.mark.parametrize("sample", ["normal", "bounded"])
def test_rollout_vs_oracle_fp64(name, d, scheme, sample):
    B, N, T = 200, 40, 0.2
    cfg = eqn_config(name, d, T=T, N=N)
    eo, ep = oeq.make(cfg), pe(cfg)
    np.random.seed(hash((name, d, scheme, sample)) % 2 ** 31)
    x0, dw, _ = (eo.sample_normal if sample == "normal" else eo.sample_bounded)(B, N)
    prop = eo.propagate_naive if scheme == "naive" else eo.propagate_adaptive
    xr, dtr, cr = prop(B, x0, dw, None, False, T, N, True)
    x, dt, coef, u, y, disc = ops.rollout_analytic(ep.params(), SCHEMES[scheme], dev(x0), native_dw(dw), T, N,
                                                   want_u=True, cost_order=_lib.COST_CRITIC)
    np.testing.assert_array_equal(coef.cpu().numpy(), cr.numpy())
    assert rel_close(x.permute(1, 2, 0).cpu(), xr, 1e-12)
    assert rel_close(dt.cpu(), dtr, 1e-12)
    ur = torch.stack([eo.u_true(xr[:, :, t]) for t in range(N)])
    assert rel_close(u.cpu(), ur, 1e-12)


@pytest.mark.parametrize("name,d", [("LQR", 20), ("EKN", 20), ("LQR_var", 20), ("VDP", 20)])
@pytest.mark.parametrize("scheme", ["naive", "adaptive"])
def test_rollout_fp32_within_tolerance(name, d, scheme):
    B, N, T = 4096, 100, 0.2
    cfg = eqn_config(name, d, T=T, N=N)
    eo, ep = oeq.make(cfg), pe(cfg)
    np.random.seed(5)
    x0, dw, _ = eo.sample_normal(B, N)
    prop = eo.propagate_naive if scheme == "naive" else eo.propagate_adaptive
    xr, dtr, cr = prop(B, x0, dw, None, False, T, N, True)
    x, dt, coef, _, y, disc = ops.rollout_analytic(ep.params(), SCHEMES[scheme], dev(x0, torch.float32),
                                                   native_dw(dw, torch.float32), T, N,
                                                   cost_order=_lib.COST_ACTOR)
    c = coef.cpu().numpy()
    same = np.all(c == cr.numpy(), axis=1)
    assert np.mean(~same) <= 1e-3, f"{np.mean(~same):.2e} of trajectories flipped an exit decision"
    xm = x.permute(1, 2, 0).cpu().double().numpy()[same]
    assert rel_close(xm, xr.numpy()[same], 2e-5)
    assert rel_close(dt.cpu().double().numpy()[same], dtr.numpy()[same], 2e-5)


@pytest.mark.parametrize("name,d", CASES)
def test_equation_eval_vs_oracle(name, d):
    cfg = eqn_config(name, d)
    eo, ep = oeq.make(cfg), pe(cfg)
    torch.manual_seed(3)
    B = 300
    x = (torch.rand(B, d, dtype=torch.float64) - 0.5) * 1.2
    u = torch.randn(B, cfg.control_dim, dtype=torch.float64)
    xd, ud = x.to(DEV), u.to(DEV)
    eqp = ep.params()
    checks = {
        _lib.EVAL_DRIFT: eo.drift(x, u),
        _lib.EVAL_SIGMA: torch.diagonal(eo.sigma(x, u, B), dim1=1, dim2=2),
        _lib.EVAL_W: eo.w_tf(x, u)[:, 0],
        _lib.EVAL_Z: eo.Z_tf(x)[:, 0],
        _lib.EVAL_V_TRUE: eo.V_true(x)[:, 0],
        _lib.EVAL_U_TRUE: eo.u_true(x),
        _lib.EVAL_V_GRAD: eo.V_grad_true(x),
        _lib.EVAL_B: eo.b_tf(x)[:, 0],
    }
    for what, ref in checks.items():
        out = ops.equation_eval(eqp, what, xd, ud)
        assert rel_close(out.cpu(), ref, 1e-12), what


@pytest.mark.parametrize("name,d", CASES)
@pytest.mark.parametrize("td", ["TD1", "TD2"])
@pytest.mark.parametrize("scheme", ["naive", "adaptive"])
def test_td_assemble_fwd_bwd_vs_oracle(name, d, td, scheme):
    """CriticModel loop (solver.py:166-187) with a given G; dy/dG vs autograd."""
    B, N, T = 64, 20, 0.2
    cfg = eqn_config(name, d, T=T, N=N)
    eo, ep = oeq.make(cfg), pe(cfg)
    np.random.seed(17)
    x0, dw, _ = eo.sample_normal(B, N)
    prop = eo.propagate_naive if scheme == "naive" else eo.propagate_adaptive
    xr, dtr, cr = prop(B, x0, dw, None, False, T, N, True)
    torch.manual_seed(0)
    U = torch.randn(N, B, cfg.control_dim, dtype=torch.float64) * 0.3  # an arbitrary control record
    G = (torch.randn(N, B, d, dtype=torch.float64)).requires_grad_(True)
    dwt = torch.as_tensor(dw)
    y, disc = 0, 1
    for t in range(N):
        xt = xr[:, :, t]
        w = eo.w_tf(xt, U[t])
        y = y + (w * disc) * (cr[:, t:t + 1] * dtr[:, t:t + 1])
        if td == "TD1":
            dd = torch.einsum("bij,bj->bi", eo.sigma(xt, U[t], B), dwt[:, :, t])
            dd = torch.sum(dd * G[t], 1, keepdim=True) * disc
            y = y - dd * (cr[:, t:t + 1] * torch.sqrt(dtr[:, t:t + 1]))
        disc = disc * torch.exp(-cfg.discount * dtr[:, t:t + 1] * cr[:, t:t + 1])
    gy = torch.randn(B, 1, dtype=torch.float64)
    if td == "TD1":
        (gG_ref,) = torch.autograd.grad(y, G, gy)
    Gd = G.detach().to(DEV).requires_grad_(True)
    tdt = _lib.TD1 if td == "TD1" else _lib.TD2
    yp, discp = ops.td_assemble(ep.params(), tdt, xr.permute(2, 0, 1).contiguous().to(DEV), U.to(DEV),
                                native_dw(dw), dtr.contiguous().to(DEV), cr.contiguous().to(DEV),
                                Gd if td == "TD1" else None)
    assert rel_close(yp.detach().cpu(), y.detach()[:, 0], 1e-12)
    assert rel_close(discp.cpu(), disc[:, 0], 1e-12)
    if td == "TD1":
        (gG,) = torch.autograd.grad(yp, Gd, gy[:, 0].to(DEV))
        assert rel_close(gG.cpu(), gG_ref, 1e-12)


def test_actor_cost_alias():
    cfg = eqn_config("LQR", 20, T=0.2, N=30)
    eo, ep = oeq.make(cfg), pe(cfg)
    np.random.seed(2)
    x0, dw, _ = eo.sample_normal(128, 30)
    eqp = ep.params()
    x, dt, coef, u, y, disc = ops.rollout_analytic(eqp, 1, dev(x0), native_dw(dw), 0.2, 30, want_u=True,
                                                   cost_order=_lib.COST_ACTOR)
    y2, disc2 = ops.actor_cost(eqp, x, u, dt, coef)
    # same sums; the TD kernel combines 4 horizon chunks, so only rounding differs
    assert rel_close(y2.cpu(), y.cpu(), 1e-13) and rel_close(disc2.cpu(), disc.cpu(), 1e-13)


# ---- sampler -------------------------------------------------------------------
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_sampler_distribution_and_sharding(dtype):
    cfg = eqn_config("LQR", 20)
    eqp = pe(cfg).params()
    B, N = 8192, 50
    x0, dw, xb = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=42, dtype=dtype, device=DEV)
    dwc = dw.double().cpu()
    assert abs(float(dwc.mean())) < 3e-3 and abs(float(dwc.var()) - 1) < 3e-3
    r = torch.linalg.norm(x0.double(), dim=1).cpu().numpy()
    assert np.all(r < 1.0)
    # P(|x0| <= s) = s^d for the uniform-in-ball law (equation.py:14-18)
    for s in (0.8, 0.9, 0.95):
        assert abs(np.mean(r <= s) - s ** 20) < 0.02
    assert torch.allclose(torch.linalg.norm(xb.double(), dim=1), torch.ones(B, dtype=torch.float64, device=DEV),
                          atol=1e-6 if dtype == torch.float32 else 1e-14)
    # keyed by global trajectory index: a shard reproduces its slice of the full batch exactly
    x0s, dws, xbs = ops.sample(eqp, _lib.SAMPLE_NORMAL, 1000, N, seed=42, traj_offset=3000, dtype=dtype, device=DEV)
    assert torch.equal(x0s, x0[3000:4000]) and torch.equal(dws, dw[:, 3000:4000]) and torch.equal(xbs, xb[3000:4000])
    _, dwb, _ = ops.sample(eqp, _lib.SAMPLE_BOUNDED, B, N, seed=7, dtype=dtype, device=DEV)
    v = dwb.double().cpu().numpy()
    s3 = float(torch.tensor(3.0, dtype=dtype).sqrt())
    assert set(np.unique(v)).issubset({-s3, 0.0, s3})
    assert abs(np.mean(v == 0) - 2 / 3) < 5e-3 and abs(np.mean(v > 0) - 1 / 6) < 5e-3
    x00, _, _ = ops.sample(eqp, _lib.SAMPLE_ZERO_X0, 16, N, seed=1, dtype=dtype, device=DEV)
    assert torch.all(x00 == torch.tensor(0.01, dtype=dtype))


def test_sampler_into_a_view_that_is_not_8_byte_aligned():
    """Round 6: the f32 sampler writes a step's two components of a lane slot as one 8-byte store
    when dw is 8-byte aligned; a caller's view starting at an odd float (legal for the C ABI) takes
    the scalar stores and gets the same numbers."""
    eqp = pe(eqn_config("LQR", 20)).params()
    B, N, d = 300, 7, 20
    x0, dw, xb = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=3, traj_offset=11, device=DEV)
    buf = torch.zeros(N * B * d + 1, device=DEV)
    dw_odd = buf[1:].view(N, B, d)
    assert dw_odd.data_ptr() % 8 == 4
    out = (torch.empty_like(x0), dw_odd, torch.empty_like(xb))
    ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=3, traj_offset=11, device=DEV, out=out)
    assert torch.equal(dw_odd, dw) and torch.equal(out[0], x0) and torch.equal(out[2], xb)
    assert float(buf[0]) == 0.0  # nothing written before the view


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("d", [1, 3, 5, 20, 33, 200])
@pytest.mark.parametrize("sample_type", [_lib.SAMPLE_NORMAL, _lib.SAMPLE_ZERO_X0])
def test_grouped_point_sampler_equals_one_thread_per_trajectory(d, dtype, sample_type):
    """Round 6: x0 and x_bdry drawn by one lane group per (trajectory, point), the squares folded
    in component order through shuffles, equal bit for bit the one-thread-per-trajectory kernel
    (DPAC_SAMPLE_POINTS_SERIAL=1; the path directions of more than 64 counter blocks take), for
    dimensions that leave partial blocks and idle lanes in the group."""
    eqp = pe(eqn_config("LQR", 20)).params()
    eqp.dim = d
    out = {}
    old = os.environ.get("DPAC_SAMPLE_POINTS_SERIAL")
    try:
        for k in ("0", "1"):
            os.environ["DPAC_SAMPLE_POINTS_SERIAL"] = k
            out[k] = ops.sample(eqp, sample_type, 1001, 1, seed=19, traj_offset=7, dtype=dtype, device=DEV,
                                want_dw=False)
    finally:
        if old is None:
            os.environ.pop("DPAC_SAMPLE_POINTS_SERIAL", None)
        else:
            os.environ["DPAC_SAMPLE_POINTS_SERIAL"] = old
    for a, b in zip(out["0"], out["1"]):
        if a is not None:
            assert torch.equal(a, b)
    nb = torch.linalg.norm(out["0"][2].double(), dim=1)
    assert torch.allclose(nb, torch.full_like(nb, float(eqp.R)), rtol=1e-5 if dtype == torch.float32 else 1e-13)


@pytest.mark.parametrize("N", [64, 63])
@pytest.mark.parametrize("name,d", [("LQR", 20), ("LQR", 5), ("VDP", 20), ("EKN", 10)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("sample_type", [_lib.SAMPLE_NORMAL, _lib.SAMPLE_BOUNDED])
def test_inkernel_philox_equals_sampled_dw(name, d, dtype, sample_type, N):
    """dw=None draws the same numbers in-kernel as dpac_sample writes to HBM (round 6: the paired
    layout, one counter block per lane slot and step pair, with an odd horizon's unpaired last
    step; the TD kernel's horizon chunks start at odd steps too)."""
    cfg = eqn_config(name, d, N=N)
    eqp = pe(cfg).params()
    B = 1000
    x0, dw, _ = ops.sample(eqp, sample_type, B, N, seed=9, traj_offset=123, dtype=dtype, device=DEV)
    a = ops.rollout_analytic(eqp, 1, x0, dw, 0.2, N, cost_order=_lib.COST_ACTOR)
    b = ops.rollout_analytic(eqp, 1, x0, None, 0.2, N, seed=9, traj_offset=123, sample_type=sample_type,
                             cost_order=_lib.COST_ACTOR)
    for ta, tb in zip(a, b):
        if ta is not None:
            assert torch.equal(ta, tb)
    # TD1 regenerates the same increments too
    xx, dt, coef, _, _, _ = a
    u = torch.zeros(N, B, cfg.control_dim, dtype=dtype, device=DEV)
    G = torch.randn(N, B, d, dtype=dtype, device=DEV)
    y1, _ = ops.td_assemble(eqp, _lib.TD1, xx, u, dw, dt, coef, G)
    y2, _ = ops.td_assemble(eqp, _lib.TD1, xx, u, None, dt, coef, G, seed=9, traj_offset=123,
                            sample_type=sample_type)
    assert torch.equal(y1, y2)


# ---- full-size properties (BASELINE synthetic shape: B=4096, d=20, N=200) -------------
@pytest.mark.parametrize("scheme", ["naive", "adaptive"])
def test_full_size_invariants_and_sharding(scheme):
    cfg = eqn_config("LQR", 20, T=0.2, N=200)
    eqp = pe(cfg).params()
    B, N = 4096, 200
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=1234, device=DEV)
    x, dt, coef, _, y, disc = ops.rollout_analytic(eqp, SCHEMES[scheme], x0, dw, 0.2, N,
                                                   cost_order=_lib.COST_ACTOR)
    # every recorded state strictly inside the ball; coef in {0,1}, non-increasing in t
    assert float(torch.linalg.norm(x, dim=2).max()) < 1.0
    assert set(torch.unique(coef).tolist()).issubset({0.0, 1.0})
    assert bool(torch.all(coef[:, 1:] <= coef[:, :-1]))
    # frozen after exit: x_{t+1} == x_t wherever coef_t == 0
    frozen = (coef == 0).t()  # [N, B] like x[1:]
    assert torch.equal(x[1:][frozen], x[:-1][frozen])
    dt0 = 0.2 / N
    if scheme == "naive":
        assert bool(torch.all(dt == torch.tensor(dt0, dtype=dt.dtype)))
    else:
        assert float(dt.min()) >= dt0 * 1e-4 * (1 - 1e-6) and float(dt.max()) <= dt0 * (1 + 1e-6)
    # discount consistent with sum of coef*dt: disc = prod exp(-g dt coef)
    ref = torch.exp(-(dt.double() * coef.double()).sum(1))
    assert torch.allclose(disc.double(), ref, rtol=1e-5)
    # sharding: rows of a half batch rolled out alone are bit-identical
    h = B // 2
    xs, dts, cs, _, ys, ds = ops.rollout_analytic(eqp, SCHEMES[scheme], x0[h:].contiguous(), dw[:, h:].contiguous(),
                                                  0.2, N, cost_order=_lib.COST_ACTOR)
    assert torch.equal(xs, x[:, h:]) and torch.equal(cs, coef[h:]) and torch.equal(ys, y[h:])


def test_odd_batch_sizes():
    """Batches that do not fill the last wavefront (B % 16 != 0) and B = 1."""
    cfg = eqn_config("LQR", 20, T=0.2, N=12)
    eo, ep = oeq.make(cfg), pe(cfg)
    for B in (1, 3, 17, 33):
        np.random.seed(B)
        if B == 1:  # the reference sampler cannot draw B = 1 (scipy squeezes size-1 axes, quirk 9)
            x0 = np.random.uniform(-0.2, 0.2, size=(1, 20))
            dw = np.random.standard_normal((1, 20, 12))
        else:
            x0, dw, _ = eo.sample_normal(B, 12)
        xr, dtr, cr = eo.propagate_adaptive(B, x0, dw, None, False, 0.2, 12, True)
        x, dt, coef, *_ = ops.rollout_analytic(ep.params(), 1, dev(x0), native_dw(dw), 0.2, 12)
        np.testing.assert_array_equal(coef.cpu().numpy(), cr.numpy())
        assert rel_close(x.permute(1, 2, 0).cpu(), xr, 1e-12)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("scheme", ["adaptive", "naive"])
@pytest.mark.parametrize("name,d,B,N", [("LQR", 20, 300, 200), ("LQR", 5, 37, 13), ("EKN", 20, 65, 7),
                                        ("LQR_var", 10, 33, 101), ("LQR", 4, 1, 40), ("VDP", 20, 70, 30)])
def test_staged_rollout_bitwise(name, d, B, N, scheme, dtype):
    """k_rollout_staged (dw copied into an LDS ring by a loader wavefront, the compute
    wavefronts only store) gives bitwise the results of k_rollout, which loads dw itself:
    full and partial hand-off chunks, partial workgroups, the u and cost outputs, both
    dtypes (VDP's one-lane groups always take k_rollout)."""
    cfg = eqn_config(name, d, T=0.2, N=N)
    eqp = pe(cfg).params()
    sch = SCHEMES[scheme]
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=3, dtype=dtype, device=DEV)
    out = {}
    old = os.environ.get("DPAC_ROLLOUT_STAGED")
    try:
        for k in ("0", "1"):
            os.environ["DPAC_ROLLOUT_STAGED"] = k
            out[k] = [ops.rollout_analytic(eqp, sch, x0, dw, 0.2, N, want_u=wu, cost_order=co)
                      for wu, co in ((False, None), (True, _lib.COST_ACTOR))]
    finally:
        if old is None:
            os.environ.pop("DPAC_ROLLOUT_STAGED", None)
        else:
            os.environ["DPAC_ROLLOUT_STAGED"] = old
    for a, b in zip(out["0"], out["1"]):
        for s, t in zip(a, b):
            assert (s is None) == (t is None)
            if s is not None:
                assert torch.equal(s, t)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("sample_type", [_lib.SAMPLE_NORMAL, _lib.SAMPLE_BOUNDED])
def test_sampler_stream_is_a_function_of_step_and_component(dtype, sample_type):
    """The dw stream depends only on (seed, global trajectory, step, component): a shorter
    horizon (odd or even) draws the leading steps of a longer one bit for bit, and a shard keeps
    its rows (the paired layout keeps both properties)."""
    eqp = pe(eqn_config("LQR", 20)).params()
    B = 777
    _, dw, _ = ops.sample(eqp, sample_type, B, 50, seed=5, dtype=dtype, device=DEV)
    for n in (1, 2, 7, 49):
        _, dws, _ = ops.sample(eqp, sample_type, B, n, seed=5, dtype=dtype, device=DEV)
        assert torch.equal(dws, dw[:n])
    _, dwo, _ = ops.sample(eqp, sample_type, 100, 49, seed=5, traj_offset=300, dtype=dtype, device=DEV)
    assert torch.equal(dwo, dw[:49, 300:400])
    # consecutive steps are independent draws, not copies (the two halves of a block)
    c = float(torch.corrcoef(torch.stack([dw[0::2].double().reshape(-1)[:100000],
                                          dw[1::2].double().reshape(-1)[:100000]]))[0, 1])
    assert abs(c) < 0.02, c


@pytest.mark.parametrize("sample_type", [_lib.SAMPLE_NORMAL, _lib.SAMPLE_BOUNDED])
@pytest.mark.parametrize("scheme", ["adaptive", "naive"])
@pytest.mark.parametrize("name,d,B,N", [("LQR", 20, 4096, 200), ("LQR", 20, 300, 37), ("EKN", 20, 65, 16),
                                        ("LQR_var", 10, 33, 101), ("LQR", 5, 37, 13), ("VDP", 20, 70, 30)])
def test_inkernel_philox_generator_rollout_bitwise(name, d, B, N, scheme, sample_type):
    """Round 6: the in-kernel Philox rollout with the increments drawn by
    generator wavefronts into the staged kernel's LDS ring (k_rollout_staged<..., GEN = 12>, the
    default for float) gives bitwise the results of k_rollout drawing them in each compute lane
    (DPAC_ROLLOUT_STAGED=0): odd horizons (a last unpaired step), partial workgroups, chunks that
    wrap the ring, the u and cost outputs (VDP and float64 keep k_rollout)."""
    cfg = eqn_config(name, d, T=0.2, N=N)
    eqp = pe(cfg).params()
    sch = SCHEMES[scheme]
    x0, _, _ = ops.sample(eqp, sample_type, B, N, seed=11, traj_offset=5, device=DEV)
    out = {}
    old = os.environ.get("DPAC_ROLLOUT_STAGED")
    try:
        for k in ("0", "1"):
            os.environ["DPAC_ROLLOUT_STAGED"] = k
            out[k] = [ops.rollout_analytic(eqp, sch, x0, None, 0.2, N, seed=11, traj_offset=5, sample_type=sample_type,
                                           want_u=wu, cost_order=co)
                      for wu, co in ((False, None), (True, _lib.COST_ACTOR))]
    finally:
        if old is None:
            os.environ.pop("DPAC_ROLLOUT_STAGED", None)
        else:
            os.environ["DPAC_ROLLOUT_STAGED"] = old
    for ra, rb in zip(out["0"], out["1"]):
        for ta, tb in zip(ra, rb):
            if ta is not None:
                assert torch.equal(ta, tb)
