"""The fused NN-control rollout (dpac_rollout_nn_fwd: actor MLP on MFMA tiles inside
the time loop, equation.py:46-106 + solver.py:260-278) against

  * the float64 oracle's propagate_* with the oracle DeepNN as NN_control,
  * the product's unfused path (PyTorch MLP between dpac_step_fwd launches),
  * PyTorch's own layer outputs for the backward saves.

Tolerances: float64 |a-b| <= 1e-10 (1+|b|) on x, dt, u (the MFMA and the GEMM
library sum the 200-term dot products in different orders; ~1e-16 per step),
coef exact; float32 vs the float64 oracle: <= 1e-3 of trajectories may flip an
exit decision, matched trajectories within 1e-4 (1+|b|).
"""
import ctypes

import numpy as np
import pytest
import torch

from deeppde_actorcritic_amd import _lib, ops
from deeppde_actorcritic_amd import equation as peq
from deeppde_actorcritic_amd import solver as psol
from deeppde_actorcritic_amd.config import set_floatx
from oracle import equations as oeq
from oracle import solver as osol
from tests.helpers import full_config, rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
SCHEMES = {"naive": _lib.SCHEME_NAIVE, "adaptive": _lib.SCHEME_ADAPTIVE}


def actor_pair(cfg, dtype):
    """Product actor DeepNN (on the GPU, `dtype`) and the oracle DeepNN with the same weights."""
    set_floatx("float64" if dtype == torch.float64 else "float32")
    gen = torch.Generator().manual_seed(3)
    net = psol.DeepNN(cfg, "actor", gen, dtype, DEV)
    onet = osol.DeepNN(cfg, "actor", net.export_params())
    return net, onet


CASES = [("LQR", 20, (200, 200, 200)), ("LQR", 5, (16, 16)), ("VDP", 4, (50, 50)),
         ("VDP", 10, (32, 48, 24)), ("EKN", 5, (40, 40)), ("EKN", 20, (64, 64, 64)),
         ("LQR_var", 10, (200, 200, 200)), ("LQR_var", 5, (24,))]


@pytest.mark.parametrize("name,d,hidden", CASES)
@pytest.mark.parametrize("scheme", ["naive", "adaptive"])
def test_fused_nn_rollout_vs_oracle_fp64(name, d, hidden, scheme):
    B, N, T = 37, 20, 0.2  # 37: a partial last 16-row tile
    cfg = full_config(name, d, N=N, hidden=hidden, scheme=scheme)
    eo = oeq.make(cfg.eqn_config)
    ep = getattr(peq, name)(cfg.eqn_config)
    net, onet = actor_pair(cfg, torch.float64)
    np.random.seed(11)
    x0, dw, _ = eo.sample_normal(B, N)
    prop = eo.propagate_naive if scheme == "naive" else eo.propagate_adaptive
    xr, dtr, cr = prop(B, x0, dw, onet, False, T, N, False)
    x, dt, coef, u, _, _, _ = ops.rollout_nn(
        ep.params(), SCHEMES[scheme], torch.as_tensor(x0, device=DEV),
        torch.as_tensor(dw, device=DEV).permute(2, 0, 1).contiguous(), T, N, net.mlp_view())
    np.testing.assert_array_equal(coef.cpu().numpy(), cr.numpy())
    assert rel_close(x.permute(1, 2, 0).cpu(), xr, 1e-10)
    assert rel_close(dt.cpu(), dtr, 1e-10)
    # the control the kernel applied is the oracle MLP at the recorded states
    ur = torch.stack([onet(xr[:, :, t], False, need_grad=False) for t in range(N)])
    assert rel_close(u.cpu(), ur, 1e-10)


@pytest.mark.parametrize("name,d,hidden", [("LQR", 20, (200, 200, 200)), ("EKN", 20, (64, 64, 64)),
                                           ("VDP", 20, (200, 200, 200))])
def test_fused_nn_rollout_fp32_vs_oracle(name, d, hidden):
    B, N, T = 512, 50, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme="adaptive", dtype="float32")
    eo = oeq.make(cfg.eqn_config)
    ep = getattr(peq, name)(cfg.eqn_config)
    net, onet = actor_pair(cfg, torch.float32)
    np.random.seed(12)
    x0, dw, _ = eo.sample_normal(B, N)
    xr, dtr, cr = eo.propagate_adaptive(B, x0, dw, onet, False, T, N, False)
    x, dt, coef, _, _, _, _ = ops.rollout_nn(
        ep.params(), _lib.SCHEME_ADAPTIVE, torch.as_tensor(x0, dtype=torch.float32, device=DEV),
        torch.as_tensor(dw, dtype=torch.float32, device=DEV).permute(2, 0, 1).contiguous(), T, N,
        net.mlp_view())
    same = np.all(coef.cpu().numpy() == cr.numpy(), axis=1)
    assert np.mean(~same) <= 1e-3
    assert rel_close(x.permute(1, 2, 0).cpu().double().numpy()[same], xr.numpy()[same], 1e-4)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_fused_matches_unfused_product_path(dtype):
    """dpac_rollout_nn_fwd vs PyTorch MLP + dpac_step_fwd per step (rollout_nn_nograd)."""
    name, d, B, N, T = "LQR", 20, 300, 40, 0.2
    cfg = full_config(name, d, N=N, hidden=(200, 200, 200), scheme="adaptive")
    ep = peq.LQR(cfg.eqn_config)
    net, _ = actor_pair(cfg, dtype)
    eqp = ep.params()
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=5, dtype=dtype, device=DEV)
    xa, dta, ca, ua, _, _, _ = ops.rollout_nn(eqp, _lib.SCHEME_ADAPTIVE, x0, dw, T, N, net.mlp_view())
    with torch.no_grad():
        xb, dtb, cb, ub = peq.rollout_nn_nograd(eqp, _lib.SCHEME_ADAPTIVE, x0, dw, T, N, net)
    tol = 1e-10 if dtype == torch.float64 else 2e-4
    same = torch.all(ca == cb, dim=1).cpu().numpy()
    assert np.mean(~same) <= (0 if dtype == torch.float64 else 1e-2)
    assert rel_close(xa[:, same].cpu(), xb[:, same].cpu(), tol)
    assert rel_close(ua[:, same].cpu(), ub[:, same].cpu(), tol)


def test_backward_saves_and_cost():
    """save_z holds every dense layer's pre-BN output; save_flag / save_disc the state
    entering each step; y / disc equal the actor-cost kernel over the same path."""
    name, d, B, N, T = "LQR", 5, 40, 12, 0.2
    hidden = (24, 40)
    cfg = full_config(name, d, N=N, hidden=hidden, scheme="adaptive")
    ep = peq.LQR(cfg.eqn_config)
    net, _ = actor_pair(cfg, torch.float64)
    eqp = ep.params()
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=6, dtype=torch.float64, device=DEV)
    x, dt, coef, u, y, disc, (z, flag, disc_t, mask) = ops.rollout_nn(
        eqp, _lib.SCHEME_ADAPTIVE, x0, dw, T, N, net.mlp_view(), cost_order=_lib.COST_ACTOR, save=True)
    assert mask is None  # sign-bit masks are a float 16-row fast-path product
    # pre-BN layer outputs, recomputed with PyTorch from the recorded states
    rs, g, bt, W = net.bn_rs, net.bn_gamma, net.bn_beta, net.W
    with torch.no_grad():
        a = torch.addcmul(bt[0], x[:N].reshape(-1, d), rs * g[0])
        zs = []
        for i in range(len(hidden)):
            zi = a @ W[i]
            zs.append(zi)
            a = torch.addcmul(bt[i + 1], zi, rs * g[i + 1])
            a = a + torch.relu(a)
        zs.append(a @ W[-1])
    assert rel_close(z.reshape(N * B, -1).cpu(), torch.cat(zs, 1).cpu(), 1e-12)
    # flags / discount entering each step
    yr, discr = ops.actor_cost(eqp, x, u, dt, coef)
    assert rel_close(y.cpu(), yr.cpu(), 1e-12) and rel_close(disc.cpu(), discr.cpu(), 1e-12)
    cum = torch.cumprod(torch.exp(-(dt * coef)), 1)  # gamma = 1
    disc_ref = torch.cat([torch.ones(B, 1, dtype=cum.dtype, device=DEV), cum[:, :-1]], 1).t()
    assert rel_close(disc_t.cpu(), disc_ref.cpu(), 1e-12)
    f0 = ops.flag_init(eqp, _lib.SCHEME_ADAPTIVE, x0, T, N)
    assert torch.equal(flag[0], f0)
    alive = (flag > 0).to(coef.dtype)
    assert torch.equal(alive[1:], coef.t()[:-1])  # alive after step t iff step t kept going


def test_invalid_mlp_rejected():
    cfg = full_config("LQR", 5, N=4, hidden=(16, 16))
    ep = peq.LQR(cfg.eqn_config)
    net, _ = actor_pair(cfg, torch.float64)
    eqp = ep.params()
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, 8, 4, seed=1, dtype=torch.float64, device=DEV)
    view = net.mlp_view()
    view.struct.width[1] = 300  # wider than DPAC_MLP_MAX_WIDTH
    with pytest.raises(_lib.DpacError):
        ops.rollout_nn(eqp, _lib.SCHEME_NAIVE, x0, dw, 0.2, 4, view)
    view = net.mlp_view()
    view.struct.ekn_head = 1  # Eikonal head on LQR
    with pytest.raises(_lib.DpacError):
        ops.rollout_nn(eqp, _lib.SCHEME_NAIVE, x0, dw, 0.2, 4, view)
    view = net.mlp_view()
    view.struct.width[0] = 4  # input width != dim
    with pytest.raises(_lib.DpacError):
        ops.rollout_nn(eqp, _lib.SCHEME_NAIVE, x0, dw, 0.2, 4, view)


@pytest.mark.parametrize("name,d,hidden,scheme", [
    ("LQR", 20, (200, 200, 200), "adaptive"), ("LQR", 5, (24, 40), "naive"),
    ("EKN", 5, (40, 40), "adaptive"), ("EKN", 20, (64, 64, 64), "naive"),
    ("VDP", 4, (50, 50), "adaptive"), ("LQR_var", 10, (32, 48, 24), "adaptive")])
def test_fused_bptt_kernel_matches_step_loop(name, d, hidden, scheme):
    """dpac_rollout_nn_bwd (one launch) gives the parameter gradients of the per-step
    reference loop (dpac_step_bwd + PyTorch MLP chain), float64, 1e-10."""
    B, N, T = 37, 12, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme=scheme)
    ep = getattr(peq, name)(cfg.eqn_config)
    net, _ = actor_pair(cfg, torch.float64)
    eqp = ep.params()
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=21, dtype=torch.float64, device=DEV)
    grads = {}
    try:
        for mode in ("loop", "fused"):
            ops.BPTT_MODE = mode
            y, disc, xN = ops.actor_rollout_nn(eqp, SCHEMES[scheme], x0, dw, T, N, net)
            loss = torch.mean(y + disc * torch.sum(xN * xN, 1))  # a smooth terminal value
            grads[mode] = torch.autograd.grad(loss, net.trainable_variables())
    finally:
        ops.BPTT_MODE = "fused"
    for a, b in zip(grads["fused"], grads["loop"]):
        assert rel_close(a.cpu(), b.cpu(), 1e-10)


@pytest.mark.parametrize("name,d,hidden,B", [("LQR", 20, (256, 256, 256, 256), 20), ("EKN", 10, (256, 7), 1),
                                             ("VDP", 20, (4, 256), 16)])
def test_fused_nn_limits_fwd_and_bptt(name, d, hidden, B):
    """Widths at DPAC_MLP_MAX_WIDTH, 4 hidden layers, tiny and odd widths, B = 1: the
    fused forward against the oracle and the fused BPTT against the reference loop."""
    N, T = 8, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme="adaptive")
    eo = oeq.make(cfg.eqn_config)
    ep = getattr(peq, name)(cfg.eqn_config)
    net, onet = actor_pair(cfg, torch.float64)
    np.random.seed(31)
    x0 = np.random.uniform(-0.3, 0.3, size=(B, d))
    dw = np.random.standard_normal((B, d, N))
    xr, dtr, cr = eo.propagate_adaptive(B, x0, dw, onet, False, T, N, False)
    x0t = torch.as_tensor(x0, device=DEV)
    dwt = torch.as_tensor(dw, device=DEV).permute(2, 0, 1).contiguous()
    x, dt, coef, _, _, _, _ = ops.rollout_nn(ep.params(), _lib.SCHEME_ADAPTIVE, x0t, dwt, T, N, net.mlp_view())
    np.testing.assert_array_equal(coef.cpu().numpy(), cr.numpy())
    assert rel_close(x.permute(1, 2, 0).cpu(), xr, 1e-10)
    grads = {}
    try:
        for mode in ("loop", "fused"):
            ops.BPTT_MODE = mode
            y, disc, xN = ops.actor_rollout_nn(ep.params(), _lib.SCHEME_ADAPTIVE, x0t, dwt, T, N, net)
            grads[mode] = torch.autograd.grad(torch.mean(y + disc * torch.sum(xN, 1)), net.trainable_variables())
    finally:
        ops.BPTT_MODE = "fused"
    for a, b in zip(grads["fused"], grads["loop"]):
        assert rel_close(a.cpu(), b.cpu(), 1e-10)


def test_fused_bptt_fp32_ekn():
    """float32 fused BPTT through the Eikonal head vs the float32 reference loop."""
    B, N, T = 64, 20, 0.2
    cfg = full_config("EKN", 20, N=N, hidden=(200, 200, 200), scheme="adaptive", dtype="float32")
    ep = peq.EKN(cfg.eqn_config)
    net, _ = actor_pair(cfg, torch.float32)
    eqp = ep.params()
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=4, dtype=torch.float32, device=DEV)
    grads = {}
    try:
        for mode in ("loop", "fused"):
            ops.BPTT_MODE = mode
            y, disc, xN = ops.actor_rollout_nn(eqp, _lib.SCHEME_ADAPTIVE, x0, dw, T, N, net)
            grads[mode] = torch.autograd.grad(torch.mean(y + disc * torch.sum(xN * xN, 1)),
                                              net.trainable_variables())
    finally:
        ops.BPTT_MODE = "fused"
    for a, b in zip(grads["fused"], grads["loop"]):
        assert rel_close(a.cpu(), b.cpu(), 1e-4)


@pytest.mark.parametrize("name,d,hidden,B", [("LQR", 20, (200, 200, 200), 2048), ("EKN", 20, (64, 64, 64), 37),
                                             ("VDP", 10, (48, 130, 33), 1500), ("LQR_var", 5, (256, 256, 256, 256), 5),
                                             ("LQR", 5, (4, 200), 1030)])
def test_fp32_four_row_kernel_matches_sixteen_row(name, d, hidden, B, monkeypatch):
    """The float rollout on 4x4x1 MFMA blocks (dpac_rollout_nn4.h, default for B <= 1024) against the
    16x16x4 kernel (DPAC_NN_TILE=16) on identical inputs: only the order of the K sums
    differs, so <= 1% of trajectories may flip an exit decision and matched ones agree to
    2e-4 (1+|b|); both RG = 1 (B <= 1024) and RG = 2 workgroups and partial ones."""
    N, T = 30, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme="adaptive", dtype="float32")
    ep = getattr(peq, name)(cfg.eqn_config)
    net, _ = actor_pair(cfg, torch.float32)
    eqp = ep.params()
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=17, dtype=torch.float32, device=DEV)
    out = {}
    for tile in ("4", "16"):
        monkeypatch.setenv("DPAC_NN_TILE", tile)
        out[tile] = ops.rollout_nn(eqp, _lib.SCHEME_ADAPTIVE, x0, dw, T, N, net.mlp_view(),
                                   cost_order=_lib.COST_ACTOR, save=True)
    xa, dta, ca, ua, ya, da, sa = out["4"]
    xb, dtb, cb, ub, yb, db, sb = out["16"]
    same = torch.all(ca == cb, dim=1).cpu().numpy()
    assert np.mean(~same) <= 1e-2
    assert rel_close(xa[:, same].cpu(), xb[:, same].cpu(), 2e-4)
    assert rel_close(ua[:, same].cpu(), ub[:, same].cpu(), 2e-4)
    assert rel_close(ya[same].cpu(), yb[same].cpu(), 2e-4)
    assert rel_close(sa[0][:, same].cpu(), sb[0][:, same].cpu(), 2e-4)  # saved z
    assert torch.equal(sa[1][:, same], sb[1][:, same])                  # saved flags


@pytest.mark.parametrize("name,d,hidden,B", [("LQR", 20, (200, 200, 200), 2048), ("EKN", 10, (48, 130, 33), 300),
                                             ("VDP", 10, (256, 7), 64)])
def test_fp32_kmajor_weights_match_row_major(name, d, hidden, B, monkeypatch):
    """The fused rollout and its BPTT reading the k-major weight images (dpac_mlp.weight_km:
    dwordx4 B loads, permuted K order) against the row-major path on identical inputs
    (16-row tiles both): <= 1% of trajectories may flip an exit decision, matched ones
    agree to 2e-4 (1+|b|); the actor gradients to 2e-3 relative."""
    N, T = 30, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme="adaptive", dtype="float32")
    ep = getattr(peq, name)(cfg.eqn_config)
    net, _ = actor_pair(cfg, torch.float32)
    eqp = ep.params()
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=23, dtype=torch.float32, device=DEV)
    monkeypatch.setenv("DPAC_NN_TILE", "16")
    monkeypatch.setenv("DPAC_NN_X3", "0")  # the f32 kernels (the x3 ones ignore weight_km)
    out, grads = {}, {}
    for km in ("on", "off"):
        monkeypatch.setattr(ops, "WEIGHT_KM", km)
        view = net.mlp_view()
        assert (view.struct.weight_km[0] is not None) == (km == "on")
        out[km] = ops.rollout_nn(eqp, _lib.SCHEME_ADAPTIVE, x0, dw, T, N, view,
                                 cost_order=_lib.COST_ACTOR, save=True)
        y, disc, xN = ops.actor_rollout_nn(eqp, _lib.SCHEME_ADAPTIVE, x0, dw, T, N, net)
        grads[km] = torch.autograd.grad((y + disc).mean() + xN.sum() * 1e-3, net.trainable_variables())
    xa, _, ca, ua, ya, _, sa = out["on"]
    xb, _, cb, ub, yb, _, sb = out["off"]
    same = torch.all(ca == cb, dim=1).cpu().numpy()
    assert np.mean(~same) <= 1e-2
    assert rel_close(xa[:, same].cpu(), xb[:, same].cpu(), 2e-4)
    assert rel_close(ua[:, same].cpu(), ub[:, same].cpu(), 2e-4)
    assert rel_close(sa[0][:, same].cpu(), sb[0][:, same].cpu(), 2e-4)
    if np.all(same):
        for a, b in zip(grads["on"], grads["off"]):
            scale = 1 + float(b.abs().max())
            assert float((a - b).abs().max()) <= 2e-3 * scale


@pytest.mark.parametrize("name,d,hidden,B,dtype,scheme", [
    ("LQR", 20, (200, 200, 200), 100, torch.float32, "adaptive"),
    ("EKN", 20, (64, 64, 64), 37, torch.float32, "naive"),
    ("VDP", 20, (48, 48), 37, torch.float64, "adaptive"),
    ("LQR_var", 10, (32, 48, 24), 21, torch.float64, "naive"),
    ("LQR", 20, (256, 256, 256, 256), 20, torch.float32, "adaptive"),
    ("EKN", 5, (40, 40), 1, torch.float64, "adaptive")])
def test_bptt_stager_writer_kernel_bitwise(name, d, hidden, B, dtype, scheme):
    """k_rollout_nn_bwd2 (step inputs and z staged in LDS by a stager wavefront, G stored by
    a writer wavefront) gives bitwise the G of k_rollout_nn_bwd (the same products in the
    same order), partial tiles, the Eikonal head, both schemes, both dtypes."""
    import os
    N, T = 12, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme=scheme,
                      dtype="float32" if dtype == torch.float32 else "float64")
    ep = getattr(peq, name)(cfg.eqn_config)
    net, _ = actor_pair(cfg, dtype)
    eqp = ep.params()
    sch = SCHEMES[scheme]
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=8, dtype=dtype, device=DEV)
    y, disc, xN, saved = ops.actor_rollout_saves(eqp, sch, x0, dw, T, N, net)
    x, u, dwc, z, flag, disc_t = saved[:6]
    params = [p.detach() for p in net.trainable_variables()]
    L = len(hidden)
    gam, bet, Ws, b = params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]
    widths = [Ws[0].shape[0]] + [w.shape[1] for w in Ws]
    view, wt, wt_km = ops.mlp_prepare(gam, bet, Ws, b, net.ekn_head, True)
    g_y = torch.full_like(y, 1.0 / B)
    g_disc = torch.rand_like(y)
    g_xN = torch.randn_like(xN)
    out = {}
    old = os.environ.get("DPAC_BPTT")
    try:
        for k in ("1", "2"):
            os.environ["DPAC_BPTT"] = k
            G = ops._bptt_fused(eqp, sch, T, N, L, x, u, dwc, z, flag, disc_t, view, wt, wt_km, widths,
                                g_xN, g_disc, g_y)
            out[k] = ops.G_all(G).clone()
    finally:
        if old is None:
            os.environ.pop("DPAC_BPTT", None)
        else:
            os.environ["DPAC_BPTT"] = old
    assert torch.isfinite(out["2"]).all()
    assert torch.equal(out["1"], out["2"])


@pytest.mark.parametrize("name,d,hidden,B,scheme", [
    ("LQR", 20, (200, 200, 200), 100, "adaptive"),
    ("EKN", 20, (200, 200, 200), 37, "naive"),
    ("VDP", 20, (200, 200), 50, "adaptive"),
    ("LQR", 4, (208, 200, 193), 20, "adaptive"),
    ("LQR_var", 20, (200,), 17, "naive")])
def test_actor_fast_path_bitwise(name, d, hidden, B, scheme):
    """The actor-shape fast path (narrow layers' weights resident in VGPRs, wide layers'
    first weight groups loaded before the preceding barrier) gives bitwise the outputs of
    the generic layer code, in the fused forward (16-row tiles) and in the BPTT kernel:
    K16 = 16 and 32 first products, 193..208-wide hidden layers, 1-3 hidden layers, the
    Eikonal head (21 outputs), VDP's 10 controls."""
    import os
    N, T = 12, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme=scheme, dtype="float32")
    ep = getattr(peq, name)(cfg.eqn_config)
    net, _ = actor_pair(cfg, torch.float32)
    eqp = ep.params()
    sch = SCHEMES[scheme]
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=9, dtype=torch.float32, device=DEV)
    params = [p.detach() for p in net.trainable_variables()]
    L = len(hidden)
    gam, bet, Ws, b = params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]
    widths = [Ws[0].shape[0]] + [w.shape[1] for w in Ws]
    view, wt, wt_km = ops.mlp_prepare(gam, bet, Ws, b, net.ekn_head, True)
    g_y = torch.full((B,), 1.0 / B, device=DEV)
    keys = ("DPAC_NN_FAST", "DPAC_NN_TILE", "DPAC_NN_X3")
    old = {k: os.environ.get(k) for k in keys}
    fwd, bwd = {}, {}
    try:
        os.environ["DPAC_NN_TILE"] = "16"
        os.environ["DPAC_NN_X3"] = "0"  # the f32 kernels' two layer codes
        for f in ("0", "1"):
            os.environ["DPAC_NN_FAST"] = f
            fwd[f] = [t.clone() if torch.is_tensor(t) else [s.clone() for s in t[:3]]
                      for t in ops.rollout_nn(eqp, sch, x0, dw, T, N, view, cost_order=_lib.COST_ACTOR, save=True)]
            x, _, _, u, _, _, (z, flag, disc_t) = fwd[f]
            G = ops._bptt_fused(eqp, sch, T, N, L, x, u, dw, z, flag, disc_t, view, wt, wt_km, widths,
                                torch.ones_like(x[-1]) * 0.01, torch.full_like(g_y, 0.5), g_y)
            bwd[f] = ops.G_all(G).clone()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for a, b in zip(fwd["0"], fwd["1"]):
        for s, t in (zip(a, b) if isinstance(a, list) else [(a, b)]):
            assert torch.equal(s, t)
    assert torch.isfinite(bwd["1"]).all()
    assert torch.equal(bwd["0"], bwd["1"])


@pytest.mark.parametrize("name,d,hidden,B,scheme", [
    ("LQR", 20, (200, 200, 200), 2048, "adaptive"),
    ("EKN", 20, (200, 200, 200), 37, "naive"),
    ("VDP", 20, (200, 200), 50, "adaptive"),
    ("LQR", 4, (208, 200, 193), 20, "adaptive"),
    ("LQR_var", 20, (200,), 17, "naive")])
def test_bptt_sign_mask_bitwise(name, d, hidden, B, scheme, monkeypatch):
    """The actor forward's sign-bit mask (dpac_rollout_nn_fwd_masked: bit r % 4 of byte
    [13 l + c/16][r/4 % 4][c % 16] of row r's 16-row tile = [BN_{l+1}(z) > 0] of hidden layer
    l) leaves every forward output
    bitwise unchanged, matches the signs recomputed from the saved z, and the BPTT reading
    it (dpac_rollout_nn_bwd_masked) gives bitwise the G of the z-based BPTT."""
    N, T = 12, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme=scheme, dtype="float32")
    ep = getattr(peq, name)(cfg.eqn_config)
    net, _ = actor_pair(cfg, torch.float32)
    eqp = ep.params()
    sch = SCHEMES[scheme]
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=13, dtype=torch.float32, device=DEV)
    params = [p.detach() for p in net.trainable_variables()]
    L = len(hidden)
    gam, bet, Ws, b = params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]
    widths = [Ws[0].shape[0]] + [w.shape[1] for w in Ws]
    view, wt, wt_km = ops.mlp_prepare(gam, bet, Ws, b, net.ekn_head, True)
    monkeypatch.setenv("DPAC_NN_TILE", "16")
    monkeypatch.setenv("DPAC_NN_FAST", "1")
    monkeypatch.setenv("DPAC_NN_X3", "0")  # the f32 pair (the x3 pair: test_gpu_nn_x3.py)
    fwd = {}
    for m in (False, True):
        monkeypatch.setattr(ops, "MASK_BPTT", m)
        fwd[m] = ops.rollout_nn(eqp, sch, x0, dw, T, N, view, cost_order=_lib.COST_ACTOR, save=True)
    assert fwd[False][6][3] is None
    mask = fwd[True][6][3]
    mb = _lib.load().dpac_rollout_nn_mask_tile_bytes(ctypes.byref(view.struct))
    assert mb == 13 * 64 * L and mask is not None and mask.shape == (N, (B + 15) // 16, mb)
    for a, c in zip(fwd[False][:6], fwd[True][:6]):
        assert (a is None and c is None) or torch.equal(a, c)
    for a, c in zip(fwd[False][6][:3], fwd[True][6][:3]):
        assert torch.equal(a, c)
    # the bits against the signs of BN(z) recomputed here (borderline |y| excluded)
    x, _, _, u, _, _, (z, flag, disc_t, _) = fwd[True]
    # [N, tiles, 13 L col tiles, 4 row quads, 16 cols] -> bit r % 4 -> [N, rows, 13 L * 16 cols]
    m5 = mask.to(torch.int32).reshape(N, -1, 13 * L, 4, 16)
    bits = torch.stack([(m5 >> k) & 1 for k in range(4)], 4)  # [N, tiles, ct, quad, row%4, 16]
    bits = bits.permute(0, 1, 3, 4, 2, 5).reshape(N, -1, 13 * L * 16)[:, :B]
    off = 0
    for l in range(L):
        w = widths[l + 1]
        zl = z[:, :, off:off + w]
        off += w
        yl = bet[l + 1] + zl * (net.bn_rs * gam[l + 1])
        got = bits[:, :, 13 * 16 * l:13 * 16 * l + w]
        clear = yl.abs() > 1e-5 * (1 + yl.abs().max())
        assert torch.equal(got[clear].bool(), (yl > 0)[clear])
    g_y = torch.full((B,), 1.0 / B, device=DEV)
    G = {}
    for use in (None, mask):
        G[use is None] = ops.G_all(ops._bptt_fused(
            eqp, sch, T, N, L, x, u, dw, z, flag, disc_t, view, wt, wt_km, widths,
            torch.ones_like(x[-1]) * 0.01, torch.full_like(g_y, 0.5), g_y, use)).clone()
    assert torch.isfinite(G[False]).all()
    assert torch.equal(G[True], G[False])
