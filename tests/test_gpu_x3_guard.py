"""GPU: the split-fp16 range guard (include/dpac.h dpac_mlp.status).

The split-fp16 (x3) kernels carry every f32 operand as hi = fp16(a), lo = fp16((a - hi) 2^12),
exact only while |a| < 2^15; the reference computes in float64 and has no such ceiling
(solver.py:260-278).  Each x3 kernel checks every operand it splits (and dpac_mlp_prepare the
weight images), sets the device's status word on a violation, and every x3 launch is followed
by the exact-f32 kernel of the same operation, which runs only once the word is set.  So:
  * operands outside the range (here: BN scales multiplied by 2^17 or 2^20, so hidden
    activations reach 1e4 .. 1e6) set the word, and every output equals the exact-f32 kernels' bit for bit (row
    forward / backward chain, fused rollout with its saves and sign-bit mask, BPTT), the
    parameter gradients within 1e-6 (the fallback's single launch bins layers differently);
  * the same inputs WITHOUT the guard (ops.X3_GUARD = False) give non-finite or wrong values —
    the test inputs really leave the range;
  * in-range inputs leave the word clear;
  * end to end, the float32 production gradient functions on such a network match the float64
    oracle's GradientTape (tolerance of tests/test_gpu_fp32_production.py).
Measured on MI355X: round 4, 9 passed (profiles/r04_call5_validation.txt); round 5's verbose
log of this file is profiles/r05_x3_guard.txt.
"""
import numpy as np
import pytest
import torch

from deeppde_actorcritic_amd import _lib, ops
from deeppde_actorcritic_amd import equation as peq
from deeppde_actorcritic_amd import solver as psol
from deeppde_actorcritic_amd.config import set_floatx
from oracle import equations as oeq
from oracle import solver as osol
from tests.helpers import full_config

pytestmark = pytest.mark.gpu
DEV = "cuda"
BIG = 2.0 ** 17
TOL_GRAD = 1e-3


@pytest.fixture(autouse=True)
def _clean(monkeypatch):
    for k in ("DPAC_NN_TILE", "DPAC_NN_FAST", "DPAC_NN_X3", "DPAC_BPTT", "DPAC_MASK_BPTT", "DPAC_WEIGHT_KM",
              "DPAC_MLP_MATH", "DPAC_PG_X3"):
        monkeypatch.delenv(k, raising=False)
    ops.x3_status_reset(DEV)
    yield
    ops.x3_status_reset(DEV)
    set_floatx("float64")


def _net(AC, big_layer=None, name="LQR", seed=3, big=BIG):
    cfg = full_config(name, 20, hidden=(200, 200, 200), dtype="float32")
    net = psol.DeepNN(cfg, AC, torch.Generator().manual_seed(seed), torch.float32, DEV)
    if big_layer is not None:
        with torch.no_grad():
            net.bn_gamma[big_layer].mul_(big)
    return net


def _rows_all(net, x, g_out):
    prep = net.mlp_prepared()
    out, z = ops.mlp_rows(prep[0], x, save=True)
    g_x, grads = ops.row_mlp_backward(net.bn_rs, [p.detach() for p in net.trainable_variables()], x, z, g_out,
                                      True, True, prepared=prep)
    torch.cuda.synchronize()
    return [out, z, g_x], grads


def _with_math(monkeypatch, math, fn):
    monkeypatch.setattr(ops, "MLP_MATH", math)
    try:
        return fn()
    finally:
        monkeypatch.setattr(ops, "MLP_MATH", "x3")


def _finite(ts):
    return all(bool(torch.isfinite(t).all()) for t in ts if t is not None)


@pytest.mark.parametrize("big_layer", [1, 2, 0])
def test_rows_out_of_range_fall_back_to_f32(big_layer, monkeypatch):
    """dpac_mlp_rows_fwd / _bwd / dpac_mlp_param_grads (the critic's V / G networks) with BN_l
    times 2^17 over 65536 rows (the fallback's grid-stride pass covers 4096 tiles)."""
    net = _net("critic_grad", big_layer)
    R = 65536
    gen = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(R, 20, generator=gen, device=DEV)
    g_out = torch.randn(R, 20, generator=gen, device=DEV) / R
    ref, gref = _with_math(monkeypatch, "f32", lambda: _rows_all(net, x, g_out))
    assert _finite(ref) and _finite(gref)
    assert not ops.x3_fell_back(DEV)  # the f32 path has no status word
    got, ggot = _rows_all(net, x, g_out)
    assert ops.x3_fell_back(DEV)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    worst = max(float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30) for a, b in zip(ggot, gref))
    print(f"\n[x3 guard rows, BN_{big_layer} x 2^17] outputs bitwise f32; parameter gradients {worst:.1e}")
    assert worst <= 1e-6
    # the same launches unguarded: the split overflows (non-finite) or loses the value
    ops.x3_status_reset(DEV)
    monkeypatch.setattr(ops, "X3_GUARD", False)
    bad, gbad = _rows_all(net, x, g_out)
    monkeypatch.setattr(ops, "X3_GUARD", True)
    err = max(float((a - b).abs().max() / b.abs().max()) for a, b in zip(bad + gbad, ref + gref))
    assert not _finite(bad + gbad) or err > 1e-2, err


def test_rows_in_range_keep_the_split_fp16_path():
    net = _net("critic_grad")
    x = torch.randn(4096, 20, device=DEV)
    got, grads = _rows_all(net, x, torch.randn(4096, 20, device=DEV) / 4096)
    assert _finite(got) and _finite(grads)
    assert not ops.x3_fell_back(DEV)


def _rollout_and_bptt(net, eqp, x0, dw, T, N):
    """The actor's forward with saves, its BPTT chain G and the parameter gradients, as
    ops.actor_bptt_grads forms them (dpac_rollout_nn_fwd_masked, dpac_rollout_nn_bwd_masked,
    dpac_mlp_param_grads)."""
    view = net.mlp_view()
    x, dt, coef, u, y, disc, saves = ops.rollout_nn(eqp, _lib.SCHEME_ADAPTIVE, x0, dw, T, N, view,
                                                    cost_order=_lib.COST_ACTOR, save=True)
    assert saves[3] is not None, "no sign-bit mask: the 16-row fast path did not run"
    z, flag, disc_t, mask = saves
    B = x0.shape[0]
    gy = torch.full((B,), 1.0 / B, device=DEV)
    gd = torch.randn(B, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1)) / B
    gx = torch.randn(B, 20, device=DEV, generator=torch.Generator(device=DEV).manual_seed(2)) / B
    params = [p.detach() for p in net.trainable_variables()]
    L = (len(params) - 1) // 3 - 1
    gam, bet, Ws, b = params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]
    bview, wt, wt_km = ops.mlp_prepare(gam, bet, Ws, b, net.ekn_head, True)
    G = ops._bptt_fused(eqp, _lib.SCHEME_ADAPTIVE, T, N, L, x, u, dw, z, flag, disc_t, bview, wt, wt_km,
                        bview.widths, gx, gd, gy, mask)
    Gall = ops.G_all(G)
    grads = ops.mlp_param_grads(bview, x[:N].reshape(N * B, -1), z.reshape(N * B, -1), Gall.reshape(N * B, -1),
                                params)
    torch.cuda.synchronize()
    return [x, dt, coef, u, y, disc, z, flag, disc_t, mask, Gall], grads


@pytest.mark.parametrize("name,big_layer", [("LQR", 1), ("EKN", 2), ("LQR", 0)])
def test_fused_rollout_and_bptt_out_of_range_fall_back_to_f32(name, big_layer, monkeypatch):
    """dpac_rollout_nn_fwd_masked / dpac_rollout_nn_bwd_masked (the actor) with BN_l times 2^20 at
    B = 2048 (16-row tiles): the fallback writes the same x, dt, coef, u, cost, saves, mask and
    BPTT chain G as the f32 kernels, and the parameter gradients match theirs."""
    cfg = full_config(name, 20, N=16, hidden=(200, 200, 200), dtype="float32")
    eqp = getattr(peq, name)(cfg.eqn_config).params()
    net = _net("actor", big_layer, name=name, big=2.0 ** 20)
    B, N, T = 2048, 16, 0.2
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=9, dtype=torch.float32, device=DEV)
    monkeypatch.setenv("DPAC_NN_X3", "0")  # the exact-f32 kernels throughout
    monkeypatch.setenv("DPAC_PG_X3", "0")
    ref, gref = _rollout_and_bptt(net, eqp, x0, dw, T, N)
    monkeypatch.delenv("DPAC_NN_X3")
    monkeypatch.delenv("DPAC_PG_X3")
    ops.x3_status_reset(DEV)
    got, ggot = _rollout_and_bptt(net, eqp, x0, dw, T, N)
    assert ops.x3_fell_back(DEV)
    assert _finite(got) and _finite(ggot)
    names = ["x", "dt", "coef", "u", "y", "disc", "z", "flag", "disc_t", "mask", "G"]
    diff = [n for n, a, b in zip(names, got, ref) if not torch.equal(a, b)]
    assert not diff, diff
    worst = max(float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30) for a, b in zip(ggot, gref))
    print(f"\n[x3 guard rollout {name}, BN_{big_layer} x 2^20] paths, saves, mask, G bitwise f32; "
          f"actor gradients {worst:.1e}")
    assert worst <= 1e-6


def test_prepare_flags_out_of_range_weights():
    """dpac_mlp_prepare sets the word when a weight image value leaves the split range
    ((W_i diag s_{i+1})^T with s times 2^20: the backward images)."""
    net = _net("critic_grad", 2, big=2.0 ** 20)
    net.mlp_prepared()
    torch.cuda.synchronize()
    assert ops.x3_fell_back(DEV)
    ops.x3_status_reset(DEV)
    net.mlp_view()  # forward images only: W itself is in range
    torch.cuda.synchronize()
    assert not ops.x3_fell_back(DEV)


def _grad_err(gp, go):
    worst = 0.0
    for a, b in zip(gp, go):
        if b is None:
            continue
        a = a.detach().to("cpu", torch.float64)
        worst = max(worst, float((a - b.detach()).abs().max()) / max(float(b.detach().abs().max()), 1e-30))
    return worst


def test_fp32_production_gradients_with_out_of_range_networks_vs_oracle():
    """The float32 production gradient functions (critic_front + critic_G_back with the fused TD1
    G network, actor_forward + actor_grads_from) on networks whose first hidden BN scale is
    2^20 larger (activations of 1e5 .. 1e7: far outside the split range) against the float64
    oracle's GradientTape on the same batch and weights: the guard makes the x3 path exact
    f32 (max |g - g_ref| <= 1e-3 max |g_ref| per tensor, as tests/test_gpu_fp32_production.py).
    Reference: solver.py:85-97 (gradients), :260-278 (DeepNN)."""
    N, T, B = 20, 0.2, 1100
    cfg = full_config("LQR", 20, N=N, hidden=(200, 200, 200), batch=B, scheme="adaptive", td="TD1",
                      dtype="float32")
    bp = peq.LQR(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bp, seed=5, sampler="host", graphs=False)
    with torch.no_grad():
        for net in (sp.model_critic.NN_value, sp.model_critic.NN_value_grad, sp.model_actor.NN_control):
            net.bn_gamma[1].mul_(2.0 ** 20)
    params = {"critic": sp.model_critic.NN_value.export_params(),
              "critic_grad": sp.model_critic.NN_value_grad.export_params(),
              "actor": sp.model_actor.NN_control.export_params()}
    so = osol.ActorCriticSolver(cfg, oeq.make(cfg.eqn_config), params=params)
    np.random.seed(17)
    dc = so.bsde.sample_normal(B, N)
    da = so.bsde.sample_normal(B, N)
    front = sp.critic_front(dc)
    assert len(front) == 7
    gp_c = front[0] + sp.critic_G_back(front)
    go_c, _ = so.grad_critic(dc, False, False)
    fwd = sp.actor_forward(da)
    gp_a = sp.actor_grads_from(fwd)
    go_a, _ = so.grad_actor(da, False, False, False)
    torch.cuda.synchronize()
    assert ops.x3_fell_back(DEV)
    assert _finite(gp_c) and _finite(gp_a)
    ec, ea = _grad_err(gp_c, go_c), _grad_err(gp_a, go_a)
    print(f"\n[x3 guard, fp32 production vs oracle, BN_1 x 2^20] critic {ec:.2e}, actor {ea:.2e}")
    assert ec <= TOL_GRAD and ea <= TOL_GRAD


def _bptt_and_grads(net, eqp, x0, dw, T, N, sink=None):
    """_rollout_and_bptt's backward half (BPTT chain G + parameter gradients) with the forward
    done inline; sink: a list, the backward calls' guard fallbacks deferred into it
    (ops.deferred_fallbacks, dpac.h guard_phase)."""
    view = net.mlp_view()
    x, dt, coef, u, y, disc, saves = ops.rollout_nn(eqp, _lib.SCHEME_ADAPTIVE, x0, dw, T, N, view,
                                                    cost_order=_lib.COST_ACTOR, save=True)
    z, flag, disc_t, mask = saves
    B = x0.shape[0]
    gy = torch.full((B,), 1.0 / B, device=DEV)
    gd = torch.randn(B, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1)) / B
    gx = torch.randn(B, 20, device=DEV, generator=torch.Generator(device=DEV).manual_seed(2)) / B
    params = [p.detach() for p in net.trainable_variables()]
    with ops.deferred_fallbacks(sink):
        grads = ops.actor_bptt_grads(eqp, _lib.SCHEME_ADAPTIVE, T, N, net.ekn_head, net.bn_rs, params,
                                     (x, u, dw, z, flag, disc_t, mask), gy, gd, gx)
    return grads


@pytest.mark.parametrize("big", [None, 2.0 ** 20])
def test_deferred_fallbacks_equal_inline_bitwise(big):
    """dpac.h guard_phase (round 6): the actor's BPTT and parameter gradients
    with their guard fallbacks deferred (phase 1 now, phase 2 later, in order) give bitwise the
    gradients of the inline guard, in range (the fallbacks stay no-ops) and with BN_1 times 2^20
    (the word is set by the forward: the phase-1 launches do nothing and the deferred fallbacks
    recompute everything) — and out of range, the deferred phase is what fixes them."""
    cfg = full_config("LQR", 20, N=16, hidden=(200, 200, 200), dtype="float32")
    eqp = peq.LQR(cfg.eqn_config).params()
    net = _net("actor", 1 if big else None, big=big or 1.0)
    B, N, T = 2048, 16, 0.2
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=9, dtype=torch.float32, device=DEV)
    ref = [g.clone() for g in _bptt_and_grads(net, eqp, x0, dw, T, N)]
    torch.cuda.synchronize()
    assert ops.x3_fell_back(DEV) == (big is not None)
    ops.x3_status_reset(DEV)
    sink = []
    got = _bptt_and_grads(net, eqp, x0, dw, T, N, sink)
    assert len(sink) == 2  # the BPTT's and the parameter gradients' phase-2 calls
    if big:  # the phase-1 launches did nothing: with the partial sums poisoned, the gradients
        for ws in ops._WS_CACHE.values():  # are NaN until the deferred fallbacks run
            ws.fill_(255)
        got = _bptt_and_grads(net, eqp, x0, dw, T, N, [])  # (its own sink is dropped)
        torch.cuda.synchronize()
        assert not _finite(got)
        ops.x3_status_reset(DEV)
        sink = []
        got = _bptt_and_grads(net, eqp, x0, dw, T, N, sink)
    for f in sink:
        f()
    torch.cuda.synchronize()
    assert ops.x3_fell_back(DEV) == (big is not None)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def test_deferred_row_backward_fallback_equals_inline_bitwise():
    """The same for the row backward chain + parameter gradients (the critic's G network,
    ops.row_mlp_backward) with BN_1 times 2^17."""
    net = _net("critic_grad", 1)
    R = 8192
    gen = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(R, 20, generator=gen, device=DEV)
    g_out = torch.randn(R, 20, generator=gen, device=DEV) / R
    params = [p.detach() for p in net.trainable_variables()]

    def run(sink):
        prep = net.mlp_prepared()
        _, z = ops.mlp_rows(prep[0], x, save=True)
        with ops.deferred_fallbacks(sink):
            return ops.row_mlp_backward(net.bn_rs, params, x, z, g_out, True, True, prepared=prep)
    gx_ref, g_ref = run(None)
    ops.x3_status_reset(DEV)
    sink = []
    gx, g = run(sink)
    assert len(sink) == 2
    for f in sink:
        f()
    torch.cuda.synchronize()
    assert ops.x3_fell_back(DEV)
    assert torch.equal(gx, gx_ref) and all(torch.equal(a, b) for a, b in zip(g, g_ref))
