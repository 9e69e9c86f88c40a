"""GPU: the split-fp16 (x3) fused NN rollout and BPTT (csrc/dpac_rollout_nn_x3.h) — the actor
MLP of solver.py:260-278 inside the rollout of equation.py:46-106, and its BPTT (solver.py:92-97),
with every product as three v_mfma_f32_16x16x32_f16 (hi*hi + hi*lo + lo*hi) in f32.

Against the exact-f32 kernels (DPAC_NN_X3=0, themselves checked against the float64 oracle in
test_gpu_rollout_nn.py) on identical inputs, and directly against the float64 oracle:
  * forward: <= 1e-3 of trajectories may flip an exit decision (the boundary |x| = R is a
    discontinuity); matched trajectories agree within 2e-5 (1 + |b|) on x, u, dt and the saves;
  * the sign-bit mask keeps FwdEpiM's byte layout: it equals the signs recomputed from the
    x3 forward's saved z, and the f32 BPTT reading it gives bitwise the G of the z-based f32 BPTT;
  * BPTT: per layer block, max |G_x3 - G_f32| <= 2e-4 max |G_f32| on the same forward saves;
  * actor gradients vs the oracle tape: test_gpu_fp32_production.py (the production path).
"""
import ctypes

import numpy as np
import pytest
import torch

from deeppde_actorcritic_amd import _lib, ops
from deeppde_actorcritic_amd import equation as peq
from oracle import equations as oeq
from tests.helpers import full_config, rel_close
from tests.test_gpu_rollout_nn import SCHEMES, actor_pair

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL_FLIP = 1e-3
TOL_PATH = 2e-5
TOL_G = 2e-4

CASES = [("LQR", 20, (200, 200, 200), 2048, "adaptive"),
         ("LQR", 20, (200, 200, 200), 1037, "naive"),       # partial last tile
         ("EKN", 20, (200, 200, 200), 1100, "adaptive"),     # Eikonal head: 21 outputs
         ("VDP", 20, (200, 200), 1043, "adaptive"),          # one-lane groups
         ("LQR", 4, (208, 200, 193), 1030, "adaptive"),      # K16 = 16 first product, 193..208 widths
         ("LQR_var", 20, (200,), 1050, "naive")]             # one hidden layer: no wide product


def _setup(name, d, hidden, B, scheme, seed):
    N, T = 24, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme=scheme, dtype="float32")
    ep = getattr(peq, name)(cfg.eqn_config)
    net, onet = actor_pair(cfg, torch.float32)
    eqp = ep.params()
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=seed, dtype=torch.float32, device=DEV)
    return cfg, eqp, net, onet, x0, dw, N, T


def _fwd(eqp, sch, x0, dw, T, N, view):
    return ops.rollout_nn(eqp, sch, x0, dw, T, N, view, cost_order=_lib.COST_ACTOR, save=True)


@pytest.mark.parametrize("name,d,hidden,B,scheme", CASES)
def test_x3_forward_matches_f32(name, d, hidden, B, scheme, monkeypatch):
    cfg, eqp, net, _, x0, dw, N, T = _setup(name, d, hidden, B, scheme, 41)
    sch = SCHEMES[scheme]
    monkeypatch.delenv("DPAC_NN_TILE", raising=False)
    view = net.mlp_view()
    assert view.struct.weight_x3[0] is not None
    out = {}
    for x3 in ("1", "0"):
        monkeypatch.setenv("DPAC_NN_X3", x3)
        out[x3] = _fwd(eqp, sch, x0, dw, T, N, view)
    xa, dta, ca, ua, ya, da, sa = out["1"]
    xb, dtb, cb, ub, yb, db, sb = out["0"]
    assert sa[3] is not None and sb[3] is not None  # both 16-row paths wrote a mask
    assert not torch.equal(ua, ub), "the x3 path did not run (bitwise the f32 kernel)"
    same = torch.all(ca == cb, dim=1).cpu().numpy()
    print(f"\n[x3 fwd {name} d={d} B={B}] flips {np.mean(~same):.2e}")
    assert np.mean(~same) <= TOL_FLIP
    for a, b in ((xa[:, same], xb[:, same]), (ua[:, same], ub[:, same]), (dta[same], dtb[same]),
                 (ya[same], yb[same]), (sa[0][:, same], sb[0][:, same]), (sa[2][:, same], sb[2][:, same])):
        err = float(((a - b).abs() / (1 + b.abs())).max())
        assert err <= TOL_PATH, err
    assert torch.equal(sa[1][:, same], sb[1][:, same])  # saved flags


@pytest.mark.parametrize("name,d,hidden,B,scheme", CASES[:1] + CASES[2:5])
def test_x3_forward_vs_oracle(name, d, hidden, B, scheme):
    """The x3 forward against the float64 oracle's propagate_* with the oracle DeepNN."""
    N, T = 24, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme=scheme, dtype="float32")
    eo = oeq.make(cfg.eqn_config)
    ep = getattr(peq, name)(cfg.eqn_config)
    net, onet = actor_pair(cfg, torch.float32)
    np.random.seed(43)
    x0, dw, _ = eo.sample_normal(B, N)
    prop = eo.propagate_naive if scheme == "naive" else eo.propagate_adaptive
    xr, dtr, cr = prop(B, x0, dw, onet, False, T, N, False)
    x, dt, coef, u, _, _, _ = ops.rollout_nn(
        ep.params(), SCHEMES[scheme], torch.as_tensor(x0, dtype=torch.float32, device=DEV),
        torch.as_tensor(dw, dtype=torch.float32, device=DEV).permute(2, 0, 1).contiguous(), T, N,
        net.mlp_view())
    same = np.all(coef.cpu().numpy() == cr.numpy(), axis=1)
    assert np.mean(~same) <= TOL_FLIP
    xm = x.permute(1, 2, 0).cpu().double().numpy()[same]
    err = np.max(np.abs(xm - xr.numpy()[same]) / (1 + np.abs(xr.numpy()[same])))
    print(f"\n[x3 fwd vs oracle {name} d={d} B={B}] flips {np.mean(~same):.2e}, matched max rel |dx| {err:.2e}")
    assert err <= 1e-5
    with torch.no_grad():
        ur = torch.stack([onet(xr[:, :, t], False, need_grad=False) for t in range(N)])
    assert rel_close(u.cpu().double().numpy()[:, same], ur.numpy()[:, same], 1e-5)


def _bits(mask, N, B, L):
    """[N, tiles, 13 L, 4 row quads, 16 cols] bytes -> [N, B, 13 L * 16] bits (FwdEpiM layout)."""
    m5 = mask.to(torch.int32).reshape(N, -1, 13 * L, 4, 16)
    bits = torch.stack([(m5 >> k) & 1 for k in range(4)], 4)
    return bits.permute(0, 1, 3, 4, 2, 5).reshape(N, -1, 13 * L * 16)[:, :B]


@pytest.mark.parametrize("name,d,hidden,B,scheme", CASES)
def test_x3_mask_layout_and_bptt(name, d, hidden, B, scheme, monkeypatch):
    cfg, eqp, net, _, x0, dw, N, T = _setup(name, d, hidden, B, scheme, 47)
    sch = SCHEMES[scheme]
    monkeypatch.delenv("DPAC_NN_TILE", raising=False)
    monkeypatch.delenv("DPAC_NN_X3", raising=False)
    params = [p.detach() for p in net.trainable_variables()]
    L = len(hidden)
    gam, bet, Ws, b = params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]
    widths = [Ws[0].shape[0]] + [w.shape[1] for w in Ws]
    view, wt, wt_km = ops.mlp_prepare(gam, bet, Ws, b, net.ekn_head, True)
    assert view.struct.weight_t_x3[0] is not None
    x, _, _, u, _, _, (z, flag, disc_t, mask) = _fwd(eqp, sch, x0, dw, T, N, view)  # x3 forward
    mb = _lib.load().dpac_rollout_nn_mask_tile_bytes(ctypes.byref(view.struct))
    assert mask is not None and mask.shape == (N, (B + 15) // 16, mb)
    # the bits are the signs of BN(z) of the saved z (borderline |y| excluded)
    bits = _bits(mask, N, B, L)
    off = 0
    for l in range(L):
        w = widths[l + 1]
        yl = bet[l + 1] + z[:, :, off:off + w] * (net.bn_rs * gam[l + 1])
        off += w
        got = bits[:, :, 13 * 16 * l:13 * 16 * l + w]
        clear = yl.abs() > 1e-5 * (1 + yl.abs().max())
        assert torch.equal(got[clear].bool(), (yl > 0)[clear])
    g_y = torch.full((B,), 1.0 / B, device=DEV)
    g_xN, g_disc = torch.ones_like(x[-1]) * 0.01, torch.full_like(g_y, 0.5)

    def bptt(m):
        return ops.G_all(ops._bptt_fused(eqp, sch, T, N, L, x, u, dw, z, flag, disc_t, view, wt, wt_km, widths,
                                         g_xN, g_disc, g_y, m)).clone()
    monkeypatch.setenv("DPAC_NN_X3", "0")
    g_f32_mask, g_f32_z = bptt(mask), bptt(None)
    assert torch.equal(g_f32_mask, g_f32_z)  # the mask layout is FwdEpiM's
    monkeypatch.delenv("DPAC_NN_X3")
    g_x3 = bptt(mask)
    assert torch.isfinite(g_x3).all()
    assert not torch.equal(g_x3, g_f32_z), "the x3 BPTT did not run"
    goff = np.cumsum([0] + widths).tolist()
    worst = 0.0
    for i in range(L + 2):
        ref = g_f32_z[:, :, goff[i]:goff[i + 1]]
        err = float((g_x3[:, :, goff[i]:goff[i + 1]] - ref).abs().max()) / max(float(ref.abs().max()), 1e-30)
        worst = max(worst, err)
    print(f"\n[x3 bptt {name} d={d} B={B}] max rel |dG| per block {worst:.2e}")
    assert worst <= TOL_G


@pytest.mark.parametrize("name,d,hidden,B,scheme", CASES + [("LQR", 20, (200, 200, 200), 1033, "adaptive")])
def test_x3_half_tile_workgroups_bitwise(name, d, hidden, B, scheme, monkeypatch):
    """8 trajectories per workgroup (DPAC_NX_ROWS=8: twice the workgroups, rows 8..15 of each
    MFMA row tile zero) against 16 (one tile): a row's products never mix rows, so the forward
    (states, controls, saves, the sign-bit mask of the live rows) and the BPTT's G are bitwise
    the same; the mask bytes of the two half-tile workgroups of a tile interleave (+32 bytes)."""
    cfg, eqp, net, _, x0, dw, N, T = _setup(name, d, hidden, B, scheme, 53)
    sch = SCHEMES[scheme]
    monkeypatch.delenv("DPAC_NN_TILE", raising=False)
    monkeypatch.delenv("DPAC_NN_X3", raising=False)
    params = [p.detach() for p in net.trainable_variables()]
    L = len(hidden)
    gam, bet, Ws, b = params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]
    widths = [Ws[0].shape[0]] + [w.shape[1] for w in Ws]
    view, wt, wt_km = ops.mlp_prepare(gam, bet, Ws, b, net.ekn_head, True)
    g_y = torch.full((B,), 1.0 / B, device=DEV)
    out, G = {}, {}
    for rows in ("16", "8"):
        monkeypatch.setenv("DPAC_NX_ROWS", rows)
        out[rows] = _fwd(eqp, sch, x0, dw, T, N, view)
        x, _, _, u, _, _, (z, flag, disc_t, mask) = out[rows]
        assert mask is not None
        g_xN, g_disc = torch.ones_like(x[-1]) * 0.01, torch.full_like(g_y, 0.5)
        G[rows] = ops.G_all(ops._bptt_fused(eqp, sch, T, N, L, x, u, dw, z, flag, disc_t, view, wt, wt_km,
                                            widths, g_xN, g_disc, g_y, mask)).clone()
    monkeypatch.delenv("DPAC_NX_ROWS")
    a, c = out["16"], out["8"]
    for i in range(6):
        assert torch.equal(a[i], c[i]), f"forward output {i}"
    for i in range(3):
        assert torch.equal(a[6][i], c[6][i]), f"save {i}"
    assert torch.equal(_bits(a[6][3], N, B, L), _bits(c[6][3], N, B, L))
    assert torch.isfinite(G["16"]).all()
    assert torch.equal(G["16"], G["8"])
