"""GPU: the float32 PRODUCTION path against the float64 oracle (north_star: "outputs must match
the reference ... within a stated fp32 tolerance (value-function L2 error and control error)").

The production float32 path differs from the float64 one in code, not only in precision:
  * the actor-shape fast path of the fused rollout / BPTT (16-row tiles, taken for B > 1024 and
    193..208-wide hidden layers), whose products run on split-fp16 MFMA (dpac_rollout_nn_x3.h:
    three v_mfma_f32_16x16x32_f16 per 32-k step, f32 accumulate), as do the critic's V / G row
    kernels (dpac_mlp_x3.h) and every network's parameter gradients (dpac_mlp_grad_x3.h);
  * the BPTT reading the forward's activation sign bits (dpac_rollout_nn_*_masked);
  * the k-major weight images (dwordx4 B loads);
  * the critic's G network with the TD1 dot fused (dpac_mlp_rows_fwd_td1), HIP graphs and the
    split critic / actor steps on side streams.
Every test here runs that path (asserted where the path is observable) against the float64
oracle (oracle/, the torch-CPU restatement of solver.py / equation.py) on the same inputs and
initial weights.

Tolerances (float32 against float64):
  * rollout: <= 1e-3 of trajectories may flip an exit decision (|x| = R is a discontinuity);
    matched trajectories within 1e-5 (1 + |ref|) on x, u and dt;
  * gradients (flipped trajectories removed from both sides): per tensor
    max |g - g_ref| <= 1e-3 * max |g_ref|;
  * training (6 iterations, validated after every one) against the committed float64 oracle
    vectors tests/golden/train_<config>_B<batch>.npz — lqr_d20 and ekn_d20 at B = 4096,
    lqr_var_d20 at 2048, vdp_d20 at 8192: |err_value - ref| <= 1e-5 and
    |err_control - ref| <= 1e-5 (absolute, relative-L2 units) at every logged step, the
    losses within 1e-4 relative, and every parameter summary within 2e-4 (1 + |ref|);
  * full-size shards (lqr_var_d20 16384 = 8 x 2048, vdp_d20 65536 = 8 x 8192): finite losses
    and gradients, and the count-weighted shard gradients sum to the whole batch's within
    1e-4 of its largest entry per tensor.
Measured on MI355X (round 3): paths 6.3e-7, gradients 9.6e-5 (critic) / 1.2e-6 (actor),
err_value 9.1e-7, err_control 4.5e-7, parameters 2.1e-5 (profiles/r03_fp32_parity.txt).
"""
import glob
import os

import numpy as np
import pytest
import torch

from deeppde_actorcritic_amd import _lib, ops
from deeppde_actorcritic_amd import equation as peq
from deeppde_actorcritic_amd import solver as psol
from deeppde_actorcritic_amd.config import baseline_config, set_floatx
from oracle import equations as oeq
from oracle import solver as osol
from tests.helpers import full_config, rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLDENS = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "train_*_B*.npz")))

TOL_FLIP = 1e-3      # fraction of trajectories allowed to flip an exit decision
TOL_PATH = 1e-5      # matched trajectories, |a - b| <= TOL_PATH (1 + |b|)
TOL_GRAD = 1e-3      # per tensor, max |g - g_ref| <= TOL_GRAD max |g_ref|
TOL_ERR = 1e-5       # err_value / err_control, absolute, every logged step
TOL_LOSS = 1e-4      # validation losses, |a - b| <= TOL_LOSS (1 + |b|)
TOL_PARAM = 2e-4     # parameter summaries, |a - b| <= TOL_PARAM (1 + |b|)


@pytest.fixture(autouse=True)
def _default_paths(monkeypatch):
    """The production selection: no test override of the kernel choice."""
    for k in ("DPAC_NN_TILE", "DPAC_NN_FAST", "DPAC_NN_X3", "DPAC_BPTT", "DPAC_MASK_BPTT", "DPAC_WEIGHT_KM",
              "DPAC_MLP_MATH", "DPAC_PG_X3"):
        monkeypatch.delenv(k, raising=False)
    assert ops.MASK_BPTT and ops.WEIGHT_KM == "on" and ops.CRITIC_TD1 == "fused"
    assert ops.BPTT_MODE == "fused" and ops.ROW_MLP == "kernel" and ops.PARAM_GRADS == "kernel"
    yield
    set_floatx("float64")


def _pair(cfg, seed):
    bp = getattr(peq, cfg.eqn_config.eqn_name)(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bp, seed=seed, sampler="host", graphs=False)
    params = {"critic": sp.model_critic.NN_value.export_params(),
              "critic_grad": sp.model_critic.NN_value_grad.export_params(),
              "actor": sp.model_actor.NN_control.export_params()}
    return sp, osol.ActorCriticSolver(cfg, oeq.make(cfg.eqn_config), params=params)


def _f32(a):
    return torch.as_tensor(np.asarray(a), dtype=torch.float32, device=DEV)


@pytest.mark.parametrize("name,B", [("LQR", 1040), ("LQR", 2050), ("EKN", 1100), ("VDP", 1043),
                                    ("LQR_var", 1060)])
def test_fp32_sixteen_row_fast_path_forward_vs_oracle(name, B):
    """The float rollout with the actor MLP at B > 1024 (16-row tiles, actor-shape fast path,
    sign-bit mask written) against the oracle's propagate_adaptive with the oracle DeepNN."""
    N, T = 50, 0.2
    cfg = full_config(name, 20, N=N, hidden=(200, 200, 200), scheme="adaptive", dtype="float32")
    sp, so = _pair(cfg, 21)
    net = sp.model_actor.NN_control
    eo = so.bsde
    np.random.seed(31)
    x0, dw, _ = eo.sample_normal(B, N)
    xr, dtr, cr = eo.propagate_adaptive(B, x0, dw, so.model_actor.NN_control, False, T, N, False)
    x, dt, coef, u, _, _, saves = ops.rollout_nn(
        sp.bsde.params(), _lib.SCHEME_ADAPTIVE, _f32(x0), _f32(dw).permute(2, 0, 1).contiguous(), T, N,
        net.mlp_view(), cost_order=_lib.COST_ACTOR, save=True)
    assert saves[3] is not None, "the 16-row fast path did not run (no sign-bit mask written)"
    same = np.all(coef.cpu().numpy() == cr.numpy(), axis=1)
    flips = float(np.mean(~same))
    print(f"\n[fp32 fwd {name} B={B}] flip fraction {flips:.2e}")
    assert flips <= TOL_FLIP
    xm = x.permute(1, 2, 0).cpu().double().numpy()[same]
    err = np.max(np.abs(xm - xr.numpy()[same]) / (1 + np.abs(xr.numpy()[same])))
    print(f"[fp32 fwd {name} B={B}] matched max rel |dx| {err:.2e}")
    assert err <= TOL_PATH
    assert rel_close(dt.cpu().double().numpy()[same], dtr.numpy()[same], TOL_PATH)
    with torch.no_grad():
        ur = torch.stack([so.model_actor.NN_control(xr[:, :, t]) for t in range(N)])  # [N, B, c]
    assert rel_close(u.cpu().double().numpy()[:, same], ur.numpy()[:, same], TOL_PATH)


def _matched(sp, so, data, N, T):
    """Trajectories whose float32 production rollout keeps every exit decision of the oracle."""
    x0, dw, _ = data
    _, _, cr = so.bsde.propagate_adaptive(x0.shape[0], x0, dw, so.model_actor.NN_control, False, T, N, False)
    _, _, coef, _, _, _, _ = ops.rollout_nn(
        sp.bsde.params(), _lib.SCHEME_ADAPTIVE, _f32(x0), _f32(dw).permute(2, 0, 1).contiguous(), T, N,
        sp.model_actor.NN_control.mlp_view(), want_u=False)
    return np.all(coef.cpu().numpy() == cr.numpy(), axis=1)


def _grad_err(gp, go):
    worst = 0.0
    for a, b in zip(gp, go):
        if b is None:
            assert a is None or float(a.abs().max()) == 0.0
            continue
        a = a.detach().to("cpu", torch.float64)
        scale = float(b.detach().abs().max())
        worst = max(worst, float((a - b.detach()).abs().max()) / max(scale, 1e-30))
    return worst


@pytest.mark.parametrize("name,B", [("LQR", 1100), ("LQR_var", 1100), ("EKN", 1040), ("VDP", 1100)])
def test_fp32_production_gradients_vs_oracle_tape(name, B):
    """The critic's and the actor's float32 gradients from the production kernels (critic_front +
    critic_G_back: fused TD1 G network; actor_forward + actor_grads_from: 16-row fast path,
    sign-bit-mask BPTT, k-major images, parameter-gradient kernel) against the oracle's
    GradientTape restatement (float64) on the same batch.  VDP runs BASELINE configs[4]'s
    shapes (d = 20, c = 10: actor 20-200-200-200-10, one-lane trajectory groups)."""
    N, T = 50, 0.2
    cfg = full_config(name, 20, N=N, hidden=(200, 200, 200), batch=B, scheme="adaptive", td="TD1",
                      dtype="float32")
    sp, so = _pair(cfg, 5)
    np.random.seed(17)
    dc = so.bsde.sample_normal(B, N)
    da = so.bsde.sample_normal(B, N)
    keep_c, keep_a = _matched(sp, so, dc, N, T), _matched(sp, so, da, N, T)
    print(f"\n[fp32 grads {name}] flips critic {np.sum(~keep_c)} actor {np.sum(~keep_a)} of {B}")
    assert np.mean(~keep_c) <= TOL_FLIP and np.mean(~keep_a) <= TOL_FLIP
    dc = tuple(a[keep_c] for a in dc)
    da = tuple(a[keep_a] for a in da)
    assert min(dc[0].shape[0], da[0].shape[0]) > 1024  # still the 16-row fast path
    # critic: the production split step, on one batch
    front = sp.critic_front(dc)
    assert len(front) == 7, "the fused TD1 critic path did not run"
    assert front[4] is not None, "the G network's sign-bit mask was not written"
    gp_c = front[0] + sp.critic_G_back(front)
    go_c, _ = so.grad_critic(dc, False, False)
    # actor: forward with saves (sign-bit mask) + BPTT kernels
    fwd = sp.actor_forward(da)
    assert fwd[3][6] is not None, "the actor forward wrote no sign-bit mask"
    gp_a = sp.actor_grads_from(fwd)
    go_a, _ = so.grad_actor(da, False, False, False)
    ec, ea = _grad_err(gp_c, go_c), _grad_err(gp_a, go_a)
    print(f"[fp32 grads {name}] critic max rel err {ec:.2e}, actor {ea:.2e}")
    assert ec <= TOL_GRAD and ea <= TOL_GRAD


def _summarize(tensors):
    out = []
    for t in tensors:
        t = t.detach().to("cpu", torch.float64).reshape(-1)
        out.append([float(t.sum()), float((t * t).sum())] + t[:16].tolist() + [0.0] * (16 - min(16, t.numel())))
    return np.array(out, dtype=np.float64)


@pytest.mark.parametrize("path", GOLDENS, ids=[os.path.basename(p)[6:-4] for p in GOLDENS])
def test_fp32_production_training_vs_oracle_vectors(path):
    """A BASELINE config trained in float32 on the production path — HIP graphs, the split
    critic step with the fused TD1 G network, the actor step on the 16-row fast path with the
    sign-bit-mask BPTT, split-fp16 MFMA — from the oracle's initial weights and numpy sample
    stream, against the float64 oracle's iterations (tests/golden/make_train_golden.py):
    lqr_d20 at B = 4096 (configs[1]), ekn_d20 at 4096 (configs[2]), lqr_var_d20 at 2048 and
    vdp_d20 at 8192 (the per-rank shards of configs[3] and [4] on 8 GPUs).
    Reference: solver.py:36-71 (train), :109-119 (err_value / err_control)."""
    g = np.load(path)
    name = str(g["name"]) if "name" in g.files else "lqr_d20"
    seed_params, seed_np, iters, batch, valid = (int(v) for v in g["meta"])
    assert iters >= 4 and batch > 1024
    cfg = baseline_config(iters, 1, "float32", batch, valid, name)
    bsde = getattr(peq, cfg.eqn_config.eqn_name)(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bsde, seed=seed_params, sampler="host", graphs=True)
    np.random.seed(seed_np)
    hist = sp.train()[0]
    assert sp._actor_split_ok() and sp._critic_split_ok()
    # the split graphs (round 5: psol.GRAPH_SETS alternating sets, solver.train_iteration), and no
    # unsplit gradient graph
    sets = [s for v in sp._gsets.values() for s in v if s is not None]
    assert len(sets) == psol.graph_sets(batch) and not sp._graphs
    assert all(isinstance(a, psol._SplitActorGraphs) and isinstance(c, psol._SplitCriticGraphs) for a, c in sets)
    ref = g["history"]
    assert hist.shape == ref.shape
    d_val = np.abs(hist[:-1, 3] - ref[:-1, 3])
    d_ctl = np.abs(hist[:-1, 5] - ref[:-1, 5])
    d_loss = np.abs(hist[:, 1:3] - ref[:, 1:3]) / (1 + np.abs(ref[:, 1:3]))
    got = _summarize(sp.critic_variables() + sp.actor_variables())
    d_par = np.abs(got - g["params"]) / (1 + np.abs(g["params"]))
    print(f"\n[fp32 training {name} B={batch}] max |d err_value| {d_val.max():.2e}, "
          f"max |d err_control| {d_ctl.max():.2e}, losses {d_loss.max():.2e}, params {d_par.max():.2e}")
    assert d_val.max() <= TOL_ERR and d_ctl.max() <= TOL_ERR
    assert d_loss.max() <= TOL_LOSS
    assert got.shape == g["params"].shape and d_par.max() <= TOL_PARAM


TOL_SHARD = 1e-4  # per tensor, max |sum of weighted shard gradients - whole batch| <= TOL_SHARD max |whole|


@pytest.mark.parametrize("name,total,world", [("lqr_var_d20", 16384, 8), ("vdp_d20", 65536, 8)])
def test_fp32_full_size_shards_sum_to_whole_batch(name, total, world):
    """BASELINE configs[3] / [4] at full size in float32 on the production kernels: the global
    batch (16384 / 65536, N = 100, 3x200 MLPs, TD1, adaptive) and its 8 per-rank shards (2048 /
    8192 trajectories: what each GPU of the 8-GPU run computes; the device sampler keyed by
    global trajectory index).  Losses and gradients are finite, and the count-weighted sum of
    the shard gradients (what parallel.DataParallel's all-reduce forms) equals the whole
    batch's within TOL_SHARD (float32 summation order: chunked row sums per launch).
    Reference: solver.py:73-83 (batch-mean losses), :85-97 (gradients)."""
    from deeppde_actorcritic_amd.parallel import shard_range
    cfg = baseline_config(1, 1, "float32", total, 256, name)
    bsde = getattr(peq, cfg.eqn_config.eqn_name)(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bsde, seed=3, sampler="device", graphs=False)
    N, key = 100, 0x5EED

    def grads(data):
        front = sp.critic_front(data)
        assert len(front) == 7  # fused TD1 critic
        gc = [g.detach().double() for g in front[0] + sp.critic_G_back(front)]
        ga = [g.detach().double() for g in sp.actor_grads_from(sp.actor_forward(data))]
        return gc + ga

    full = bsde.sample_device("normal", total, N, key, 0, torch.float32)
    with torch.no_grad():
        lc = float(sp._valid_loss_critic(full, total))
        la = float(sp._valid_loss_actor(full, total))
    assert np.isfinite(lc) and np.isfinite(la)
    g_full = grads(full)
    assert all(bool(torch.isfinite(g).all()) for g in g_full)
    g_sum = None
    for r in range(world):
        off, cnt = shard_range(total, r, world)
        shard = bsde.sample_device("normal", cnt, N, key, off, torch.float32)
        assert torch.equal(shard.x0, full.x0[off:off + cnt])
        g = grads(shard)
        assert all(bool(torch.isfinite(t).all()) for t in g)
        g = [t * (cnt / total) for t in g]
        g_sum = g if g_sum is None else [a + b for a, b in zip(g_sum, g)]
    worst = max(float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30) for a, b in zip(g_sum, g_full))
    print(f"\n[fp32 shards {name} {world}x{total // world}] losses {lc:.4e} {la:.4e}; "
          f"max rel |sum of shards - whole| {worst:.2e}")
    assert worst <= TOL_SHARD
