"""GPU: the critic's G network with the TD1 dot fused into its epilogue (SURVEY §8(f)
rank 2, reference solver.py:179-184) against the split path it replaces.

Split: G = dpac_mlp_rows_fwd over the N*B rollout rows, written to HBM, then
dpac_td_assemble_fwd(TD1) forms Σ_j (σ(x,u)dw)_j G_j per step; backward
dpac_td_assemble_bwd writes dL/dG [N,B,d] and dpac_mlp_rows_bwd reads it.
Fused: dpac_mlp_rows_fwd_td1 writes only the per-step dots, dpac_td_assemble_fwd
(DPAC_TD1_GDOT) reads them; dpac_td_assemble_bwd_gdot writes dL/d(dot) [N,B] and
dpac_mlp_rows_bwd_td1 forms dL/dG in its prologue.
The fused dot owns the components and sums them exactly as k_td does, so y, disc,
the saves and every parameter gradient must be BITWISE equal (both dtypes, the four
equations, including VDP's one-lane split and LQR_var's state-dependent σ).
The split path itself is checked against the oracle in test_gpu_kernels.py /
test_gpu_models.py.
"""
import ctypes
import os

import pytest
import torch

from deeppde_actorcritic_amd import _lib, ops
from deeppde_actorcritic_amd import equation as peq
from deeppde_actorcritic_amd import solver as psol
from deeppde_actorcritic_amd.config import floatx, set_floatx
from tests.helpers import full_config

pytestmark = pytest.mark.gpu

@pytest.fixture(autouse=True)
def _keep_floatx():
    old = floatx()
    yield
    set_floatx(old)


CASES = [("LQR", 20, "adaptive"), ("LQR_var", 20, "naive"), ("VDP", 20, "adaptive"),
         ("EKN", 5, "adaptive"), ("LQR", 4, "naive"), ("LQR_var", 10, "adaptive")]


def setup(name, d, scheme, dtype, B=83, N=14, hidden=(48, 40)):
    set_floatx(dtype)
    cfg = full_config(name, d, N=N, hidden=hidden, batch=B, valid=B, scheme=scheme, dtype=dtype)
    bp = getattr(peq, name)(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bp, seed=11, sampler="device", graphs=False)
    data = sp.sample(B, N)
    x, dt, coef, u = bp.rollout(scheme, data.x0, data.dw, cfg.eqn_config.total_time_critic, N,
                                cheat=True)
    return sp, bp, data, x, dt, coef, u


@pytest.mark.parametrize("dtype", ["float64", "float32"])
@pytest.mark.parametrize("name,d,scheme", CASES)
def test_fused_td1_bitwise_equals_split(name, d, scheme, dtype):
    sp, bp, data, x, dt, coef, u = setup(name, d, scheme, dtype)
    N, B = dt.shape[1], dt.shape[0]
    eqp = bp.params()
    Gnet = sp.model_critic.NN_value_grad
    view = Gnet.mlp_view()
    rows = x[:N].reshape(N * B, -1)
    u_rows, dw_rows = u.reshape(N * B, -1), data.dw.reshape(N * B, -1)
    # forward
    G, z_s = ops.mlp_rows(view, rows, save=True)
    y_s, disc_s = ops.td_assemble(eqp, _lib.TD1, x, u, data.dw, dt, coef, G.view(N, B, -1))
    gdot, z_f = ops.mlp_rows_td1(eqp, view, rows, u_rows, dw_rows, save=True)
    y_f, disc_f = ops.td_assemble_gdot(eqp, x, u, dt, coef, gdot.view(N, B))
    assert torch.equal(z_s, z_f)
    assert torch.equal(disc_s, disc_f)
    assert torch.equal(y_s, y_f), float((y_s - y_f).abs().max())
    # without saves too
    gdot2, _ = ops.mlp_rows_td1(eqp, view, rows, u_rows, dw_rows, save=False)
    assert torch.equal(gdot, gdot2)
    # backward
    g_y = torch.randn(B, dtype=torch.float64).to(x.device, x.dtype)
    params = Gnet.trainable_variables()
    gG = ops.td_assemble_bwd(eqp, x, u, data.dw, dt, coef, g_y)
    _, gr_s = ops.row_mlp_backward(Gnet.bn_rs, params, rows, z_s, gG.reshape(N * B, -1), False, True)
    g_gdot = ops.td_assemble_bwd_gdot(eqp, dt, coef, g_y)
    gr_f = ops.row_mlp_backward_td1(eqp, Gnet.bn_rs, params, rows, z_f, u_rows, dw_rows,
                                    g_gdot.reshape(N * B), True)
    assert len(gr_s) == len(gr_f)
    for a, b in zip(gr_s, gr_f):
        assert torch.equal(a, b), float((a - b).abs().max())


@pytest.mark.parametrize("name,d", [("LQR", 20), ("LQR_var", 10), ("VDP", 10)])
def test_critic_step_fused_equals_split(name, d):
    """The production critic step (critic_front + critic_G_back) in both modes:
    bitwise the same gradients of V's and G's variables."""
    set_floatx("float64")
    cfg = full_config(name, d, N=12, hidden=(40, 40), batch=50, valid=50, td="TD1")
    bp = getattr(peq, name)(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bp, seed=3, sampler="device", graphs=False)
    data = sp.sample(50, 12)
    old = ops.CRITIC_TD1
    try:
        out = {}
        for mode in ("split", "fused"):
            ops.CRITIC_TD1 = mode
            front = sp.critic_front(data)
            out[mode] = front[0] + sp.critic_G_back(front)
    finally:
        ops.CRITIC_TD1 = old
    for a, b in zip(out["split"], out["fused"]):
        assert torch.equal(a, b)


def test_fused_td1_rejects_mismatched_network():
    """The fused entry point needs the G network's output width == d."""
    sp, bp, data, x, dt, coef, u = setup("LQR", 20, "adaptive", "float64", B=16, N=4)
    view = sp.model_actor.NN_control.mlp_view()  # output width c == d here: accepted
    N, B = 4, 16
    rows = x[:N].reshape(N * B, -1)
    ops.mlp_rows_td1(bp.params(), view, rows, u.reshape(N * B, -1), data.dw.reshape(N * B, -1))
    eq = bp.params()
    eq.dim = 10  # the equation's d no longer matches the network's width
    eq.control_dim = 10
    with pytest.raises(_lib.DpacError):
        ops.call("dpac_mlp_rows_fwd_td1", ctypes.byref(eq), _lib.F64, N * B, ctypes.byref(view.struct),
                 ctypes.c_void_p(rows.data_ptr()), 20, ctypes.c_void_p(u.data_ptr()),
                 ctypes.c_void_p(data.dw.data_ptr()), ctypes.c_void_p(rows.data_ptr()), None,
                 ops._stream(rows))


@pytest.mark.parametrize("name,d", [("LQR", 4), ("LQR_var", 10)])
def test_fused_td1_dead_row_blocks_read_nothing_past_the_end(name, d):
    """Round 5 regression: the split-fp16 forward's last 64-row workgroup computes the TD1 dots
    in 16-row blocks, and a block wholly past the last row used to read its first row's sigma dw
    (and x, u for LQR_var) anyway — past the end of those arrays (seen once as a GPU fault in
    this file's LQR d = 4 case).  Here the rows end 48 rows into the last workgroup (three dead
    blocks) and x, u, dw are views ending exactly at the end of their own 2 MiB-rounded
    allocations, so any read past them leaves the allocation; the dots must agree with
    sum_j (sigma dw)_j G_j formed from the unfused forward's G within f32 rounding."""
    set_floatx("float32")
    cfg = full_config(name, d, N=8, hidden=(200, 200, 200), dtype="float32")
    bp = getattr(peq, name)(cfg.eqn_config)
    net = psol.DeepNN(cfg, "critic_grad", torch.Generator().manual_seed(4), torch.float32, "cuda")
    view = net.mlp_view()
    R = 64 * 9 + 16  # the last workgroup holds 16 live rows and 48 dead ones
    gen = torch.Generator(device="cuda").manual_seed(9)

    def at_end(cols):
        nbytes = R * cols * 4
        cap = (nbytes + 2 ** 21 - 1) // 2 ** 21 * 2 ** 21
        buf = torch.empty(cap, dtype=torch.uint8, device="cuda")
        v = buf[cap - nbytes:].view(torch.float32).view(R, cols)
        v.copy_(torch.randn(R, cols, generator=gen, device="cuda") * 0.5)
        return v, buf
    (x, bx), (u, bu), (dw, bd) = at_end(d), at_end(bp.control_dim), at_end(d)
    eqp = bp.params()
    gdot, _ = ops.mlp_rows_td1(eqp, view, x, u, dw, save=True)
    G, _ = ops.mlp_rows(view, x, save=True)
    sig = ops.equation_eval(eqp, _lib.EVAL_SIGMA, x, u)
    torch.cuda.synchronize()
    assert torch.isfinite(gdot).all()
    ref = torch.sum(sig * dw * G, 1)  # another summation order than the kernel's DPP tree
    assert torch.allclose(gdot, ref, rtol=1e-5, atol=1e-6)
    del bx, bu, bd


_BOUNDS_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "variants",
                           "libdpac_bounds.so")


@pytest.mark.parametrize("math", ["x3", "f32"])
@pytest.mark.parametrize("lib", ["main", "bounds"])
def test_row_kernels_ragged_rows_in_a_fresh_process_without_the_caching_allocator(lib, math):
    """VERDICT r05 item 6 / ADVICE r05: tests/bounds_check.py in a fresh process with
    PYTORCH_NO_CUDA_MEMORY_CACHING=1 (every buffer its own hipMalloc, each operand a view ending
    exactly at the end of its allocation), the row kernels' TD1 operands and prologue reads over
    ragged row counts — once with the shipped library (the loads go through row descriptors
    since round 6: a dead row reads 0) and once with the DPAC_CHECK_BOUNDS build, whose every
    row-indexed load checks its row and prints a violation line otherwise."""
    import subprocess
    import sys
    env = dict(os.environ, PYTORCH_NO_CUDA_MEMORY_CACHING="1", DPAC_MLP_MATH=math)
    if lib == "bounds":
        if not os.path.exists(_BOUNDS_LIB):
            pytest.skip("tools/variants/libdpac_bounds.so not built (make bounds)")
        env["DPAC_LIB"] = _BOUNDS_LIB
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-u", os.path.join(root, "tests", "bounds_check.py")], cwd=root, env=env,
                       capture_output=True, text=True, timeout=180)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "bounds_check ok" in r.stdout, out[-3000:]
    assert "dpac bounds violation" not in out, out[-3000:]
    print(r.stdout.strip().splitlines()[-1])
