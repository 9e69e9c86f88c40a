#!/usr/bin/env python3
"""Time the critic's G network + TD1 assembly split (G written, dpac_mlp_rows_fwd +
dpac_td_assemble_fwd; backward dpac_td_assemble_bwd + dpac_mlp_rows_bwd) against the
fused path (dpac_mlp_rows_fwd_td1 + DPAC_TD1_GDOT; backward
dpac_td_assemble_bwd_gdot + dpac_mlp_rows_bwd_td1) at lqr_d20's shape (N=100, B=2048
or 4096, 3x200 hidden, fp32), on a real rollout.  Parameter gradients are the same
call in both paths and are left out.

    python tools/probe_td_fused.py [B ...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deeppde_actorcritic_amd import _lib, ops  # noqa: E402
from deeppde_actorcritic_amd import equation as peq  # noqa: E402
from deeppde_actorcritic_amd import solver as psol  # noqa: E402
from deeppde_actorcritic_amd.config import set_floatx  # noqa: E402
from tests.helpers import full_config  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000.0  # us


def main():
    set_floatx("float32")
    for B in [int(a) for a in sys.argv[1:]] or [2048, 4096]:
        N = 100
        cfg = full_config("LQR", 20, N=N, hidden=(200, 200, 200), batch=B, valid=B, dtype="float32")
        bp = peq.LQR(cfg.eqn_config)
        sp = psol.ActorCriticSolver(cfg, bp, seed=1, sampler="device", graphs=False)
        data = sp.sample(B, N)
        x, dt, coef, u = bp.rollout("adaptive", data.x0, data.dw, 0.2, N, cheat=True)
        eqp = bp.params()
        net = sp.model_critic.NN_value_grad
        view = net.mlp_view()
        params = [p.detach() for p in net.trainable_variables()]
        L, gam, bet, Ws, b = ops._split_params(params)
        bview, wt, wt_km = ops.mlp_prepare(gam, bet, Ws, b, False, True)
        rows = x[:N].reshape(N * B, -1)
        u_rows, dw_rows = u.reshape(N * B, -1), data.dw.reshape(N * B, -1)
        g_y = torch.randn(B, device="cuda")
        R = N * B
        Gbuf = torch.empty(R, sum(view.widths), device="cuda")
        G, z = ops.mlp_rows(view, rows, save=True)

        def split_fwd():
            G, _ = ops.mlp_rows(view, rows, save=True)
            ops.td_assemble(eqp, _lib.TD1, x, u, data.dw, dt, coef, G.view(N, B, -1))

        def fused_fwd():
            gd, _ = ops.mlp_rows_td1(eqp, view, rows, u_rows, dw_rows, save=True)
            ops.td_assemble_gdot(eqp, x, u, dt, coef, gd.view(N, B))

        def split_bwd():
            gG = ops.td_assemble_bwd(eqp, x, u, data.dw, dt, coef, g_y)
            ops.call("dpac_mlp_rows_bwd", _lib.F32, R, ops.ctypes.byref(bview.struct),
                     ops._ptr_array(wt), ops._ptr_array(wt_km), ops._ptr(z), ops._ptr(gG),
                     ops._ptr(Gbuf), None, ops._stream(rows))

        def fused_bwd():
            gg = ops.td_assemble_bwd_gdot(eqp, dt, coef, g_y)
            ops.call("dpac_mlp_rows_bwd_td1", ops.ctypes.byref(eqp), _lib.F32, R,
                     ops.ctypes.byref(bview.struct), ops._ptr_array(wt), ops._ptr_array(wt_km),
                     ops._ptr(z), ops.ctypes.c_void_p(rows.data_ptr()), rows.stride(0),
                     ops._ptr(u_rows), ops._ptr(dw_rows), ops._ptr(gg), ops._ptr(Gbuf), None,
                     ops._stream(rows))

        out = {"B": B, "N": N, "rows": R}
        for name, fn in (("split_fwd", split_fwd), ("fused_fwd", fused_fwd),
                         ("split_bwd", split_bwd), ("fused_bwd", fused_bwd),
                         ("split_fwd_again", split_fwd), ("fused_fwd_again", fused_fwd)):
            out[name + "_us"] = round(timed(fn), 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
