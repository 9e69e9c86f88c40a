#!/usr/bin/env python3
"""Time the actor step's kernels one by one at lqr_d20's shape (GPU only): the fused
forward rollout with backward saves (k_rollout_nn), the BPTT (k_rollout_nn_bwd) and
the parameter gradients (k_param_grads), each over `reps` launches with HIP events on
the launch stream.

    python tools/probe_bptt.py [--B 2048] [--N 100] [--reps 10] [--dtype f32] [--only bwd]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MLP_FLOP_PER_ROW = 2 * (20 * 200 + 200 * 200 * 2 + 200 * 20)  # 176 000


def timed(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", default="2048")
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--only", default="fwd,bwd,pg")
    ap.add_argument("--eqn", default="LQR", help="LQR, VDP, EKN or LQR_var (d = 20)")
    ap.add_argument("--dump", default=None, help="save the forward's and the BPTT's outputs (torch.save) for a "
                                                 "bitwise A/B of two builds (tools/cmp_dumps.py)")
    a = ap.parse_args()
    from deeppde_actorcritic_amd import _lib, ops
    from deeppde_actorcritic_amd import equation as peq
    from deeppde_actorcritic_amd import solver as psol
    from deeppde_actorcritic_amd.config import set_floatx
    from tests.helpers import full_config
    dt_ = torch.float32 if a.dtype == "f32" else torch.float64
    set_floatx("float32" if a.dtype == "f32" else "float64")
    N = a.N
    only = a.only.split(",")
    for B in [int(v) for v in a.B.split(",")]:
        cfg = full_config(a.eqn, 20, N=N, hidden=(200, 200, 200), batch=B,
                          dtype="float32" if a.dtype == "f32" else "float64")
        bsde = getattr(peq, a.eqn)(cfg.eqn_config)
        net = psol.DeepNN(cfg, "actor", torch.Generator().manual_seed(0), dt_, "cuda")
        eqp = bsde.params()
        x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=1, dtype=dt_, device="cuda")
        sch = _lib.SCHEME_ADAPTIVE
        fwd = lambda: ops.actor_rollout_saves(eqp, sch, x0, dw, 0.2, N, net)
        y, disc, xN, saved = fwd()
        x, u, dwc, z, flag, disc_t, mask = saved[:7]
        params = net.trainable_variables()
        L = 3
        gam, bet, Ws, b = params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]
        widths = [Ws[0].shape[0]] + [w.shape[1] for w in Ws]
        view, wt, wt_km = ops.mlp_prepare([p.detach() for p in gam], [p.detach() for p in bet],
                                          [p.detach() for p in Ws], b.detach(), False, True)
        g_y = torch.full_like(y, 1.0 / B)
        torch.manual_seed(B)  # the same dL/d(disc), dL/dx_N in every process (--dump A/B)
        g_disc = torch.rand_like(y) / B
        g_xN = torch.randn_like(xN) / B
        bwd = lambda: ops._bptt_fused(eqp, sch, 0.2, N, L, x, u, dwc, z, flag, disc_t, view, wt, wt_km, widths,
                                      g_xN, g_disc, g_y, mask)
        G = bwd()
        Gall = ops.G_all(G)
        if a.dump:
            torch.save({"y": y, "disc": disc, "xN": xN, "x": x, "u": u, "z": z, "mask": mask, "G": Gall},
                       f"{a.dump}_{B}.pt")
        pg = lambda: ops.mlp_param_grads(view, x[:N].reshape(N * B, 20), z.reshape(N * B, -1),
                                         Gall.reshape(N * B, -1), params)
        out = {"eqn": a.eqn, "B": B, "N": N, "dtype": a.dtype}
        flop = MLP_FLOP_PER_ROW * B * N
        for name, fn, fl in (("fwd", fwd, flop), ("bwd", bwd, flop), ("pg", pg, flop)):
            if name not in only:
                continue
            ms = timed(fn, a.reps)
            out[name] = {"ms": ms, "us_per_step": ms * 1e3 / N, "TFLOPs": fl / (ms * 1e-3) / 1e12,
                         "frac_f32_mfma": fl / (ms * 1e-3) / 157.3e12}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
