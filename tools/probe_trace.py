#!/usr/bin/env python3
"""Phase timing of the fused NN rollout and the BPTT kernel from a -DDPAC_NN_TRACE=1 build
(GPU only): workgroup 0 records the shader clock at fixed points of its first 64 steps
(NN_MARK in dpac_rollout_nn.h / dpac_rollout_nn_bwd.h).  Prints, per point, the mean
cycles since the step's first mark, for every wavefront.

    DPAC_LIB=tools/variants/libdpac_trace.so python tools/probe_trace.py --B 2048 --N 100
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FWD_POINTS = {0: "top", 10: "l0 A", 11: "l0 mfma", 12: "l1 mfma (x3)", 13: "l2 mfma (x3)", 1: "l0 done", 2: "l0 bar", 3: "l1 done", 4: "l1 bar", 5: "l2 done", 6: "l2 bar",
              7: "l3 done", 8: "l3 bar", 15: "step done"}
BWD_POINTS = {0: "top", 12: "l1 mfma (x3)", 13: "l2 mfma (x3) / end", 1: "vjp done", 2: "vjp bar", 3: "l3 done", 4: "l3 bar", 5: "l2 done", 6: "l2 bar",
              7: "l1 done", 8: "l1 bar", 9: "l0 done", 10: "l0 bar", 13: "end", 14: "end bar"}


def table(lib, nwaves, points, steps, rev=False):
    buf = np.zeros(64 * 16 * 16, dtype=np.uint32)
    assert lib.dpac_debug_trace(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(buf.nbytes)) == 0
    tr = buf.reshape(64, 16, 16).astype(np.int64)
    out = {}
    for w in range(nwaves):
        row = {}
        for p, name in points.items():
            d = (tr[steps, w, p] - tr[steps, 0, 0]) & 0xFFFFFFFF
            d = np.where(d > 2 ** 31, d - 2 ** 32, d)
            row[name] = float(np.median(d))
        out[f"wave{w}"] = row
    a, b = (steps, steps + 1) if rev else (steps + 1, steps)
    nxt = (tr[a, 0, 0] - tr[b, 0, 0]) & 0xFFFFFFFF
    out["step_cycles"] = float(np.median(nxt))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--N", type=int, default=100)
    a = ap.parse_args()
    from deeppde_actorcritic_amd import _lib, ops
    from deeppde_actorcritic_amd import equation as peq
    from deeppde_actorcritic_amd import solver as psol
    from deeppde_actorcritic_amd.config import set_floatx
    from tests.helpers import full_config
    lib = _lib.load()
    lib.dpac_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    set_floatx("float32")
    B, N = a.B, a.N
    cfg = full_config("LQR", 20, N=N, hidden=(200, 200, 200), batch=B, dtype="float32")
    bsde = peq.LQR(cfg.eqn_config)
    net = psol.DeepNN(cfg, "actor", torch.Generator().manual_seed(0), torch.float32, "cuda")
    eqp = bsde.params()
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=1, dtype=torch.float32, device="cuda")
    sch = _lib.SCHEME_ADAPTIVE
    y, disc, xN, saved = ops.actor_rollout_saves(eqp, sch, x0, dw, 0.2, N, net)
    torch.cuda.synchronize()
    steps = np.arange(8, 62)
    res = {"B": B, "N": N, "fwd": table(lib, 8, FWD_POINTS, steps)}
    x, u, dwc, z, flag, disc_t, mask = saved[:7]
    params = net.trainable_variables()
    L = 3
    gam, bet, Ws, b = params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]
    widths = [Ws[0].shape[0]] + [w.shape[1] for w in Ws]
    view, wt, wt_km = ops.mlp_prepare([p.detach() for p in gam], [p.detach() for p in bet],
                                      [p.detach() for p in Ws], b.detach(), False, True)
    g_y = torch.full_like(y, 1.0 / B)
    ops._bptt_fused(eqp, sch, 0.2, N, L, x, u, dwc, z, flag, disc_t, view, wt, wt_km, widths,
                    torch.randn_like(xN) / B, torch.rand_like(y) / B, g_y, mask)
    torch.cuda.synchronize()
    # the BPTT walks t = N-1 .. 0: steps 8..61 are its last ones
    res["bwd"] = table(lib, 10, BWD_POINTS, steps, rev=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
