#!/usr/bin/env python3
"""Time the row-parallel MLP kernels at the critic G network's shape (R = N*B rows) with
split-fp16 MFMA (DPAC_MLP_MATH=x3) and exact f32 MFMA: forward with saves, the fused-TD1
forward, and the backward chain (dpac_mlp_rows_bwd); with --pg also the parameter gradients.

    python tools/probe_x3.py [R] [f32,x3] [--pg]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=20):
    for _ in range(3):
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
    argv = [a for a in sys.argv if not a.startswith("--")]
    R = int(argv[1]) if len(argv) > 1 else 204800
    from deeppde_actorcritic_amd import ops, _lib
    from deeppde_actorcritic_amd import solver as psol
    from deeppde_actorcritic_amd import equation as peq
    from deeppde_actorcritic_amd.config import set_floatx
    from tests.helpers import full_config
    set_floatx("float32")
    cfg = full_config("LQR", 20, hidden=(200, 200, 200), dtype="float32")
    eqp = peq.LQR(cfg.eqn_config).params()
    net = psol.DeepNN(cfg, "critic_grad", torch.Generator().manual_seed(0), torch.float32, "cuda")
    x = torch.randn(R, 20, device="cuda") * 0.5
    u = torch.randn(R, 20, device="cuda") * 0.5
    dw = torch.randn(R, 20, device="cuda")
    g = torch.randn(R, 20, device="cuda") * 1e-3
    flop = 2 * R * (20 * 200 + 2 * 200 * 200 + 200 * 20)
    params = [p.detach() for p in net.trainable_variables()]
    maths = argv[2].split(",") if len(argv) > 2 else ["f32", "x3"]
    for math in maths:
        ops.MLP_MATH = math
        view = net.mlp_view()
        _, z = ops.mlp_rows(view, x, save=True)
        L, gam, bet, Ws, b = ops._split_params(params)
        bview, wt, wt_km = ops.mlp_prepare(gam, bet, Ws, b, False, True)
        G = torch.empty(R, sum(bview.widths), device="cuda")
        import ctypes

        def bwd():
            _lib.call("dpac_mlp_rows_bwd", _lib.F32, R, ctypes.byref(bview.struct), ops._ptr_array(wt),
                      ops._ptr_array(wt_km), ops._ptr(z), ops._ptr(g), ops._ptr(G), None, ops._stream(x))
        _, _, mask = ops.mlp_rows(view, x, save=True, mask=True)

        def bwd_masked():
            _lib.call("dpac_mlp_rows_bwd_masked", _lib.F32, R, ctypes.byref(bview.struct), ops._ptr_array(wt),
                      ops._ptr_array(wt_km), ops._ptr(z), ops._ptr(mask), ops._ptr(g), ops._ptr(G), None,
                      ops._stream(x))
        res = {"fwd": timeit(lambda: ops.mlp_rows(view, x, save=False)),
               "fwd_saves": timeit(lambda: ops.mlp_rows(view, x, save=True)),
               "fwd_saves_mask": timeit(lambda: ops.mlp_rows(view, x, save=True, mask=True)),
               "fwd_td1_saves": timeit(lambda: ops.mlp_rows_td1(eqp, view, x, u, dw, save=True)),
               "fwd_td1_saves_mask": timeit(lambda: ops.mlp_rows_td1(eqp, view, x, u, dw, save=True, mask=True)),
               "bwd_chain": timeit(bwd)}
        if mask is not None:
            res["bwd_chain_masked"] = timeit(bwd_masked)
        if "--pg" in sys.argv:  # the parameter gradients (every layer + the chunk reduce)
            bwd()
            res["param_grads"] = timeit(lambda: ops.mlp_param_grads(view, x, z, G, params))
        for k, ms in res.items():
            print(json.dumps({"math": math, "R": R, "what": k, "us": ms * 1e3,
                              "TFLOPs_f32_equiv": flop / ms / 1e9}), flush=True)


if __name__ == "__main__":
    main()
