#!/usr/bin/env python3
"""Phase timing of the split-fp16 row kernels from a -DDPAC_X3_TRACE=1 build (GPU only):
the first 256 workgroups record the shader clock at start (0), prologue done (1) and per
layer K loop done (2 + 2l) / barrier passed (3 + 2l).  Prints the median cycles since each
workgroup's start, per wave, for the forward (fwd_saves at R rows) and the backward chain.

    DPAC_LIB=tools/variants/libdpac_x3trace.so python tools/probe_x3_trace.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def table(lib, npts):
    buf = np.zeros(256 * 8 * 16, dtype=np.uint32)
    assert lib.dpac_debug_x3_trace(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(buf.nbytes)) == 0
    tr = buf.reshape(256, 8, 16).astype(np.int64)
    out = {}
    for w in range(8):
        d = (tr[:, w, :npts] - tr[:, 0, :1]) & 0xFFFFFFFF
        d = np.where(d > 2 ** 31, d - 2 ** 32, d)
        out[f"wave{w}"] = [float(v) for v in np.median(d, axis=0)]
    return out


def main():
    R = 204800
    from deeppde_actorcritic_amd import _lib, ops
    from deeppde_actorcritic_amd import solver as psol
    from deeppde_actorcritic_amd.config import set_floatx
    from tests.helpers import full_config
    lib = _lib.load()
    lib.dpac_debug_x3_trace.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    set_floatx("float32")
    cfg = full_config("LQR", 20, hidden=(200, 200, 200), dtype="float32")
    net = psol.DeepNN(cfg, "critic_grad", torch.Generator().manual_seed(0), torch.float32, "cuda")
    x = torch.randn(R, 20, device="cuda") * 0.5
    u = torch.randn(R, 20, device="cuda") * 0.5
    dw = torch.randn(R, 20, device="cuda")
    g = torch.randn(R, 20, device="cuda") * 1e-3
    from deeppde_actorcritic_amd import equation as peq
    eqp = peq.LQR(cfg.eqn_config).params()
    ops.MLP_MATH = "x3"
    view = net.mlp_view()
    for _ in range(3):  # the production forward of the critic's G network: TD1 dot fused, saves, mask
        _, z, m = ops.mlp_rows_td1(eqp, view, x, u, dw, save=True, mask=True)
    torch.cuda.synchronize()
    print(json.dumps({"fwd_td1": table(lib, 10)}), flush=True)
    for _ in range(3):  # the same network without saves, mask or TD1 (what the saves cost)
        ops.mlp_rows(view, x, save=False)
    torch.cuda.synchronize()
    print(json.dumps({"fwd_nosave": table(lib, 10)}), flush=True)
    for _ in range(3):  # saves only
        ops.mlp_rows(view, x, save=True)
    torch.cuda.synchronize()
    print(json.dumps({"fwd_saves": table(lib, 10)}), flush=True)
    params = [p.detach() for p in net.trainable_variables()]
    for _ in range(3):
        ops.row_mlp_backward(net.bn_rs, params, x, z, g, False, False, mask=m)
    torch.cuda.synchronize()
    print(json.dumps({"bwd": table(lib, 10)}), flush=True)


if __name__ == "__main__":
    main()
