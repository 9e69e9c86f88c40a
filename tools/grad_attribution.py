#!/usr/bin/env python3
"""Per-tensor errors of the float32 production gradients against the float64 oracle tape
(the batch and networks of tests/test_gpu_fp32_production.py::
test_fp32_production_gradients_vs_oracle_tape), to attribute them: run once as shipped
(split-fp16 MLP products) and once with DPAC_MLP_MATH=f32 (every MLP product exact f32):

    python tools/grad_attribution.py LQR            # x3
    DPAC_MLP_MATH=f32 python tools/grad_attribution.py LQR

One JSON line per network: for every parameter tensor, max |a - b| / max |b| and max |b|."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deeppde_actorcritic_amd import ops  # noqa: E402
from tests import test_gpu_fp32_production as t  # noqa: E402
from tests.helpers import full_config  # noqa: E402


def per_tensor(gp, go, names):
    out = []
    for n, a, b in zip(names, gp, go):
        if b is None:
            continue
        a = a.detach().to("cpu", torch.float64)
        b = b.detach()
        top = float(b.abs().max())
        out.append({"tensor": n, "rel_err": float((a - b).abs().max()) / max(top, 1e-30), "max_abs": top})
    return out


def names_of(net_names, L=3):
    return ([f"{net_names}.gamma{i}" for i in range(L + 2)] + [f"{net_names}.beta{i}" for i in range(L + 2)]
            + [f"{net_names}.W{i}" for i in range(L + 1)] + [f"{net_names}.b"])


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "LQR"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1100
    N, T = 50, 0.2
    cfg = full_config(name, 20, N=N, hidden=(200, 200, 200), batch=B, scheme="adaptive", td="TD1",
                      dtype="float32")
    sp, so = t._pair(cfg, 5)
    np.random.seed(17)
    dc = so.bsde.sample_normal(B, N)
    da = so.bsde.sample_normal(B, N)
    keep_c, keep_a = t._matched(sp, so, dc, N, T), t._matched(sp, so, da, N, T)
    dc = tuple(a[keep_c] for a in dc)
    da = tuple(a[keep_a] for a in da)
    front = sp.critic_front(dc)
    gp_c = front[0] + sp.critic_G_back(front)
    go_c, _ = so.grad_critic(dc, False, False)
    gp_a = sp.actor_grads_from(sp.actor_forward(da))
    go_a, _ = so.grad_actor(da, False, False, False)
    crit = names_of("V") + names_of("G")
    for net, rows in (("critic", per_tensor(gp_c, go_c, crit)), ("actor", per_tensor(gp_a, go_a, names_of("u")))):
        rows.sort(key=lambda r: -r["rel_err"])
        print(json.dumps({"eqn": name, "mlp_math": ops.MLP_MATH, "net": net,
                          "max_rel_err": rows[0]["rel_err"], "worst5": rows[:5]}), flush=True)


if __name__ == "__main__":
    main()
