#!/usr/bin/env python3
"""Time dpac_mlp_rows_fwd / _bwd at the critic G network's shape (R = N*B rows)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 204800
    from deeppde_actorcritic_amd import ops
    from deeppde_actorcritic_amd import solver as psol
    from deeppde_actorcritic_amd.config import set_floatx
    from tests.helpers import full_config
    for dt_, name in ((torch.float32, "float32"), (torch.float64, "float64")):
        set_floatx(name)
        cfg = full_config("LQR", 20, hidden=(200, 200, 200), dtype=name)
        net = psol.DeepNN(cfg, "critic_grad", torch.Generator().manual_seed(0), dt_, "cuda")
        x = torch.randn(R, 20, dtype=dt_, device="cuda") * 0.5
        wgt = torch.randn(R, 20, dtype=dt_, device="cuda")
        view = net.mlp_view()
        fwd = lambda: ops.mlp_rows(view, x, save=True)

        def both():
            loss = torch.sum(ops.row_mlp(net, x) * wgt)
            return torch.autograd.grad(loss, net.trainable_variables())
        for label, fn in (("fwd_saves", fwd), ("fwd_bwd_grads", both)):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 10
            flop = 2 * R * (20 * 200 + 2 * 200 * 200 + 200 * 20)
            print(json.dumps({"dtype": name, "R": R, "what": label, "ms": ms,
                              "fwd_TFLOPs_equiv": flop / ms / 1e9}), flush=True)


if __name__ == "__main__":
    main()
