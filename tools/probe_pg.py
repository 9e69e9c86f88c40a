#!/usr/bin/env python3
"""Time dpac_mlp_param_grads at the critic/actor training shape (R = N*B rows)."""
import json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deeppde_actorcritic_amd import ops  # noqa: E402
from tests.test_gpu_mlp import random_net  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 204800
    for dtype in (torch.float32, torch.float64):
        widths = (20, 200, 200, 200, 20)
        scales, shifts, Ws, b = random_net(widths, dtype, 1)
        x = torch.randn(R, 20, dtype=dtype, device="cuda")
        z = torch.randn(R, 620, dtype=dtype, device="cuda")
        G = torch.randn(R, 640, dtype=dtype, device="cuda")
        view = ops.MlpView(scales, shifts, Ws, b, False)
        like = scales + shifts + Ws + [b]
        for _ in range(3):
            ops.mlp_param_grads(view, x, z, G, like)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.mlp_param_grads(view, x, z, G, like)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        flop = 2 * R * sum(widths[i] * widths[i + 1] for i in range(4))
        byts = R * (20 + 620 + 640) * (4 if dtype == torch.float32 else 8)
        print(json.dumps({"dtype": str(dtype), "R": R, "ms": ms, "TFLOPs": flop / ms / 1e9,
                          "GBs_min": byts / ms / 1e6}), flush=True)


if __name__ == "__main__":
    main()
