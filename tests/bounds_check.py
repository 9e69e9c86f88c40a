"""Run in a fresh process by tests/test_gpu_td_fused.py: the
row kernels' TD1 operands and prologue reads over ragged row counts, with every operand a view
that ends exactly at the end of its own allocation and PyTorch's caching allocator off
(PYTORCH_NO_CUDA_MEMORY_CACHING=1: each buffer is its own hipMalloc), so a read past a row
array leaves mapped memory instead of landing in a neighbour inside a 20 MiB segment.  Under
the DPAC_CHECK_BOUNDS build (DPAC_LIB=tools/variants/libdpac_bounds.so, `make bounds`) every
row-indexed load also checks that its row is live and prints a "dpac bounds violation" line
otherwise.  DPAC_MLP_MATH=f32 in the environment takes the exact-f32 row kernels.
Prints "bounds_check ok" after every case ran and gave finite, consistent values."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deeppde_actorcritic_amd import _lib, ops  # noqa: E402
from deeppde_actorcritic_amd import equation as peq  # noqa: E402
from deeppde_actorcritic_amd import solver as psol  # noqa: E402
from deeppde_actorcritic_amd.config import set_floatx  # noqa: E402
from tests.helpers import full_config  # noqa: E402


def at_end(rows, cols, gen, scale=0.5):
    """A [rows, cols] float32 view ending exactly at the end of a 2 MiB-multiple allocation."""
    nbytes = rows * cols * 4
    cap = (nbytes + 2 ** 21 - 1) // 2 ** 21 * 2 ** 21
    buf = torch.empty(cap, dtype=torch.uint8, device="cuda")
    v = buf[cap - nbytes:].view(torch.float32).view(rows, cols)
    v.copy_(torch.randn(rows, cols, generator=gen, device="cuda") * scale)
    return v, buf


def main():
    set_floatx("float32")
    ncase = 0
    for name, d in (("LQR", 4), ("LQR_var", 10), ("LQR", 20)):
        cfg = full_config(name, d, N=8, hidden=(200, 200, 200), dtype="float32")
        bp = getattr(peq, name)(cfg.eqn_config)
        eqp = bp.params()
        net = psol.DeepNN(cfg, "critic_grad", torch.Generator().manual_seed(4), torch.float32, "cuda")
        params = [p.detach() for p in net.trainable_variables()]
        for R in (64 * 9 + 16, 64 * 3 + 1, 31, 32 * 5 + 7):  # dead 16-row blocks, ragged 32-row tails
            gen = torch.Generator(device="cuda").manual_seed(R)
            keep = []
            (x, b1), (u, b2), (dw, b3) = at_end(R, d, gen), at_end(R, bp.control_dim, gen), at_end(R, d, gen)
            (g_out, b4), (g_gdot, b5) = at_end(R, d, gen, 1.0 / R), at_end(R, 1, gen, 1.0 / R)
            keep += [b1, b2, b3, b4, b5]
            view = net.mlp_view()
            gdot, z, m = ops.mlp_rows_td1(eqp, view, x, u, dw, save=True, mask=True)
            G, _ = ops.mlp_rows(view, x, save=True)
            sig = ops.equation_eval(eqp, _lib.EVAL_SIGMA, x, u)
            g1 = ops.row_mlp_backward_td1(eqp, net.bn_rs, params, x, z, u, dw, g_gdot.view(R), True, mask=m)
            gx, g2 = ops.row_mlp_backward(net.bn_rs, params, x, z, g_out, True, True)
            torch.cuda.synchronize()
            ref = torch.sum(sig * dw * G, 1)
            assert torch.isfinite(gdot).all() and torch.allclose(gdot, ref, rtol=1e-5, atol=1e-6), (name, d, R)
            assert all(bool(torch.isfinite(t).all()) for t in g1 + g2 + [gx]), (name, d, R)
            ncase += 1
    print(f"bounds_check ok: {ncase} cases, MLP_MATH={ops.MLP_MATH}, lib={_lib.LIB_PATH}", flush=True)


if __name__ == "__main__":
    main()
