"""GPU parity at the exact configuration bench.py times.

bench.py's headline launch: LQR d = c = 20, B = 4096, N = 200, T = 0.2 (dt = 1e-3), adaptive
scheme, analytic control (propagate_adaptive with cheat=True, /root/reference/equation.py:73-106),
dw drawn on the device by dpac_sample with seed 1234 (bench.RolloutSets' set 0), launched
through the same ctypes call as the bench.  The outputs are compared with the float64 oracle
run on the same x0 and dw (copied to the host, widened to float64):
  * float64 kernel: |a - b| <= 1e-12 (1 + |b|) on x and dt, coef exact;
  * float32 kernel: at most 1e-3 of trajectories may take a different exit decision, and on
    the matched ones |a - b| <= 1e-5 (1 + |b|) on x and dt.
The flip fraction and the errors are printed (pytest -s / -v shows them).
"""
import numpy as np
import pytest
import torch

import bench
from deeppde_actorcritic_amd import _lib
from deeppde_actorcritic_amd import equation as peq
from oracle import equations as oeq
from oracle import precision

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_bench_headline_rollout_vs_oracle(dtype):
    B, N, d, T = bench.B_PER_GPU, bench.HORIZON, bench.DIM, bench.T_TOTAL
    assert (B, N, d, T) == (4096, 200, 20, 0.2)
    torch.cuda.set_device(0)
    lib = _lib.load()
    eqp = peq.LQR(bench.lqr_config()).params()
    rs = bench.RolloutSets(lib, eqp, _lib.SCHEME_ADAPTIVE, dtype, B, N, d, 0, 1)
    rs.launcher(1)(0)
    torch.cuda.synchronize()
    x0, dw, x, dt, coef = rs.sets[0]
    # the oracle on the bench's own inputs, in the reference's precision
    precision.set_dtype(torch.float64)
    eo = oeq.LQR(bench.lqr_config())
    x0h = x0.double().cpu()
    dwh = dw.double().cpu().permute(1, 2, 0).contiguous()  # [N][B][d] -> the reference's [B][d][N]
    xr, dtr, cr = eo.propagate_adaptive(B, x0h, dwh, None, False, T, N, True)
    xr, dtr, cr = xr.numpy(), dtr.numpy(), cr.numpy()
    xg = x.double().cpu().permute(1, 2, 0).numpy()  # [N+1][B][d] -> [B][d][N+1]
    dtg, cg = dt.double().cpu().numpy(), coef.double().cpu().numpy()
    same = np.all(cg == cr, axis=1)
    flips = float(np.mean(~same))
    ex = np.abs(xg - xr) / (1 + np.abs(xr))
    edt = np.abs(dtg - dtr) / (1 + np.abs(dtr))
    exm, edtm = float(ex[same].max()), float(edt[same].max())
    print(f"bench shape {dtype}: flip fraction {flips:.2e} ({int((~same).sum())} of {B}); "
          f"matched max rel err x {exm:.2e}, dt {edtm:.2e}; "
          f"exited trajectories {int((cr[:, -1] == 0).sum())}, min dt / (T/N) {dtr.min() / (T / N):.3e}")
    if dtype == torch.float64:
        np.testing.assert_array_equal(cg, cr)
        assert float(ex.max()) <= 1e-12 and float(edt.max()) <= 1e-12
    else:
        assert flips <= 1e-3, f"{flips:.2e} of trajectories flipped an exit decision"
        assert exm <= 1e-5 and edtm <= 1e-5
