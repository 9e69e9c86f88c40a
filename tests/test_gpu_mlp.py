"""dpac_mlp_param_grads (DeepNN parameter gradients over independent rows, the
Dense/BatchNormalization gradient ops of solver.py:227-278 under the tape of
solver.py:88,95) against a plain PyTorch float64 statement of the same sums, and
inside the actor's BPTT against the PyTorch product path.

Tolerances: float64 |a-b| <= 1e-11 (1+|b|) (only the summation order differs);
float32 vs the float64 reference: 2e-5 (1+|b|) relative to the largest entry.
"""
import numpy as np
import pytest
import torch

from deeppde_actorcritic_amd import _lib, ops
from deeppde_actorcritic_amd import equation as peq
from deeppde_actorcritic_amd.config import set_floatx
from deeppde_actorcritic_amd import solver as psol
from tests.helpers import full_config, rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda"


def random_net(widths, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    L = len(widths) - 2
    mk = lambda *s: (torch.rand(*s, generator=g, dtype=torch.float64) - 0.5).to(dtype).to(DEV)
    scales = [mk(w) + 0.7 for w in widths]
    shifts = [mk(w) for w in widths]
    Ws = [mk(widths[i], widths[i + 1]) for i in range(L + 1)]
    b = mk(widths[-1])
    return scales, shifts, Ws, b


def reference_grads(widths, scales, shifts, Ws, b, rs, x, z, G):
    """The sums of include/dpac.h dpac_mlp_param_grads, in float64 PyTorch."""
    f = lambda t: t.double()
    L = len(widths) - 2
    zo = [0]
    for w in widths[1:]:
        zo.append(zo[-1] + w)
    go = [0]
    for w in widths:
        go.append(go[-1] + w)
    zl = [None] + [f(z[:, zo[i - 1]:zo[i]]) for i in range(1, L + 2)]
    Gl = [f(G[:, go[i]:go[i + 1]]) for i in range(L + 2)]
    s = [f(t) for t in scales]
    sh = [f(t) for t in shifts]
    zin = [f(x)] + zl[1:L + 1] + [zl[L + 1] + f(b)]
    dgam = [rs * torch.sum(Gl[i] * zin[i], 0) for i in range(L + 2)]
    dbet = [torch.sum(Gl[i], 0) for i in range(L + 2)]
    A = [sh[0] + f(x) * s[0]]
    for i in range(1, L + 1):
        y = sh[i] + zl[i] * s[i]
        A.append(y + torch.relu(y))
    dW = [A[i].t() @ (Gl[i + 1] * s[i + 1]) for i in range(L + 1)]
    db = torch.sum(Gl[L + 1] * s[L + 1], 0)
    return dgam + dbet + dW + [db]


@pytest.mark.parametrize("widths,R", [
    ((20, 200, 200, 200, 20), 20000),      # the lqr_d20 networks, many chunks
    ((20, 200, 200, 200, 21), 777),        # Eikonal actor head, ragged rows
    ((5, 256, 256, 256, 256, 1), 3001),    # 4 hidden layers at the width limit, critic V head
    ((4, 7, 2), 1),                        # one row, tiny widths
    ((10, 48, 130, 33, 10), 4099)])        # widths that split MFMA tiles and column groups
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_param_grads_vs_torch(widths, R, dtype):
    scales, shifts, Ws, b = random_net(widths, dtype, seed=len(widths) + R)
    g = torch.Generator().manual_seed(R)
    rnd = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64).to(dtype).to(DEV)
    x = rnd(R, widths[0])
    z = rnd(R, sum(widths[1:]))
    G = rnd(R, sum(widths))
    view = ops.MlpView(scales, shifts, Ws, b, False)
    like = scales + shifts + Ws + [b]
    rs = ops.bn_rs_host(dtype)
    got = ops.mlp_param_grads(view, x, z, G, like)
    ref = reference_grads(widths, scales, shifts, Ws, b, rs, x, z, G)
    tol = 1e-11 if dtype == torch.float64 else 2e-5
    for a, r in zip(got, ref):
        assert a.shape == r.shape
        err = float((a.double() - r).abs().max() / (1 + r.abs().max()))
        assert err <= tol, (a.shape, err)


@pytest.mark.parametrize("widths,R", [
    ((20, 200, 200, 200, 20), 20000),      # the lqr_d20 networks, many chunks
    ((20, 200, 200, 200, 21), 777),        # Eikonal actor head, ragged rows
    ((5, 256, 256, 256, 256, 1), 3001),    # 16-tile inputs: those layers take the f32 kernel
    ((4, 7, 2), 1),                        # one row; the input layer into 7 takes the f32 kernel
    ((10, 48, 130, 33, 10), 4099),         # widths that split MFMA tiles and column groups
    ((12, 52, 100, 36, 8), 1234),          # merged-group kernel at other widths (k_param_grads_x3w)
    ((20, 200, 200, 200, 20), 204800)])    # the lqr_d20 critic G network's N*B rows
@pytest.mark.parametrize("gscale", [1.0, 1e-6, "ramp"])
def test_param_grads_split_fp16_vs_torch(widths, R, gscale, monkeypatch):
    """The split-fp16 parameter-gradient kernel (dpac_mlp_grad_x3.h, selected by a view that
    carries weight_x3 images) against the float64 sums and the exact-f32 kernel on the same
    inputs, per tensor within 2e-5 of its largest entry (the f32 kernel's bound) and within
    4x the f32 kernel's error + 5e-6 (the BN sums are plain f32 sums in both kernels, in
    another order: cancelling sums of a few thousand rows differ by a few e-6); for O(1)
    gradients, for gradients of 1e-6 scale (fp16-subnormal without the kernel's per-column
    scale) and for a ramp over rows from 1e-9 to 1 (each column's running exponent rises
    sub-chunk after sub-chunk: accumulator rescaling)."""
    if R == 204800 and gscale != 1.0:
        pytest.skip("one scale at full size")
    scales, shifts, Ws, b = random_net(widths, torch.float32, seed=len(widths) + R)
    g = torch.Generator().manual_seed(R)
    rnd = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64).to(torch.float32).to(DEV)
    x = rnd(R, widths[0])
    z = rnd(R, sum(widths[1:]))
    G = rnd(R, sum(widths))
    if gscale == "ramp":
        G = G * torch.logspace(-9, 0, R, dtype=torch.float64).to(torch.float32).to(DEV).unsqueeze(1)
    else:
        G = G * gscale
    view = ops.MlpView(scales, shifts, Ws, b, False, weights_x3=[_x3_image(W) for W in Ws])
    like = scales + shifts + Ws + [b]
    rs = ops.bn_rs_host(torch.float32)
    monkeypatch.delenv("DPAC_PG_X3", raising=False)
    got = ops.mlp_param_grads(view, x, z, G, like)
    monkeypatch.setenv("DPAC_PG_X3", "0")
    f32 = ops.mlp_param_grads(view, x, z, G, like)
    ref = reference_grads(widths, scales, shifts, Ws, b, rs, x, z, G)
    worst = 0.0
    for a, a32, r in zip(got, f32, ref):
        assert a.shape == r.shape
        top = float(r.abs().max())
        err = float((a.double() - r).abs().max()) / (top + 1e-300)
        err32 = float((a32.double() - r).abs().max()) / (top + 1e-300)
        worst = max(worst, err)
        assert err <= 2e-5 and err <= 4 * err32 + 5e-6, (a.shape, err, err32)
    print(f"\n[x3 param grads {widths} R={R} G~{gscale}] max rel err {worst:.2e}")


@pytest.mark.parametrize("widths,R", [
    ((20, 200, 200, 200, 20), 20000),      # the lqr_d20 networks
    ((20, 200, 200, 200, 20), 777),        # ragged: the last chunk ends inside a sub-chunk
    ((12, 52, 100, 36, 8), 1234),          # 4- and 7-tile inputs, 100- and 36-column outputs
    ((8, 64, 40, 12), 999)])               # a one-tile input layer, a 12-column output layer
@pytest.mark.parametrize("gscale", [1.0, "ramp"])
@pytest.mark.parametrize("kern", ["w", "d"])
def test_param_grads_merged_group_kernel_bitwise(widths, R, gscale, kern, monkeypatch):
    """The merged-group split-fp16 kernel (k_param_grads_x3w: one 256-column group, operand
    rows by LDS-DMA; for the input layer, the hidden layers with more than 32 inputs and the
    narrow output layer) forms the same products in the same order as the earlier kernels
    (DPAC_PGX_W=0: two 128-column groups, or 8 waves over the row tiles for <= 32 columns): the
    gradients, BN_0's sums included, are bitwise equal, column rescaling included (ramp).
    kern (DPAC_PGW_KERNEL): the 16-wavefront kernel (w) or its double-buffered 8-wavefront form
    k_param_grads_x3d (d, round 6), which must also equal w bit for bit."""
    monkeypatch.setenv("DPAC_PGW_KERNEL", kern)
    scales, shifts, Ws, b = random_net(widths, torch.float32, seed=3 * R + len(widths))
    g = torch.Generator().manual_seed(R + 1)
    rnd = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64).to(torch.float32).to(DEV)
    x, z, G = rnd(R, widths[0]), rnd(R, sum(widths[1:])), rnd(R, sum(widths))
    if gscale == "ramp":
        G = G * torch.logspace(-9, 0, R, dtype=torch.float64).to(torch.float32).to(DEV).unsqueeze(1)
    view = ops.MlpView(scales, shifts, Ws, b, False, weights_x3=[_x3_image(W) for W in Ws])
    like = scales + shifts + Ws + [b]
    monkeypatch.delenv("DPAC_PG_X3", raising=False)
    monkeypatch.delenv("DPAC_PGX_W", raising=False)
    monkeypatch.delenv("DPAC_PG_MERGE", raising=False)
    merged = ops.mlp_param_grads(view, x, z, G, like)
    monkeypatch.setenv("DPAC_PG_MERGE", "0")  # round 5: adjacent wide layers in one launch, or not
    single = ops.mlp_param_grads(view, x, z, G, like)
    monkeypatch.delenv("DPAC_PG_MERGE")
    for a, c in zip(merged, single):
        assert torch.equal(a, c), float((a - c).abs().max())
    monkeypatch.setenv("DPAC_PGX_W", "0")
    two = ops.mlp_param_grads(view, x, z, G, like)
    monkeypatch.setenv("DPAC_PG_X3", "0")
    f32 = ops.mlp_param_grads(view, x, z, G, like)
    assert any(not torch.equal(a, c) for a, c in zip(merged, f32)), "the split-fp16 kernels did not run"
    for a, c in zip(merged, two):
        assert torch.isfinite(a).all()
        assert torch.equal(a, c), float((a - c).abs().max())
    monkeypatch.delenv("DPAC_PG_X3")
    monkeypatch.delenv("DPAC_PGX_W")
    monkeypatch.setenv("DPAC_PGW_KERNEL", "d" if kern == "w" else "w")
    other = ops.mlp_param_grads(view, x, z, G, like)
    for a, c in zip(merged, other):
        assert torch.equal(a, c), float((a - c).abs().max())


@pytest.mark.parametrize("widths,R", [
    ((20, 200, 200, 200, 1), 6144),        # the lqr_d20 critic V network over 3 B rows (B = 2048)
    ((20, 200, 200, 200, 1), 777),         # ragged: the last chunk ends inside a sub-chunk
    ((4, 200, 200, 200, 1), 1),            # one row, a one-tile input layer
    ((10, 150, 200, 16), 3000)])           # a 10-tile input, a 16-column output
@pytest.mark.parametrize("gscale", [1.0, "ramp"])
def test_param_grads_segmented_launch_bitwise(widths, R, gscale, monkeypatch):
    """Round 6: for small row counts every layer of the 8-wavefront split-fp16 kernel runs in
    one launch (k_param_grads_x3_seg, each workgroup on its layer's segment of the grid); the
    gradients equal the one-launch-per-layer path (DPAC_PG_SEG=0) bit for bit."""
    scales, shifts, Ws, b = random_net(widths, torch.float32, seed=5 * R + len(widths))
    g = torch.Generator().manual_seed(R + 2)
    rnd = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64).to(torch.float32).to(DEV)
    x, z, G = rnd(R, widths[0]), rnd(R, sum(widths[1:])), rnd(R, sum(widths))
    if gscale == "ramp":
        G = G * torch.logspace(-9, 0, R, dtype=torch.float64).to(torch.float32).to(DEV).unsqueeze(1)
    view = ops.MlpView(scales, shifts, Ws, b, False, weights_x3=[_x3_image(W) for W in Ws])
    like = scales + shifts + Ws + [b]
    monkeypatch.delenv("DPAC_PG_X3", raising=False)
    monkeypatch.delenv("DPAC_PG_SEG", raising=False)
    seg = ops.mlp_param_grads(view, x, z, G, like)
    monkeypatch.setenv("DPAC_PG_SEG", "0")
    per_layer = ops.mlp_param_grads(view, x, z, G, like)
    monkeypatch.setenv("DPAC_PG_X3", "0")
    f32 = ops.mlp_param_grads(view, x, z, G, like)
    assert any(not torch.equal(a, c) for a, c in zip(seg, f32)), "the split-fp16 kernels did not run"
    for a, c in zip(seg, per_layer):
        assert torch.isfinite(a).all()
        assert torch.equal(a, c), float((a - c).abs().max())


@pytest.mark.parametrize("kern", ["w", "d"])
def test_param_grads_merged_group_high_address_words(kern, monkeypatch):
    """Regression test of round 4's address fault in k_param_grads_x3w (the operand rows'
    global_load_lds_dwordx4 takes a wave-uniform row address built from two readfirstlane
    halves; its first build sign-extended the low word, so any row whose address had bit 31
    set was loaded from an address 2^32·(2^32-1) off).  Operands are placed by hand inside
    one 4.5 GiB allocation: x and G where every row's low address word is >= 2^31, and z
    (read by LDS-DMA both as a layer's A and as the BN sums' operand) straddling a 4 GiB
    boundary, so its rows have low words just below 2^32 and then just above 0 with the high
    word carried.  The gradients must equal, bit for bit, those of the same kernel on
    ordinarily placed copies and those of the two-group kernels (DPAC_PGX_W=0), and lie within
    the split-fp16 tolerance of the exact-f32 kernel.  kern: DPAC_PGW_KERNEL (w, or d: round 6's
    double-buffered k_param_grads_x3d, whose z rows also move by LDS-DMA)."""
    monkeypatch.setenv("DPAC_PGW_KERNEL", kern)
    widths, R = (20, 200, 200, 200, 20), 20000
    scales, shifts, Ws, b = random_net(widths, torch.float32, seed=4242)
    g = torch.Generator().manual_seed(4243)
    rnd = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64).to(torch.float32).to(DEV)
    x, z, G = rnd(R, widths[0]), rnd(R, sum(widths[1:])), rnd(R, sum(widths))
    buf = torch.empty(int(4.5 * 2 ** 30), dtype=torch.uint8, device=DEV)
    base, span = buf.data_ptr(), buf.numel()

    def place(addr, t):
        off = addr - base
        n = t.numel() * 4
        assert off % 256 == 0 and 0 <= off and off + n <= span
        v = buf[off:off + n].view(torch.float32).view(t.shape)
        v.copy_(t)
        return v
    k = ((base + 2 ** 32 - 1) >> 32) << 32  # the first 4 GiB boundary inside the allocation
    assert base <= k < base + span
    zn = z.numel() * 4
    zh = place(k - ((zn // 2) // 256) * 256, z)  # straddles k
    hi_start = k - 2 ** 31 + 4096 if k - 2 ** 31 >= base else k + 2 ** 31 + 4096
    xh = place(hi_start, x)
    gh = place(hi_start + ((x.numel() * 4 + 4095) // 4096) * 4096, G)
    lo_words = [(t.data_ptr() + r * t.stride(0) * 4) & 0xFFFFFFFF for t in (xh, gh) for r in (0, R - 1)]
    assert all(w >= 2 ** 31 for w in lo_words)
    assert (zh.data_ptr() >> 32) != ((zh.data_ptr() + zn - 4) >> 32)
    view = ops.MlpView(scales, shifts, Ws, b, False, weights_x3=[_x3_image(W) for W in Ws])
    like = scales + shifts + Ws + [b]
    monkeypatch.delenv("DPAC_PG_X3", raising=False)
    monkeypatch.delenv("DPAC_PGX_W", raising=False)
    high = ops.mlp_param_grads(view, xh, zh, gh, like)
    plain = ops.mlp_param_grads(view, x, z, G, like)
    monkeypatch.setenv("DPAC_PGX_W", "0")
    two = ops.mlp_param_grads(view, xh, zh, gh, like)
    monkeypatch.setenv("DPAC_PG_X3", "0")
    f32 = ops.mlp_param_grads(view, xh, zh, gh, like)
    torch.cuda.synchronize()
    for a, p, c, e in zip(high, plain, two, f32):
        assert torch.isfinite(a).all()
        assert torch.equal(a, p), float((a - p).abs().max())
        assert torch.equal(a, c), float((a - c).abs().max())
        top = float(e.abs().max())
        assert float((a - e).abs().max()) <= 2e-5 * top + 1e-30
    del buf


def test_param_grads_strided_input_and_bad_args():
    widths = (20, 64, 20)
    scales, shifts, Ws, b = random_net(widths, torch.float64, seed=5)
    R = 300
    xfull = torch.randn(R, 32, dtype=torch.float64, device=DEV)
    x = xfull[:, :20]  # row stride 32
    z = torch.randn(R, 84, dtype=torch.float64, device=DEV)
    G = torch.randn(R, 104, dtype=torch.float64, device=DEV)
    view = ops.MlpView(scales, shifts, Ws, b, False)
    like = scales + shifts + Ws + [b]
    got = ops.mlp_param_grads(view, x, z, G, like)
    ref = reference_grads(widths, scales, shifts, Ws, b, ops.bn_rs_host(torch.float64), x, z, G)
    for a, r in zip(got, ref):
        assert rel_close(a.cpu(), r.cpu(), 1e-11)
    import ctypes
    lib = _lib.load()
    assert lib.dpac_mlp_param_grads(_lib.F64, 0, ctypes.byref(view.struct), 1.0, None, 20, None,
                                    None, None, 0, None, None) == _lib.DPAC_EINVAL
    ws = torch.empty(16, dtype=torch.uint8, device=DEV)
    out = torch.empty(10, dtype=torch.float64, device=DEV)
    rc = lib.dpac_mlp_param_grads(_lib.F64, R, ctypes.byref(view.struct), 1.0,
                                  ctypes.c_void_p(x.data_ptr()), 32, ctypes.c_void_p(z.data_ptr()),
                                  ctypes.c_void_p(G.data_ptr()), ctypes.c_void_p(ws.data_ptr()), 16,
                                  ctypes.c_void_p(out.data_ptr()), None)
    assert rc == _lib.DPAC_EINVAL and b"workspace too small" in lib.dpac_last_error()


@pytest.mark.parametrize("name,d,hidden,dtype,tol", [
    ("LQR", 20, (200, 200, 200), torch.float64, 1e-10), ("EKN", 5, (40, 40), torch.float64, 1e-10),
    ("VDP", 10, (32, 48, 24), torch.float64, 1e-10), ("LQR", 20, (200, 200, 200), torch.float32, 1e-4)])
def test_actor_bptt_param_grads_kernel_vs_torch(name, d, hidden, dtype, tol):
    B, N, T = 300, 16, 0.2
    cfg = full_config(name, d, N=N, hidden=hidden, scheme="adaptive",
                      dtype="float64" if dtype == torch.float64 else "float32")
    set_floatx("float64" if dtype == torch.float64 else "float32")
    ep = getattr(peq, name)(cfg.eqn_config)
    net = psol.DeepNN(cfg, "actor", torch.Generator().manual_seed(9), dtype, DEV)
    eqp = ep.params()
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=8, dtype=dtype, device=DEV)
    grads = {}
    try:
        for mode in ("torch", "kernel"):
            ops.PARAM_GRADS = mode
            y, disc, xN = ops.actor_rollout_nn(eqp, _lib.SCHEME_ADAPTIVE, x0, dw, T, N, net)
            grads[mode] = torch.autograd.grad(torch.mean(y + disc * torch.sum(xN * xN, 1)),
                                              net.trainable_variables())
    finally:
        ops.PARAM_GRADS = "kernel"
    for a, r in zip(grads["kernel"], grads["torch"]):
        assert rel_close(a.cpu(), r.cpu(), tol)


# ---------------------------------------------------------------------------
# dpac_mlp_rows_fwd / _bwd: DeepNN over independent rows (the critic's V and G
# networks) against the PyTorch statement of the same network.
# ---------------------------------------------------------------------------
def net_pair(AC, name, d, hidden, dtype, seed=4):
    cfg = full_config(name, d, hidden=hidden, dtype="float64" if dtype == torch.float64 else "float32")
    set_floatx("float64" if dtype == torch.float64 else "float32")
    return psol.DeepNN(cfg, AC, torch.Generator().manual_seed(seed), dtype, DEV)


def torch_path(fn):
    try:
        ops.ROW_MLP = "torch"
        return fn()
    finally:
        ops.ROW_MLP = "kernel"


ROW_CASES = [("critic_grad", "LQR", 20, (200, 200, 200), 20000), ("critic", "LQR", 20, (200, 200, 200), 6144),
             ("critic", "VDP", 4, (256, 256, 256, 256), 1), ("actor", "EKN", 5, (40, 7), 333),
             ("critic_grad", "LQR_var", 10, (48, 130, 33), 4099)]


@pytest.mark.parametrize("AC,name,d,hidden,R", ROW_CASES)
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_row_mlp_forward_and_saves(AC, name, d, hidden, R, dtype):
    net = net_pair(AC, name, d, hidden, dtype)
    x = torch.randn(R, d, dtype=dtype, device=DEV, generator=torch.Generator(DEV).manual_seed(R)) * 0.5
    with torch.no_grad():
        got = net(x)
        ref = torch_path(lambda: net(x))
        out, z = ops.mlp_rows(net.mlp_view(), x, save=True)
    tol = 1e-12 if dtype == torch.float64 else 2e-5
    assert got.shape == ref.shape
    assert rel_close(got.cpu(), ref.cpu(), tol)
    # the saves are the pre-BN dense outputs: recompute layer by layer in PyTorch
    rs, g, bt, W = net.bn_rs, net.bn_gamma, net.bn_beta, net.W
    y = torch.addcmul(bt[0], x, rs * g[0])
    zs, L = [], len(net.sizes) - 2
    for i in range(L + 1):
        zi = y @ W[i]
        zs.append(zi)
        y = torch.addcmul(bt[i + 1], zi if i < L else zi + net.b, rs * g[i + 1])
        if i < L:
            y = y + torch.relu(y)
    assert rel_close(z.cpu(), torch.cat(zs, 1).detach().cpu(), 1e-11 if dtype == torch.float64 else 1e-4)


@pytest.mark.parametrize("AC,name,d,hidden,R", ROW_CASES)
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_row_mlp_gradients(AC, name, d, hidden, R, dtype):
    net = net_pair(AC, name, d, hidden, dtype)
    gen = torch.Generator(DEV).manual_seed(R + 1)
    x = (torch.randn(R, d, dtype=dtype, device=DEV, generator=gen) * 0.5).requires_grad_(True)
    wgt = torch.randn(R, net.sizes[-1] - (1 if net.ekn_head else 0), dtype=dtype, device=DEV, generator=gen)

    def grads():
        loss = torch.sum(net(x) * wgt) / R
        return torch.autograd.grad(loss, [x] + net.trainable_variables())

    got = grads()
    ref = torch_path(grads)
    tol = 1e-10 if dtype == torch.float64 else 1e-4
    for a, r in zip(got, ref):
        assert a.shape == r.shape
        scale = float(r.abs().max())
        assert float((a - r).abs().max()) <= tol * (1 + scale)


def test_row_mlp_stacked_input_and_errors():
    """[S, R, d] input (the critic's G over all N steps) and argument checks."""
    net = net_pair("critic_grad", "LQR", 5, (24, 40), torch.float64)
    x = torch.randn(7, 33, 5, dtype=torch.float64, device=DEV)
    with torch.no_grad():
        got = net(x)
        ref = torch_path(lambda: net(x))
    assert got.shape == (7, 33, 5) and rel_close(got.cpu(), ref.cpu(), 1e-12)
    import ctypes
    lib = _lib.load()
    view = net.mlp_view()
    assert lib.dpac_mlp_rows_fwd(_lib.F64, 10, ctypes.byref(view.struct), None, 5, None, None,
                                 None) == _lib.DPAC_EINVAL
    assert lib.dpac_mlp_rows_fwd(_lib.F64, 10, ctypes.byref(view.struct),
                                 ctypes.c_void_p(x.data_ptr()), 3, ctypes.c_void_p(x.data_ptr()),
                                 None, None) == _lib.DPAC_EINVAL  # ldx < d


@pytest.mark.parametrize("hidden,R", [((200, 200, 200), 20000), ((200, 200, 200), 777), ((52, 100, 36), 1234),
                                      ((24, 40), 33)])
@pytest.mark.parametrize("td1", [False, True])
def test_row_backward_sign_mask_bitwise(hidden, R, td1, monkeypatch):
    """Round 5: the split-fp16 row forward records the hidden BN outputs'
    sign bits (dpac_mlp_rows_fwd[_td1]_masked) and the backward chain reads them instead of z
    (dpac_mlp_rows_bwd[_td1]_masked).  The mask's bits equal [shift_h + z_h * scale_h > 0]
    formed from the saved z (f32, the kernels' expression), and the masked backward's G,
    dL/dx and parameter gradients equal the z-reading backward's bit for bit (ragged row
    counts, widths that are not multiples of 4 or 16, the TD1 prologue)."""
    monkeypatch.setattr(ops, "MLP_MATH", "x3")
    cfg = full_config("LQR", 20, hidden=hidden, dtype="float32")
    net = psol.DeepNN(cfg, "critic_grad", torch.Generator().manual_seed(R), torch.float32, DEV)
    gen = torch.Generator(device=DEV).manual_seed(R + 7)
    x = torch.randn(R, 20, generator=gen, device=DEV) * 0.5
    params = [p.detach() for p in net.trainable_variables()]
    prep = net.mlp_prepared()
    view = prep[0]
    if td1:
        eqp = peq.LQR(cfg.eqn_config).params()
        u = torch.randn(R, 20, generator=gen, device=DEV)
        dw = torch.randn(R, 20, generator=gen, device=DEV)
        g_gdot = torch.randn(R, generator=gen, device=DEV) / R
        out, z, mask = ops.mlp_rows_td1(eqp, view, x, u, dw, save=True, mask=True)
        out0, z0 = ops.mlp_rows_td1(eqp, view, x, u, dw, save=True)
        res = {m: ops.row_mlp_backward_td1(eqp, net.bn_rs, params, x, z, u, dw, g_gdot, True, mask=m)
               for m in (None, mask)}
        chk = lambda a, b: [torch.equal(s, t) for s, t in zip(a, b)]
    else:
        g_out = torch.randn(R, 20, generator=gen, device=DEV) / R
        out, z, mask = ops.mlp_rows(view, x, save=True, mask=True)
        out0, z0 = ops.mlp_rows(view, x, save=True)
        res = {m: ops.row_mlp_backward(net.bn_rs, params, x, z, g_out, True, True, prepared=prep, mask=m)
               for m in (None, mask)}
        chk = lambda a, b: [torch.equal(a[0], b[0])] + [torch.equal(s, t) for s, t in zip(a[1], b[1])]
    torch.cuda.synchronize()
    assert mask is not None and mask.dtype == torch.uint8
    assert torch.equal(out, out0) and torch.equal(z, z0)  # writing the mask changes nothing else
    # the bits against the saved z (dpac.h: word ((h-1) nblk + b) 512 + 64 w + 16 q + r, bit
    # 4 (2 t + j) + e = [BN_h output of row 64 b + 16 t + r, feature 16 (w + 8 j) + 4 q + e > 0])
    widths = view.widths
    L = len(widths) - 2
    nblk = (R + 63) // 64
    assert mask.numel() == L * nblk * 512 * 4
    words = mask.view(torch.int32).view(L, nblk, 8, 4, 16).long() & 0xFFFFFFFF
    shift = (4 * (2 * torch.arange(4, device=DEV).view(4, 1, 1) + torch.arange(2, device=DEV).view(1, 2, 1))
             + torch.arange(4, device=DEV).view(1, 1, 4))  # [t, j, e]
    zo = 0
    for h in range(1, L + 1):
        w = widths[h]
        y = view.shifts[h] + z[:, zo:zo + w] * view.scales[h]
        pos = torch.zeros(nblk * 64, 256, dtype=torch.int64, device=DEV)
        pos[:R, :w] = (y > 0).long()
        pos = pos.view(nblk, 4, 16, 2, 8, 4, 4).permute(0, 4, 5, 2, 1, 3, 6)  # [b, w, q, r, t, j, e]
        expect = (pos << shift).sum((4, 5, 6))
        assert torch.equal(words[h - 1], expect), h
        zo += w
    assert all(chk(res[mask], res[None]))
    # the float64 path writes no mask
    net64 = psol.DeepNN(full_config("LQR", 20, hidden=hidden), "critic_grad", torch.Generator().manual_seed(1),
                        torch.float64, DEV)
    _, _, m64 = ops.mlp_rows(net64.mlp_view(), x.double(), save=True, mask=True)
    assert m64 is None


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_adam_kernel_matches_foreach_update(dtype):
    """dpac_adam_apply (one launch over a list of tensors, more than one launch's 32)
    gives bitwise the TF-form Adam update written as separate torch foreach ops on
    the GPU (solver.TFAdam's previous path), over three steps.  (Torch's CPU sqrt and
    division differ from the GPU's in the last bit, so the reference runs on the GPU.)"""
    from deeppde_actorcritic_amd import ops
    gen = torch.Generator().manual_seed(5)
    shapes = [(200, 200), (200,), (20, 1), (1,), (20, 200)] * 7  # 35 tensors
    vs = [torch.randn(s, generator=gen, dtype=dtype) for s in shapes]
    ref = [v.cuda() for v in vs]
    dev = [v.cuda() for v in vs]
    m_ref = [torch.zeros_like(v) for v in ref]
    s_ref = [torch.zeros_like(v) for v in ref]
    m_dev = [torch.zeros_like(v) for v in dev]
    s_dev = [torch.zeros_like(v) for v in dev]
    b1, b2, eps = 0.9, 0.999, 1e-8
    from deeppde_actorcritic_amd.solver import tf_adam_scalars
    for t in range(1, 4):
        gs = [torch.randn(s, generator=gen, dtype=dtype).cuda() for s in shapes]
        alpha, omb1, omb2 = tf_adam_scalars(1e-3, t, b1, b2, dtype)  # TF forms them in T
        torch._foreach_add_(m_ref, torch._foreach_mul(torch._foreach_sub(gs, m_ref), omb1))
        g2 = torch._foreach_mul(gs, gs)
        torch._foreach_add_(s_ref, torch._foreach_mul(torch._foreach_sub(g2, s_ref), omb2))
        den = torch._foreach_add(torch._foreach_sqrt(s_ref), eps)
        torch._foreach_sub_(ref, torch._foreach_div(torch._foreach_mul(m_ref, alpha), den))
        ops.adam_apply(dev, gs, m_dev, s_dev, alpha, b1, b2, eps)
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(dev + m_dev + s_dev, ref + m_ref + s_ref)):
        a, b = a.cpu(), b.cpu()
        bad = (a != b).nonzero()
        assert bad.numel() == 0, (i // len(shapes), i % len(shapes), bad[:3].tolist(),
                                  a[tuple(bad[0])].item(), b[tuple(bad[0])].item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_mlp_prepare_matches_tensor_ops(dtype):
    """dpac_mlp_prepare gives bitwise rs*gamma_i and (W_i * s_{i+1})^T as tensor ops form them."""
    widths = (20, 200, 130, 7, 21)
    gen = torch.Generator().manual_seed(11)
    gam = [torch.rand(w, generator=gen, dtype=dtype).cuda() for w in widths]
    bet = [torch.randn(w, generator=gen, dtype=dtype).cuda() for w in widths]
    Ws = [torch.randn(widths[i], widths[i + 1], generator=gen, dtype=dtype).cuda()
          for i in range(len(widths) - 1)]
    b = torch.zeros(widths[-1], dtype=dtype, device="cuda")
    view, wt, wt_km = ops.mlp_prepare(gam, bet, Ws, b, False, True)
    rs = torch.rsqrt(torch.tensor(1.0 + 1e-6, dtype=dtype)).cuda()
    s = [rs * g for g in gam]
    for a, e in zip(view.scales, s):
        assert torch.equal(a, e)
    for i, w in enumerate(wt):
        assert torch.equal(w, (Ws[i] * s[i + 1]).t().contiguous())
    assert view.widths == list(widths)
    k16 = lambda k: (k + 15) // 16 * 16
    if dtype == torch.float32:  # k-major images: W_i^T and W_i * s_{i+1}, zero-padded K
        L1 = len(Ws)
        km = view.km
        for i in range(L1):
            ref_f = torch.zeros(widths[i + 1], k16(widths[i]), dtype=dtype, device="cuda")
            ref_f[:, :widths[i]] = Ws[i].t()
            assert torch.equal(km[i], ref_f)
            ref_b = torch.zeros(widths[i], k16(widths[i + 1]), dtype=dtype, device="cuda")
            ref_b[:, :widths[i + 1]] = Ws[i] * s[i + 1]
            assert torch.equal(wt_km[i], ref_b)
    else:
        assert wt_km is None


def _x3_image(M):
    """The split-fp16 image (include/dpac.h dpac_mlp.weight_x3) of an operand M [K][cols]:
    hi = fp16(M), lo = fp16((M - hi) * 2^12), zero past K and cols, fragment-major
    [tile][chunk][hi|lo][lane][8]: element (t, c, p, l, e) holds column 16 t + l % 16 at
    k = 32 c + 8 (l // 16) + e."""
    K, n = M.shape
    nch, nt = (K + 31) // 32, (n + 15) // 16
    P = torch.zeros(nch * 32, nt * 16, dtype=torch.float32, device=M.device)
    P[:K, :n] = M
    hi = P.half()
    lo = ((P - hi.float()) * 4096.0).half()
    X = torch.stack([hi, lo]).reshape(2, nch, 4, 8, nt, 16)  # (p, c, q, e, t, r)
    return X.permute(4, 1, 0, 2, 5, 3).reshape(-1)         # (t, c, p, q, r, e)


def test_mlp_prepare_split_fp16_images(monkeypatch):
    """dpac_mlp_prepare's split-fp16 images: bitwise the split of W_i (forward) and of
    W_i * s_{i+1} (backward) formed with tensor ops; absent for float64 or DPAC_MLP_MATH=f32."""
    monkeypatch.setattr(ops, "MLP_MATH", "x3")
    widths = (20, 200, 130, 7, 21)
    gen = torch.Generator().manual_seed(12)
    gam = [torch.rand(w, generator=gen).cuda() for w in widths]
    bet = [torch.randn(w, generator=gen).cuda() for w in widths]
    Ws = [torch.randn(widths[i], widths[i + 1], generator=gen).cuda() * 0.1 for i in range(len(widths) - 1)]
    b = torch.zeros(widths[-1], device="cuda")
    view, wt, _ = ops.mlp_prepare(gam, bet, Ws, b, False, True)
    rs = torch.rsqrt(torch.tensor(1.0 + 1e-6)).cuda()
    s = [rs * g for g in gam]
    for i in range(len(Ws)):
        assert torch.equal(view.x3_fwd[i], _x3_image(Ws[i]))
        assert torch.equal(view.x3_bwd[i], _x3_image((Ws[i] * s[i + 1]).t()))
        assert view.struct.weight_x3[i] == view.x3_fwd[i].data_ptr()
        assert view.struct.weight_t_x3[i] == view.x3_bwd[i].data_ptr()
    v64, _, _ = ops.mlp_prepare([g.double() for g in gam], [t.double() for t in bet],
                                [w.double() for w in Ws], b.double(), False, True)
    assert v64.x3_fwd is None and v64.struct.weight_x3[0] is None
    monkeypatch.setattr(ops, "MLP_MATH", "f32")
    v32, _, _ = ops.mlp_prepare(gam, bet, Ws, b, False, True)
    assert v32.x3_fwd is None and v32.x3_bwd is None


@pytest.mark.parametrize("AC,name,d,hidden,R", ROW_CASES + [("critic_grad", "LQR", 20, (200, 200, 200), 63),
                                                          ("critic", "EKN", 20, (256, 17), 65)])
def test_row_mlp_split_fp16_vs_float64(AC, name, d, hidden, R, monkeypatch):
    """The split-fp16 row kernels (dpac_mlp_x3.h) against the float64 statement of the same
    network and the exact-f32 kernels: the forward, the saves, the input-gradient chain and
    every parameter gradient within the float32 kernels' tolerances, and no further from the
    float64 values than 2x the exact-f32 kernels' error (+ 1e-6)."""
    net = net_pair(AC, name, d, hidden, torch.float32)
    net64 = net_pair(AC, name, d, hidden, torch.float64)
    with torch.no_grad():
        for a, b in zip(net64.trainable_variables(), net.trainable_variables()):
            a.copy_(b.double())
    gen = torch.Generator(DEV).manual_seed(R + 3)
    x = torch.randn(R, d, device=DEV, generator=gen) * 0.5
    wgt = torch.randn(R, net.sizes[-1] - (1 if net.ekn_head else 0), device=DEV, generator=gen)

    def run(model, xx, w):
        xx = xx.clone().requires_grad_(True)
        out = model(xx)
        g = torch.autograd.grad(torch.sum(out * w) / R, [xx] + model.trainable_variables())
        return [out.detach()] + list(g)

    ref = torch_path(lambda: run(net64, x.double(), wgt.double()))
    errs = {}
    for math in ("f32", "x3"):
        monkeypatch.setattr(ops, "MLP_MATH", math)
        got = run(net, x, wgt)
        errs[math] = [float((a.double() - r).abs().max()) / (1 + float(r.abs().max())) for a, r in zip(got, ref)]
    print(f"\n[x3 rows {AC} {hidden} R={R}] max err f32 {max(errs['f32']):.2e} x3 {max(errs['x3']):.2e}")
    for e32, ex3 in zip(errs["f32"], errs["x3"]):
        assert ex3 <= 1e-4 and ex3 <= 2 * e32 + 1e-6
