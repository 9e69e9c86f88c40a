"""Torch-facing wrappers of the libdpac C ABI (device-native layouts).

Layouts (HBM, step-major): x0/x_bdry [B, d]; x [N+1, B, d]; dw, G [N, B, d];
u [N, B, c]; dt, coef [B, N] (trajectory-major, the reference's own dt/coef
layout, equation.py:70,99); flags int32 [B]; y, disc [B].

Every op requires CUDA (ROCm) tensors and raises if libdpac or the GPU is
missing: there is no CPU path in the product.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import call

_DT = {torch.float32: _lib.F32, torch.float64: _lib.F64}


def _require_gpu(*tensors: torch.Tensor) -> None:
    _lib.load()
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise _lib.DpacUnavailable(
                "libdpac ops run on the GPU only; got a tensor on " f"{t.device}")


def _ptr(t):
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("libdpac needs contiguous tensors")
    return ctypes.c_void_p(t.data_ptr())


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _dtype_id(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"libdpac supports float32/float64, got {t.dtype}") from None


def _check_same(ref: torch.Tensor, *others):
    for o in others:
        if o is not None and (o.dtype != ref.dtype or o.device != ref.device):
            raise TypeError("all floating inputs must share dtype and device "
                            f"({ref.dtype}@{ref.device} vs {o.dtype}@{o.device})")


# ---------------------------------------------------------------------------
def sample(eqp, sample_type: int, num_sample: int, num_steps: int, seed: int,
           traj_offset: int = 0, dtype=torch.float32, device=None, want_dw=True, out=None):
    """On-device Philox sampler (equation.py:13-44 semantics, different stream).  out: existing
    (x0 [B,d], dw [N,B,d], x_bdry [B,d]) buffers to draw into (contiguous, the call's dtype)."""
    device = torch.device(device if device is not None else "cuda")
    if device.type != "cuda":
        raise _lib.DpacUnavailable("dpac_sample needs a GPU device")
    if device.index is None:  # "cuda": the current device, as torch.empty places it
        device = torch.device("cuda", torch.cuda.current_device())
    _lib.load()
    d = eqp.dim
    if out is not None:
        x0, dw, x_bdry = out
        shapes = ((num_sample, d), (num_steps, num_sample, d), (num_sample, d))
        for t, shp in zip((x0, dw, x_bdry), shapes):
            if tuple(t.shape) != shp or t.dtype != dtype or not t.is_contiguous() or t.device != device:
                raise ValueError(f"sample(out=): expected contiguous {dtype} {shp} on {device}")
    else:
        x0 = torch.empty(num_sample, d, dtype=dtype, device=device)
        x_bdry = torch.empty(num_sample, d, dtype=dtype, device=device)
        dw = torch.empty(num_steps, num_sample, d, dtype=dtype, device=device) if want_dw else None
    call("dpac_sample", ctypes.byref(eqp), sample_type, _DT[dtype], num_sample, num_steps,
         seed & 0xFFFFFFFFFFFFFFFF, traj_offset, _ptr(x0), _ptr(dw), _ptr(x_bdry), _stream(x0))
    return x0, dw, x_bdry


def rollout_analytic(eqp, scheme: int, x0: torch.Tensor, dw: torch.Tensor | None,
                     total_time: float, num_steps: int, *, seed: int = 0,
                     traj_offset: int = 0, sample_type: int = _lib.SAMPLE_NORMAL,
                     want_u: bool = False, cost_order: int | None = None, out=None):
    """Fused rollout with u = u_true (equation.py:46-106 with cheat=True).

    Returns (x [N+1,B,d], dt [B,N], coef [B,N], u [N,B,c] | None, y [B] | None,
    disc [B] | None).  dw=None draws increments in-kernel from the Philox stream.
    """
    _require_gpu(x0, dw)
    _check_same(x0, dw)
    B, d = x0.shape
    N = num_steps
    if dw is not None and tuple(dw.shape) != (N, B, d):
        raise ValueError(f"dw must be [N, B, d] = {(N, B, d)}, got {tuple(dw.shape)}")
    kw = dict(dtype=x0.dtype, device=x0.device)
    if out is None:
        x = torch.empty(N + 1, B, d, **kw)
        dt = torch.empty(B, N, **kw)
        coef = torch.empty(B, N, **kw)
    else:
        x, dt, coef = out
    u = torch.empty(N, B, eqp.control_dim, **kw) if want_u else None
    y = disc = None
    if cost_order is not None:
        y = torch.empty(B, **kw)
        disc = torch.empty(B, **kw)
    call("dpac_rollout_fwd", ctypes.byref(eqp), scheme, _dtype_id(x0), B, N, float(total_time),
         _ptr(x0.contiguous()), _ptr(dw), seed & 0xFFFFFFFFFFFFFFFF, traj_offset, sample_type,
         _ptr(x), _ptr(dt), _ptr(coef), _ptr(u), _lib.COST_CRITIC if cost_order is None
         else cost_order, _ptr(y), _ptr(disc), _stream(x0))
    return x, dt, coef, u, y, disc


class MlpView:
    """The actor MLP as dpac_rollout_nn_fwd reads it (include/dpac.h dpac_mlp).

    `tensors` keeps every device buffer the struct points to alive; all must be
    contiguous, on the GPU, in the rollout's dtype."""

    def __init__(self, scales, shifts, weights, bias, ekn_head: bool, weights_km=None,
                 weights_x3=None, weights_t_x3=None, status=None):
        L = len(weights) - 1
        if not 1 <= L <= _lib.MLP_MAX_HIDDEN:
            raise ValueError(f"the fused rollout supports 1..{_lib.MLP_MAX_HIDDEN} hidden layers, got {L}")
        self.tensors = [t.contiguous() for t in list(scales) + list(shifts) + list(weights) + [bias]]
        sc, sh = self.tensors[:L + 2], self.tensors[L + 2:2 * L + 4]
        ws, b = self.tensors[2 * L + 4:3 * L + 5], self.tensors[-1]
        m = _lib.Mlp()
        m.n_hidden, m.ekn_head = L, int(bool(ekn_head))
        m.width[0] = ws[0].shape[0]
        for i, w in enumerate(ws):
            m.width[i + 1] = w.shape[1]
            m.weight[i] = w.data_ptr()
        for i in range(L + 2):
            m.bn_scale[i], m.bn_shift[i] = sc[i].data_ptr(), sh[i].data_ptr()
        m.bias = b.data_ptr()
        self.km, self.x3_fwd, self.x3_bwd = weights_km, weights_x3, weights_t_x3
        self.halves = []
        if weights_km is not None:  # k-major images (dpac_mlp.weight_km), kept alive here
            self.tensors += list(weights_km)
            for i, w in enumerate(weights_km):
                m.weight_km[i] = w.data_ptr()
        for slot, imgs in (("weight_x3", weights_x3), ("weight_t_x3", weights_t_x3)):
            if imgs is not None:  # split-fp16 images (dpac_mlp.weight_x3 / weight_t_x3): kept
                self.halves += list(imgs)  # alive here, outside the same-dtype `tensors`
                for i, w in enumerate(imgs):
                    getattr(m, slot)[i] = w.data_ptr()
        self.status = status  # the split-fp16 range guard word (dpac_mlp.status), or None
        if status is not None:
            m.status = status.data_ptr()
        self.struct = m
        self.widths = [m.width[i] for i in range(L + 2)]

    def supported(self) -> bool:
        return max(self.widths) <= _lib.MLP_MAX_WIDTH

    def phase_struct(self, phase: int):
        """A copy of the struct with dpac_mlp.guard_phase = phase (dpac.h DPAC_GUARD_*)."""
        m = _lib.Mlp.from_buffer_copy(self.struct)
        m.guard_phase = phase
        return m

    @property
    def scales(self):
        return self.tensors[:len(self.widths)]

    @property
    def shifts(self):
        return self.tensors[len(self.widths):2 * len(self.widths)]


# "on": float networks also get the k-major weight images (dpac_mlp.weight_km) the fused
# rollout / BPTT read with 4 k per load; "off": the row-major path (test reference).
WEIGHT_KM = os.environ.get("DPAC_WEIGHT_KM", "on")
# Products of float networks: "x3" = split-fp16 MFMA (dpac_mlp.weight_x3: three
# v_mfma_f32_16x16x32_f16 per 32-k step, f32-accurate) in the kernels that
# have it (the row-parallel V / G networks); "f32" = v_mfma_f32_16x16x4_f32 everywhere.
MLP_MATH = os.environ.get("DPAC_MLP_MATH", "x3")
if MLP_MATH not in ("x3", "f32"):
    raise ValueError(f"DPAC_MLP_MATH must be 'x3' or 'f32', got {MLP_MATH!r}")


# The split-fp16 range guard (dpac.h dpac_mlp.status): every float view with split-fp16
# images carries its device's status word, so an operand outside the split range (|a| >= 2^15,
# inf, NaN) makes that launch, and every later one on the device, run the exact-f32 kernels.
# DPAC_X3_GUARD=0 passes no word (the unguarded kernels; timing comparisons only).
X3_GUARD = os.environ.get("DPAC_X3_GUARD", "1") != "0"
_X3_STATUS = {}


def x3_status(device) -> torch.Tensor:
    """The device's split-fp16 status word (int32 [1], sticky; never freed: captured HIP graphs
    keep its address)."""
    device = torch.device(device)
    key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
    st = _X3_STATUS.get(key)
    if st is None:
        st = _X3_STATUS[key] = torch.zeros(1, dtype=torch.int32, device=torch.device("cuda", key[1]))
    return st


def x3_fell_back(device="cuda") -> bool:
    """Whether a split-fp16 launch on `device` met an operand outside the split range (its
    launches, and every later one, then ran on the exact-f32 kernels).  Synchronises."""
    return bool(int(x3_status(device).item()) & _lib.X3_FELL_BACK)


# Deferred range-guard fallbacks (dpac.h dpac_mlp.guard_phase, round 6).  Inside
# deferred_fallbacks(sink) the guarded backward calls below (the actor's BPTT, the row backward
# chains, the parameter gradients) launch only their split-fp16 kernels (phase 1) and append to
# `sink` a callable that launches their guarded f32 fallbacks (phase 2) on the then-current
# stream.  The caller runs the sink, in order, once every phase-1 call's inputs are final and
# before any of their outputs is used: the solver captures it into one "redo" graph replayed
# after the actor's and G's gradient chains have joined, so the no-op fallbacks no longer sit
# between a chain's kernels waiting for CUs the other stream holds.  Only
# chains whose outputs reach the caller with no torch op in between may be deferred: a phase-2
# call rewrites its outputs, not what was computed from them.  The closures hold every tensor
# the calls read or write, so a captured graph's pool cannot reuse them.
_DEFER = None


@contextlib.contextmanager
def deferred_fallbacks(sink):
    """Defer the guarded fallbacks of the calls inside into `sink` (a list); None: no deferral."""
    global _DEFER
    prev, _DEFER = _DEFER, sink
    try:
        yield sink
    finally:
        _DEFER = prev


def _guarded_call(view: "MlpView", name: str, build):
    """call(name, *build(ref to a dpac_mlp)) for a guarded entry point: inline (phase 0), or,
    inside deferred_fallbacks, phase 1 now and phase 2 appended to the sink."""
    if _DEFER is None or view.status is None:
        call(name, *build(ctypes.byref(view.struct)))
        return
    s1, s2 = view.phase_struct(_lib.GUARD_SPLIT_ONLY), view.phase_struct(_lib.GUARD_FALLBACK_ONLY)
    call(name, *build(ctypes.byref(s1)))
    _DEFER.append(lambda: call(name, *build(ctypes.byref(s2))))


def x3_status_reset(device="cuda") -> None:
    """Clear the device's status word: the split-fp16 kernels run again.  Synchronises the device
    first: no guarded launch may be in flight (dpac.h)."""
    torch.cuda.synchronize(device)
    x3_status(device).zero_()
    torch.cuda.synchronize(device)


def _x3_halves(k, n):
    """Halves of a split-fp16 image with n columns over K = k (dpac.h weight_x3: 16-column
    tiles x 32-k chunks x 1024 halves)."""
    return (n + 15) // 16 * 1024 * ((k + 31) // 32)


def _k16(k):
    return (k + 15) // 16 * 16


def mlp_prepare(gam, bet, Ws, b, ekn: bool, want_wt: bool, want_km: bool = True):
    """A DeepNN's kernel operands from its raw variables in one dpac_mlp_prepare launch:
    (MlpView with BN scales s_i = rs*gamma_i, wt or None, wt_km or None) with wt[i] =
    (W_i * s_{i+1})^T [w_{i+1}, w_i], the weight_t operand of the backward kernels.
    Float networks also get k-major images (want_km, WEIGHT_KM): the view's forward
    images W_i^T and, with want_wt, wt_km[i] = (W_i * s_{i+1}) padded, the backward entry
    points' weight_t_km argument.  Bitwise the products `rs * gamma` and
    `(W * s).t()` as tensor ops."""
    ref = gam[0]
    _require_gpu(*gam, *Ws)
    widths = [Ws[0].shape[0]] + [w.shape[1] for w in Ws]
    L1 = len(Ws)
    kw = dict(dtype=ref.dtype, device=ref.device)
    km = want_km and WEIGHT_KM == "on" and ref.dtype == torch.float32
    x3 = MLP_MATH == "x3" and ref.dtype == torch.float32
    status = x3_status(ref.device) if (x3 and X3_GUARD) else None
    raw = MlpView(gam, bet, Ws, b, ekn, status=status)  # bn_scale slots point at the raw gammas
    S = torch.empty(sum(widths), **kw)
    nw = [widths[i] * widths[i + 1] for i in range(L1)]
    nk = [widths[i + 1] * _k16(widths[i]) for i in range(L1)]
    nt = [widths[i] * _k16(widths[i + 1]) for i in range(L1)]
    WT = torch.empty(sum(nw), **kw) if want_wt else None
    KM = torch.empty(sum(nk), **kw) if km else None
    TKM = torch.empty(sum(nt), **kw) if (km and want_wt) else None
    nx = [_x3_halves(widths[i], widths[i + 1]) for i in range(L1)]
    ny = [_x3_halves(widths[i + 1], widths[i]) for i in range(L1)]
    hk = dict(dtype=torch.float16, device=ref.device)
    X3 = torch.empty(sum(nx), **hk) if x3 else None
    TX3 = torch.empty(sum(ny), **hk) if (x3 and want_wt) else None
    call("dpac_mlp_prepare", _dtype_id(ref), ctypes.byref(raw.struct), bn_rs_host(ref.dtype),
         _ptr(S), _ptr(WT), _ptr(KM), _ptr(TKM), _ptr(X3), _ptr(TX3), _stream(ref))

    def split(buf, sizes, shapes):
        offs = np.cumsum([0] + sizes).tolist()
        return [buf[offs[i]:offs[i + 1]].view(*shapes[i]) for i in range(L1)]
    km_f = split(KM, nk, [(widths[i + 1], _k16(widths[i])) for i in range(L1)]) if km else None
    x3_f = split(X3, nx, [(nx[i],) for i in range(L1)]) if X3 is not None else None
    x3_b = split(TX3, ny, [(ny[i],) for i in range(L1)]) if TX3 is not None else None
    view = MlpView(list(torch.split(S, widths)), bet, Ws, b, ekn, km_f, x3_f, x3_b, status)
    wt = split(WT, nw, [(widths[i + 1], widths[i]) for i in range(L1)]) if want_wt else None
    wt_km = split(TKM, nt, [(widths[i], _k16(widths[i + 1])) for i in range(L1)]) \
        if TKM is not None else None
    return view, wt, wt_km


def rollout_nn(eqp, scheme: int, x0: torch.Tensor, dw: torch.Tensor, total_time: float,
               num_steps: int, mlp: MlpView, *, want_u: bool = True, cost_order: int | None = None,
               save: bool = False):
    """Fused rollout with u_t = actor MLP(x_t) (equation.py:46-106 with NN_control,
    solver.py:260-278), one launch of dpac_rollout_nn_fwd.

    Returns (x [N+1,B,d], dt [B,N], coef [B,N], u [N,B,c] | None, y | None, disc | None,
    saves | None) with saves = (z [N,B,Σ widths[1:]], flag [N,B] int32, disc_t [N,B], mask)
    and mask the hidden activations' sign bits [N,ceil(B/16),mask_tile_bytes] (uint8, dpac.h)
    where the kernel wrote them
    (the float 16-row fast path: dpac_rollout_nn_fwd_masked), else None."""
    _require_gpu(x0, dw, *mlp.tensors)
    _check_same(x0, dw, *mlp.tensors)
    B, d = x0.shape
    N = num_steps
    if tuple(dw.shape) != (N, B, d):
        raise ValueError(f"dw must be [N, B, d] = {(N, B, d)}, got {tuple(dw.shape)}")
    kw = dict(dtype=x0.dtype, device=x0.device)
    x = torch.empty(N + 1, B, d, **kw)
    dt = torch.empty(B, N, **kw)
    coef = torch.empty(B, N, **kw)
    u = torch.empty(N, B, eqp.control_dim, **kw) if want_u else None
    y = disc = None
    if cost_order is not None:
        y = torch.empty(B, **kw)
        disc = torch.empty(B, **kw)
    saves = mask = None
    written = ctypes.c_int32(0)
    if save:
        saves = (torch.empty(N, B, sum(mlp.widths[1:]), **kw),
                 torch.empty(N, B, dtype=torch.int32, device=x0.device), torch.empty(N, B, **kw))
        if MASK_BPTT:  # only where the kernel will write one (16-row fast path)
            lib = _lib.load()
            nb = lib.dpac_rollout_nn_mask_bytes(ctypes.byref(mlp.struct), _dtype_id(x0), B, N)
            if nb < 0:
                raise _lib.DpacError("dpac_rollout_nn_mask_bytes", int(nb), lib.dpac_last_error().decode())
            if nb > 0:
                mb = lib.dpac_rollout_nn_mask_tile_bytes(ctypes.byref(mlp.struct))
                mask = torch.empty(N, (B + 15) // 16, mb, dtype=torch.uint8, device=x0.device)
    call("dpac_rollout_nn_fwd_masked", ctypes.byref(eqp), scheme, _dtype_id(x0), B, N, float(total_time),
         ctypes.byref(mlp.struct), _ptr(x0.contiguous()), _ptr(dw.contiguous()), _ptr(x), _ptr(dt),
         _ptr(coef), _ptr(u), _lib.COST_CRITIC if cost_order is None else cost_order, _ptr(y),
         _ptr(disc), _ptr(saves[0] if saves else None), _ptr(saves[1] if saves else None),
         _ptr(saves[2] if saves else None), _ptr(mask), ctypes.byref(written), _stream(x0))
    if saves is not None:
        saves = saves + (mask if written.value else None,)
    return x, dt, coef, u, y, disc, saves


class _ActorRolloutNN(torch.autograd.Function):
    """The actor's pathwise cost (solver.py:207-219) over a fused NN-control rollout,
    differentiable in the actor's parameters (BPTT, what GradientTape does for
    solver.py:92-97).

    forward: one dpac_rollout_nn_fwd launch with the backward saves.
    backward: a reverse time loop of dpac_step_bwd plus the MLP's input-gradient
    chain (per layer one scaled multiply and one [B x w] @ [w x w'] product),
    storing the gradient entering every BatchNorm output for all steps; the
    parameter gradients are then a few products/reductions over all N*B rows.
    Inputs: x0, dw, rs, then DeepNN.trainable_variables() (gamma[L+2], beta[L+2],
    W[L+1], b).  Outputs: y [B], disc_N [B], x_N [B, d]."""

    @staticmethod
    def forward(ctx, x0, dw, rs, eqp, scheme, T, N, ekn, *params):
        L = (len(params) - 1) // 3 - 1
        gam, bet, Ws, b = params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]
        view, _, _ = mlp_prepare(gam, bet, Ws, b, ekn, False)
        x, dt, coef, u, y, disc, (z, flag, disc_t, mask) = rollout_nn(
            eqp, scheme, x0, dw, T, N, view, cost_order=_lib.COST_ACTOR, save=True)
        ctx.save_for_backward(x, u, dw, z, flag, disc_t, rs, *params)
        ctx.mask = mask  # None where the forward kernel wrote no mask
        ctx.cfg = (eqp, scheme, T, N, ekn, L)
        return y, disc, x[N].clone()

    @staticmethod
    def backward(ctx, g_y, g_disc, g_xN):
        x, u, dw, z, flag, disc_t, rs, *params = ctx.saved_tensors
        eqp, scheme, T, N, ekn, L = ctx.cfg
        grads = actor_bptt_grads(eqp, scheme, T, N, ekn, rs, params, (x, u, dw, z, flag, disc_t, ctx.mask),
                                 g_y, g_disc, g_xN)
        return (None,) * 8 + tuple(grads)


def actor_rollout_saves(eqp, scheme: int, x0, dw, total_time: float, num_steps: int, net):
    """The actor's rollout with `net` as control and the backward saves, no autograd:
    (y [B], disc_N [B], x_N [B, d], saved) with saved = (x, u, dw, z, flag, disc_t, mask,
    prepared) as actor_bptt_grads takes it (the forward of _ActorRolloutNN).  prepared = the
    network's forward AND backward images from one dpac_mlp_prepare launch (round 5: the
    backward's images are formed here, beside the critic step, not in front of the BPTT —
    the actor's parameters do not change in between)."""
    prepared = net.mlp_prepared()
    x, dt, coef, u, y, disc, (z, flag, disc_t, mask) = rollout_nn(
        eqp, scheme, x0, dw, total_time, num_steps, prepared[0], cost_order=_lib.COST_ACTOR,
        save=True)
    return y, disc, x[num_steps], (x, u, dw.contiguous(), z, flag, disc_t, mask, prepared)


def actor_bptt_grads(eqp, scheme, T, N, ekn, rs, params, saved, g_y, g_disc, g_xN):
    """Gradients of DeepNN.trainable_variables() (params) of the actor from the saves of
    its fused rollout and the upstream gradients of (y, disc_N, x_N), each optional:
    the BPTT of solver.py:92-97 (dpac_rollout_nn_bwd, then dpac_mlp_param_grads)."""
    x, u, dw, z, flag, disc_t = saved[:6]
    mask = saved[6] if len(saved) > 6 else None
    prepared = saved[7] if len(saved) > 7 else None  # the forward's images of the same parameters
    L = (len(params) - 1) // 3 - 1
    gam, bet, Ws, b = params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]
    B, d = x.shape[1], x.shape[2]
    widths = [Ws[0].shape[0]] + [w.shape[1] for w in Ws]
    if prepared is not None and BPTT_MODE == "fused":
        view, wt, wt_km = prepared
    else:
        view, wt, wt_km = mlp_prepare(gam, bet, Ws, b, ekn, BPTT_MODE == "fused")
    s = view.scales
    zoff = np.cumsum([0] + widths[1:]).tolist()
    zl = [None] + [z[:, :, zoff[i - 1]:zoff[i]] for i in range(1, L + 2)]
    gx_in = None if g_xN is None else g_xN.contiguous()
    gd_in = None if g_disc is None else g_disc.contiguous()
    gy_in = None if g_y is None else g_y.contiguous()
    if BPTT_MODE == "fused":
        G = _bptt_fused(eqp, scheme, T, N, L, x, u, dw, z, flag, disc_t, view, wt, wt_km, widths,
                        gx_in, gd_in, gy_in, mask)
    else:
        G = _bptt_loop(eqp, scheme, T, N, ekn, L, x, u, dw, zl, flag, disc_t, s, bet, Ws, b,
                       widths, gx_in, gd_in, gy_in)
    if PARAM_GRADS == "kernel":
        return mlp_param_grads(view, x[:N].reshape(N * B, d),
                               z.reshape(N * B, -1), G_all(G).reshape(N * B, -1), params)
    # parameter gradients over all N*B rows (PyTorch reference path)
    rows = lambda tt: tt.reshape(N * B, -1)
    zin = [x[:N]] + [zl[i] for i in range(1, L + 1)] + [zl[L + 1] + b]
    dgam = [rs * torch.sum(rows(G[i] * zin[i]), 0) for i in range(L + 2)]
    dbet = [torch.sum(rows(G[i]), 0) for i in range(L + 2)]
    A = [torch.addcmul(bet[0], x[:N], s[0])]
    for i in range(1, L + 1):
        yl = torch.addcmul(bet[i], zl[i], s[i])
        A.append(yl + torch.relu(yl))
    # per-step partial products summed over N (split-K; one GEMM with an N*B-long
    # reduction runs far below the MFMA rate)
    dW = [torch.bmm(A[i].transpose(1, 2), G[i + 1] * s[i + 1]).sum(0) for i in range(L + 1)]
    db = torch.sum(rows(G[L + 1] * s[L + 1]), 0)
    return [*dgam, *dbet, *dW, db]


# The actor's forward records the hidden activations' sign bits and the BPTT reads them
# instead of z (dpac_rollout_nn_*_masked; bitwise the same G).  False: z everywhere.
MASK_BPTT = os.environ.get("DPAC_MASK_BPTT", "1") != "0"
# "fused": the reverse time loop as one dpac_rollout_nn_bwd launch; "loop": the
# reference implementation of the same loop, dpac_step_bwd + PyTorch per step.
BPTT_MODE = "fused"
# "kernel": parameter gradients from dpac_mlp_param_grads (one launch + reduce);
# "torch": the same sums as PyTorch products/reductions (test reference).
PARAM_GRADS = "kernel"


def G_all(G):
    """The [N, B, Σ widths] buffer behind the per-layer views of _bptt_fused / _bptt_loop."""
    base = G[0]._base if G[0]._base is not None else None
    if base is not None and all(g._base is base for g in G) and base.is_contiguous():
        return base
    return torch.cat(G, dim=-1).contiguous()


_WS_CACHE = {}


def _workspace(nbytes: int, device, tag: int = 0) -> torch.Tensor:
    """A reusable device scratch buffer, one per (device, size, tag) and never freed: a
    captured HIP graph keeps the address it saw, so a buffer must outlive every graph
    that used it.  Users of one tag run stream-ordered; work that runs beside them on
    another stream (the critic's G-network backward beside the actor's BPTT) takes
    its own tag."""
    key = (device.type, device.index, int(nbytes), int(tag))
    ws = _WS_CACHE.get(key)
    if ws is None:
        ws = _WS_CACHE[key] = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
    return ws


def bn_rs_host(dtype) -> float:
    """1/sqrt(1 + 1e-6) rounded as DeepNN.bn_rs is (solver.py BN_EPS), on the host: the
    device copy must not be read inside a captured graph."""
    return float(torch.rsqrt(torch.tensor(1.0 + 1e-6, dtype=dtype)))


def mlp_param_grads(view: "MlpView", x, z, G, like, ws_tag: int = 0):
    """Gradients of DeepNN's trainable variables (order of trainable_variables()) from
    the backward chain's G [R, Σ widths], the saved z [R, Σ widths[1:]] and the
    network input x [R, d]; one dpac_mlp_param_grads launch.  `like` gives the
    parameter shapes; ws_tag selects the scratch buffer (_workspace)."""
    _require_gpu(x, z, G)
    R = x.shape[0]
    dt = _dtype_id(x)
    nbytes = _lib.load().dpac_mlp_param_grads_workspace(dt, R, ctypes.byref(view.struct))
    if nbytes < 0:
        raise _lib.DpacError("dpac_mlp_param_grads_workspace", nbytes, _lib.load().dpac_last_error().decode())
    ws = _workspace(int(nbytes), x.device, ws_tag)
    total = sum(p.numel() for p in like)
    flat = torch.empty(total, dtype=x.dtype, device=x.device)
    if x.stride(1) != 1 or not z.is_contiguous() or not G.is_contiguous():
        raise ValueError("mlp_param_grads: x needs unit column stride, z and G contiguous")
    _guarded_call(view, "dpac_mlp_param_grads", lambda v: (
        dt, R, v, bn_rs_host(x.dtype), ctypes.c_void_p(x.data_ptr()), x.stride(0), _ptr(z), _ptr(G),
        _ptr(ws), ws.numel(), _ptr(flat), _stream(x)))
    out, o = [], 0
    for p in like:
        out.append(flat[o:o + p.numel()].view(p.shape))
        o += p.numel()
    return out


def _ptr_array(ts):
    """A C array of device pointers (NULL for a None list)."""
    if ts is None:
        return None
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def _bptt_fused(eqp, scheme, T, N, L, x, u, dw, z, flag, disc_t, view, wt, wt_km, widths,
                g_xN, g_disc, g_y, mask=None):
    """G[i] = dL/d(output of BN_i) for every step, [N, B, width[i]], from one launch
    (view, wt, wt_km from mlp_prepare; mask: the forward's sign bits, or None)."""
    B = x.shape[1]
    goff = np.cumsum([0] + widths).tolist()
    Gall = torch.empty(N, B, goff[-1], dtype=x.dtype, device=x.device)
    _guarded_call(view, "dpac_rollout_nn_bwd_masked", lambda v: (
        ctypes.byref(eqp), scheme, _dtype_id(x), B, N, float(T), v, _ptr_array(wt), _ptr_array(wt_km),
        _ptr(x), _ptr(u), _ptr(dw), _ptr(z), _ptr(flag), _ptr(disc_t), _ptr(mask), _ptr(g_xN),
        _ptr(g_disc), _ptr(g_y), _ptr(Gall), None, _stream(x)))
    return [Gall[:, :, goff[i]:goff[i + 1]] for i in range(L + 2)]


def _bptt_loop(eqp, scheme, T, N, ekn, L, x, u, dw, zl, flag, disc_t, s, bet, Ws, b, widths,
               g_xN, g_disc, g_y):
    """The same G as _bptt_fused, step by step: dpac_step_bwd + the MLP's input-gradient
    chain in PyTorch (per layer one scaled multiply and one [B x w] @ [w x w'] product)."""
    B, d = x.shape[1], x.shape[2]
    kw = dict(dtype=x.dtype, device=x.device)
    fac = [None] * (L + 1)
    for i in range(1, L + 1):
        yl = torch.addcmul(bet[i], zl[i], s[i])
        fac[i] = 1.0 + (yl > 0).to(yl.dtype)
    Wss = [(Ws[i] * s[i + 1]).t().contiguous() for i in range(L + 1)]  # (W diag(s))^T
    G = [torch.empty(N, B, w, **kw) for w in widths]
    gx = torch.zeros(B, d, **kw) if g_xN is None else g_xN
    gd = torch.zeros(B, **kw) if g_disc is None else g_disc.clone()  # ping-pong buffer below
    gy = torch.zeros(B, **kw) if g_y is None else g_y
    gx_dir, gu, gd_new = torch.empty_like(gx), torch.empty(B, u.shape[2], **kw), torch.empty_like(gd)
    if ekn:
        ob = torch.addcmul(bet[L + 1], zl[L + 1] + b, s[L + 1])  # BN_last output, all steps
        c = widths[L + 1] - 1
    for t in range(N - 1, -1, -1):
        call("dpac_step_bwd", ctypes.byref(eqp), scheme, _dtype_id(x), B, N, float(T),
             _ptr(x[t]), _ptr(u[t]), _ptr(dw[t]), _ptr(flag[t]), _ptr(disc_t[t]),
             _lib.COST_ACTOR, _ptr(gx), _ptr(gd), _ptr(gy), _ptr(gx_dir), _ptr(gu),
             _ptr(gd_new), _stream(x))
        if ekn:  # u = o[:c] / (1e-15 + relu(o_c) + |o[:c]|), solver.py:272-274
            o = ob[t]
            oc, oh = o[:, c], o[:, :c]
            nrm = torch.sqrt(torch.sum(oh * oh, 1))
            den = (1e-15 + torch.relu(oc)) + nrm
            k = torch.sum(gu * oh, 1) / (den * den)
            G[L + 1][t, :, :c] = gu / den[:, None] - (k / nrm)[:, None] * oh
            G[L + 1][t, :, c] = -k * (oc > 0).to(o.dtype)
        else:
            G[L + 1][t].copy_(gu)
        ga = G[L + 1][t] @ Wss[L]
        for i in range(L, 0, -1):
            torch.mul(ga, fac[i][t], out=G[i][t])
            ga = G[i][t] @ Wss[i - 1]
        G[0][t].copy_(ga)
        gx = torch.addcmul(gx_dir, ga, s[0])
        gd, gd_new = gd_new, gd
    return G


def actor_rollout_nn(eqp, scheme: int, x0, dw, total_time: float, num_steps: int, net):
    """(y [B], disc_N [B], x_N [B,d]) of the actor's rollout with `net` (a DeepNN) as
    control, differentiable in net's parameters through _ActorRolloutNN."""
    if not torch.is_grad_enabled():  # evaluation only: no backward saves
        x, _, _, _, y, disc, _ = rollout_nn(eqp, scheme, x0, dw, total_time, num_steps,
                                            net.mlp_view(), want_u=False, cost_order=_lib.COST_ACTOR)
        return y, disc, x[num_steps]
    return _ActorRolloutNN.apply(x0.contiguous(), dw.contiguous(), net.bn_rs, eqp, scheme,
                                 float(total_time), int(num_steps), bool(net.ekn_head),
                                 *net.trainable_variables())


# "kernel": DeepNN on independent rows runs dpac_mlp_rows_fwd/bwd + dpac_mlp_param_grads;
# "torch": PyTorch GEMMs and autograd (test reference).
ROW_MLP = "kernel"


def _split_params(params):
    L = (len(params) - 1) // 3 - 1
    return L, params[:L + 2], params[L + 2:2 * L + 4], params[2 * L + 4:3 * L + 5], params[-1]


# The row kernels' sign-bit mask (dpac.h dpac_mlp_rows_*_masked, round 5): the split-fp16
# forward records whether each hidden BN output is positive, and the backward chain reads
# those bits instead of z (bitwise the same G).  DPAC_ROW_MASK=0: z everywhere.
ROW_MASK = os.environ.get("DPAC_ROW_MASK", "1") != "0"


def _row_mask_buffer(view: MlpView, x: torch.Tensor):
    """The sign-bit mask buffer the masked row forward fills for x's rows, or None where no
    mask is written (float64, no split-fp16 images)."""
    nb = _lib.load().dpac_mlp_rows_mask_bytes(ctypes.byref(view.struct), _dtype_id(x), x.shape[0])
    if nb < 0:
        raise _lib.DpacError("dpac_mlp_rows_mask_bytes", int(nb), _lib.load().dpac_last_error().decode())
    return torch.empty(int(nb), dtype=torch.uint8, device=x.device) if nb > 0 else None


def mlp_rows(view: MlpView, x: torch.Tensor, save: bool = False, mask: bool = False):
    """out [R, w_out] (the network before any Eikonal head) for every row of x [R, d],
    one dpac_mlp_rows_fwd launch; with save=True also z [R, Σ widths[1:]].  With mask=True
    (and save) returns (out, z, sign-bit mask or None where the kernel wrote none)."""
    _require_gpu(x, *view.tensors)
    _check_same(x, *view.tensors)
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("mlp_rows: x must be [rows, d] with unit column stride")
    R = x.shape[0]
    out = torch.empty(R, view.widths[-1], dtype=x.dtype, device=x.device)
    z = torch.empty(R, sum(view.widths[1:]), dtype=x.dtype, device=x.device) if save else None
    m = _row_mask_buffer(view, x) if (save and mask) else None
    written = ctypes.c_int32(0)
    call("dpac_mlp_rows_fwd_masked", _dtype_id(x), R, ctypes.byref(view.struct),
         ctypes.c_void_p(x.data_ptr()), x.stride(0), _ptr(out), _ptr(z), _ptr(m), ctypes.byref(written),
         _stream(x))
    if mask:
        return out, z, (m if written.value else None)
    return out, z


class _RowMLP(torch.autograd.Function):
    """DeepNN (solver.py:260-271, before the Eikonal head) over independent rows with
    the hand-written kernels: forward = dpac_mlp_rows_fwd with saves; backward =
    dpac_mlp_rows_bwd (input-gradient chain, G of every BN output, dL/dx) +
    dpac_mlp_param_grads.  Inputs: x [R, d], rs, DeepNN.trainable_variables()."""

    @staticmethod
    def forward(ctx, x, rs, *params):
        L, gam, bet, Ws, b = _split_params(params)
        view, _, _ = mlp_prepare(gam, bet, Ws, b, False, False)
        need = any(ctx.needs_input_grad)
        out, z = mlp_rows(view, x, save=need)
        if need:
            ctx.save_for_backward(x, z, rs, *params)
        return out

    @staticmethod
    def backward(ctx, g_out):
        x, z, rs, *params = ctx.saved_tensors
        g_x, grads = row_mlp_backward(rs, params, x, z, g_out, ctx.needs_input_grad[0],
                                      any(ctx.needs_input_grad[2:]))
        return (g_x, None, *(grads if grads is not None else [None] * len(params)))


def row_mlp_backward(rs, params, x, z, g_out, want_x: bool, want_params: bool, ws_tag: int = 0,
                     prepared=None, mask=None):
    """The backward of mlp_rows(save=True) given dL/d(output) g_out [R, w_out]:
    dpac_mlp_rows_bwd (the input-gradient chain: G of every BN output, and dL/dx if
    want_x) then dpac_mlp_param_grads (if want_params).  params =
    DeepNN.trainable_variables(); prepared = mlp_prepare(..., want_wt=True) of the same
    parameters if the caller already has it (one launch fewer); mask = the forward's sign
    bits (mlp_rows(mask=True)) or None (z is read); returns (g_x or None, parameter
    gradients or None)."""
    if prepared is None:
        L, gam, bet, Ws, b = _split_params(params)
        prepared = mlp_prepare(gam, bet, Ws, b, False, True)
    view, wt, wt_km = prepared
    R = x.shape[0]
    G = torch.empty(R, sum(view.widths), dtype=x.dtype, device=x.device)
    g_x = torch.empty(R, view.widths[0], dtype=x.dtype, device=x.device) if want_x else None
    g_out = g_out.contiguous()
    _guarded_call(view, "dpac_mlp_rows_bwd_masked", lambda v: (
        _dtype_id(x), R, v, _ptr_array(wt), _ptr_array(wt_km), _ptr(z), _ptr(mask), _ptr(g_out), _ptr(G),
        _ptr(g_x), _stream(x)))
    grads = mlp_param_grads(view, x, z, G, params, ws_tag) if want_params else None
    return g_x, grads


# ---- the critic's G network with the TD1 dot fused ----
# "fused": critic_front runs dpac_mlp_rows_fwd_td1 (G never reaches HBM, only the
# per-step dots), the TD assembly reads those dots (DPAC_TD1_GDOT), and the G
# backward forms dL/dG in its prologue (dpac_mlp_rows_bwd_td1); "split": G [N*B, d]
# and dL/dG are written and read (dpac_mlp_rows_fwd + dpac_td_assemble_fwd/_bwd).
# Both give bitwise the same y, disc and gradients (tests/test_gpu_td_fused.py).
CRITIC_TD1 = os.environ.get("DPAC_CRITIC_TD1", "fused")
if CRITIC_TD1 not in ("fused", "split"):
    raise ValueError(f"DPAC_CRITIC_TD1 must be 'fused' or 'split', got {CRITIC_TD1!r}")


def mlp_rows_td1(eqp, view: MlpView, x: torch.Tensor, u: torch.Tensor, dw: torch.Tensor,
                 save: bool = False, mask: bool = False):
    """gdot [R] = Σ_j (σ(x,u)·dw)_j · G_j(x) for G = the network (width d in and out)
    over the rows x [R, d] (solver.py:179-184 without G ever written), one
    dpac_mlp_rows_fwd_td1 launch; u [R, c] and dw [R, d] row-aligned with x.  With
    save=True also the backward saves z [R, Σ widths[1:]]; with mask=True (and save)
    returns (gdot, z, sign-bit mask or None) as mlp_rows does."""
    _require_gpu(x, u, dw, *view.tensors)
    _check_same(x, u, dw, *view.tensors)
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("mlp_rows_td1: x must be [rows, d] with unit column stride")
    R = x.shape[0]
    if u.shape[0] != R or dw.shape != (R, eqp.dim):
        raise ValueError("mlp_rows_td1: u [R, c] and dw [R, d] must be row-aligned with x")
    gdot = torch.empty(R, dtype=x.dtype, device=x.device)
    z = torch.empty(R, sum(view.widths[1:]), dtype=x.dtype, device=x.device) if save else None
    m = _row_mask_buffer(view, x) if (save and mask) else None
    written = ctypes.c_int32(0)
    call("dpac_mlp_rows_fwd_td1_masked", ctypes.byref(eqp), _dtype_id(x), R, ctypes.byref(view.struct),
         ctypes.c_void_p(x.data_ptr()), x.stride(0), _ptr(u.contiguous()), _ptr(dw.contiguous()),
         _ptr(gdot), _ptr(z), _ptr(m), ctypes.byref(written), _stream(x))
    if mask:
        return gdot, z, (m if written.value else None)
    return gdot, z


def td_assemble_gdot(eqp, x, u, dt, coef, gdot, *, cost_order: int = _lib.COST_CRITIC):
    """(y [B], disc_N [B]) of TD1 from the fused dots gdot [N, B] (DPAC_TD1_GDOT; no
    autograd: the critic's split step differentiates by hand)."""
    _require_gpu(x, u, dt, coef, gdot)
    B, N = dt.shape
    y = torch.empty(B, dtype=x.dtype, device=x.device)
    disc = torch.empty_like(y)
    call("dpac_td_assemble_fwd", ctypes.byref(eqp), _lib.TD1_GDOT, cost_order, _dtype_id(x), B, N,
         _ptr(x.contiguous()), _ptr(u.contiguous()), None, 0, 0, _lib.SAMPLE_NORMAL,
         _ptr(dt.contiguous()), _ptr(coef.contiguous()), _ptr(gdot.contiguous()), _ptr(y),
         _ptr(disc), _stream(x))
    return y, disc


def critic_loss_grad(V, y, disc, z_bdry, scale: float, delta_clip: float):
    """dpac_critic_loss_grad: (g_out [3B, 1], -g [B]) — loss_critic's gradient at
    V = NN_value([x_0; x_N; x_bdry]) (solver.py:73-78, 189-190), one launch."""
    _require_gpu(V, y, disc, z_bdry)
    B = y.shape[0]
    V, y, disc, z_bdry = V.contiguous(), y.contiguous(), disc.contiguous(), z_bdry.contiguous()
    if V.numel() != 3 * B or disc.numel() != B or z_bdry.numel() != B:
        raise ValueError("critic_loss_grad: V needs 3B entries, disc and z_bdry B")
    g_out = torch.empty(3 * B, 1, dtype=y.dtype, device=y.device)
    neg_g = torch.empty(B, dtype=y.dtype, device=y.device)
    call("dpac_critic_loss_grad", _dtype_id(y), B, _ptr(V), _ptr(y), _ptr(disc), _ptr(z_bdry),
         float(scale), float(delta_clip), _ptr(g_out), _ptr(neg_g), _stream(y))
    return g_out, neg_g


def td_assemble_bwd_gdot(eqp, dt, coef, g_y):
    """d L / d gdot [N, B] = −g_y·disc_t·coef_t·√dt_t given dL/dy [B]."""
    _require_gpu(dt, coef, g_y)
    B, N = dt.shape
    g_gdot = torch.empty(N, B, dtype=dt.dtype, device=dt.device)
    call("dpac_td_assemble_bwd_gdot", ctypes.byref(eqp), _dtype_id(dt), B, N,
         _ptr(dt.contiguous()), _ptr(coef.contiguous()), _ptr(g_y.contiguous()), _ptr(g_gdot),
         _stream(dt))
    return g_gdot


def row_mlp_backward_td1(eqp, rs, params, x, z, u, dw, g_gdot, want_params: bool = True,
                         ws_tag: int = 0, mask=None):
    """row_mlp_backward for mlp_rows_td1: dpac_mlp_rows_bwd_td1 (dL/dG = g_gdot·σ dw in
    its prologue; mask: the forward's sign bits or None) then dpac_mlp_param_grads; returns
    the parameter gradients."""
    L, gam, bet, Ws, b = _split_params(params)
    view, wt, wt_km = mlp_prepare(gam, bet, Ws, b, False, True)
    R = x.shape[0]
    G = torch.empty(R, sum(view.widths), dtype=x.dtype, device=x.device)
    u, dw, g_gdot = u.contiguous(), dw.contiguous(), g_gdot.contiguous()
    _guarded_call(view, "dpac_mlp_rows_bwd_td1_masked", lambda v: (
        ctypes.byref(eqp), _dtype_id(x), R, v, _ptr_array(wt), _ptr_array(wt_km), _ptr(z), _ptr(mask),
        ctypes.c_void_p(x.data_ptr()), x.stride(0), _ptr(u), _ptr(dw), _ptr(g_gdot), _ptr(G), None,
        _stream(x)))
    return mlp_param_grads(view, x, z, G, params, ws_tag) if want_params else None


def row_mlp(net, x: torch.Tensor, const_params: bool = False) -> torch.Tensor:
    """net(x) before the Eikonal head, x [..., d] -> [..., w_out], through the kernels.
    const_params: the parameters are constants for autograd (only dL/dx is formed),
    as for the critic's V inside the actor's tape (solver.py:95 watches the actor)."""
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(1) != 1:
        x2 = x2.contiguous()
    params = net.trainable_variables()
    if const_params:
        params = [p.detach() for p in params]
    if torch.is_grad_enabled() and (x2.requires_grad or any(p.requires_grad for p in params)):
        out = _RowMLP.apply(x2, net.bn_rs, *params)
    else:
        out, _ = mlp_rows(net.mlp_view(), x2)
    return out.reshape(*lead, out.shape[-1])


def flag_init(eqp, scheme: int, x0: torch.Tensor, total_time: float, num_steps: int):
    _require_gpu(x0)
    flag = torch.empty(x0.shape[0], dtype=torch.int32, device=x0.device)
    call("dpac_flag_init", ctypes.byref(eqp), scheme, _dtype_id(x0), x0.shape[0], num_steps,
         float(total_time), _ptr(x0.contiguous()), _ptr(flag), _stream(x0))
    return flag


class _SdeStep(torch.autograd.Function):
    """One propagate-loop transition with an external control, fused with the
    running cost/discount update; backward = dpac_step_bwd."""

    @staticmethod
    def forward(ctx, x, u, disc, y, dw_t, flag, eqp, scheme, T, N, cost_order):
        B, d = x.shape
        x_out = torch.empty_like(x)
        disc_out = torch.empty_like(disc)
        y_out = torch.empty_like(y)
        dt = torch.empty_like(disc)
        coef = torch.empty_like(disc)
        flag_out = torch.empty_like(flag)
        call("dpac_step_fwd", ctypes.byref(eqp), scheme, _dtype_id(x), B, N, float(T),
             _ptr(x), _ptr(u), _ptr(dw_t), _ptr(flag), _ptr(disc), _ptr(y), cost_order,
             _ptr(x_out), _ptr(flag_out), _ptr(disc_out), _ptr(y_out), _ptr(dt), _ptr(coef),
             _stream(x))
        ctx.save_for_backward(x, u, disc, dw_t, flag)
        ctx.cfg = (eqp, scheme, T, N, cost_order)
        ctx.mark_non_differentiable(dt, coef, flag_out)
        return x_out, disc_out, y_out, dt, coef, flag_out

    @staticmethod
    def backward(ctx, g_x, g_disc, g_y, _gdt, _gcoef, _gflag):
        x, u, disc, dw_t, flag = ctx.saved_tensors
        eqp, scheme, T, N, cost_order = ctx.cfg
        B = x.shape[0]
        g_x = torch.zeros_like(x) if g_x is None else g_x.contiguous()
        g_disc_c = None if g_disc is None else g_disc.contiguous()
        g_y_c = None if g_y is None else g_y.contiguous()
        gx = torch.empty_like(x)
        gu = torch.empty_like(u)
        gd = torch.empty_like(disc)
        call("dpac_step_bwd", ctypes.byref(eqp), scheme, _dtype_id(x), B, N, float(T), _ptr(x),
             _ptr(u), _ptr(dw_t), _ptr(flag), _ptr(disc), cost_order, _ptr(g_x), _ptr(g_disc_c),
             _ptr(g_y_c), _ptr(gx), _ptr(gu), _ptr(gd), _stream(x))
        if g_disc is None and g_y is None:
            gd.zero_()
        gy_in = g_y if g_y is not None else None
        return gx, gu, gd, gy_in, None, None, None, None, None, None, None


def sde_step(eqp, scheme: int, total_time: float, num_steps: int, x, u, dw_t, flag, disc, y,
             cost_order: int = _lib.COST_ACTOR):
    """x_{t+1}, disc_{t+1}, y_{t+1}, dt_t, coef_t, flag_{t+1} = step(x_t, u_t, ...)."""
    _require_gpu(x, u, dw_t, disc, y)
    _check_same(x, u, dw_t, disc, y)
    return _SdeStep.apply(x.contiguous(), u.contiguous(), disc.contiguous(), y.contiguous(),
                          dw_t.contiguous(), flag.contiguous(), eqp, scheme, total_time,
                          num_steps, cost_order)


class _TdAssemble(torch.autograd.Function):
    """y, disc_N = TD target assembly (solver.py:166-187); grad flows to G only."""

    @staticmethod
    def forward(ctx, G, x, u, dw, dt, coef, eqp, td_type, cost_order, seed, traj_offset,
                sample_type):
        B, N = dt.shape
        y = torch.empty(B, dtype=x.dtype, device=x.device)
        disc = torch.empty_like(y)
        call("dpac_td_assemble_fwd", ctypes.byref(eqp), td_type, cost_order, _dtype_id(x), B, N,
             _ptr(x), _ptr(u), _ptr(dw), seed & 0xFFFFFFFFFFFFFFFF, traj_offset, sample_type,
             _ptr(dt), _ptr(coef), _ptr(G), _ptr(y), _ptr(disc), _stream(x))
        ctx.save_for_backward(x, u, dw, dt, coef)
        ctx.cfg = (eqp, td_type, seed, traj_offset, sample_type, G is not None)
        ctx.mark_non_differentiable(disc)
        return y, disc

    @staticmethod
    def backward(ctx, g_y, _g_disc):
        x, u, dw, dt, coef = ctx.saved_tensors
        eqp, td_type, seed, traj_offset, sample_type, has_g = ctx.cfg
        gG = None
        if has_g and td_type == _lib.TD1 and g_y is not None and ctx.needs_input_grad[0]:
            B, N = dt.shape
            gG = torch.empty(N, B, eqp.dim, dtype=x.dtype, device=x.device)
            call("dpac_td_assemble_bwd", ctypes.byref(eqp), _dtype_id(x), B, N, _ptr(x),
                 _ptr(u), _ptr(dw), seed & 0xFFFFFFFFFFFFFFFF, traj_offset, sample_type,
                 _ptr(dt), _ptr(coef), _ptr(g_y.contiguous()), _ptr(gG), _stream(x))
        return gG, None, None, None, None, None, None, None, None, None, None, None


def td_assemble(eqp, td_type: int, x, u, dw, dt, coef, G=None, *,
                cost_order: int = _lib.COST_CRITIC, seed: int = 0, traj_offset: int = 0,
                sample_type: int = _lib.SAMPLE_NORMAL):
    """(y [B], disc_N [B]) over a finished trajectory; TD1 needs G [N,B,d]."""
    _require_gpu(x, u, dw, dt, coef, G)
    _check_same(x, u, dw, dt, coef, G)
    if td_type == _lib.TD1 and G is None:
        raise ValueError("TD1 needs G = NN_value_grad(x_t)")
    G = None if (G is None or td_type != _lib.TD1) else G.contiguous()
    return _TdAssemble.apply(G, x.contiguous(), u.contiguous(),
                             None if dw is None else dw.contiguous(), dt.contiguous(),
                             coef.contiguous(), eqp, td_type, cost_order, seed, traj_offset,
                             sample_type)


def td_assemble_bwd(eqp, x, u, dw, dt, coef, g_y, *, seed: int = 0, traj_offset: int = 0,
                    sample_type: int = _lib.SAMPLE_NORMAL):
    """dL/dG [N, B, d] of the TD1 target y (solver.py:177-184) given dL/dy [B] (the
    backward of td_assemble without autograd)."""
    _require_gpu(x, u, dw, dt, coef, g_y)
    B, N = dt.shape
    gG = torch.empty(N, B, eqp.dim, dtype=x.dtype, device=x.device)
    call("dpac_td_assemble_bwd", ctypes.byref(eqp), _dtype_id(x), B, N, _ptr(x.contiguous()),
         _ptr(u.contiguous()), _ptr(None if dw is None else dw.contiguous()),
         seed & 0xFFFFFFFFFFFFFFFF, traj_offset, sample_type, _ptr(dt.contiguous()),
         _ptr(coef.contiguous()), _ptr(g_y.contiguous()), _ptr(gG), _stream(x))
    return gG


def actor_cost(eqp, x, u, dt, coef):
    """Σ_t coef·w·dt·disc and disc_N over a finished trajectory (solver.py:213-219)."""
    _require_gpu(x, u, dt, coef)
    B, N = dt.shape
    y = torch.empty(B, dtype=x.dtype, device=x.device)
    disc = torch.empty_like(y)
    call("dpac_actor_cost_fwd", ctypes.byref(eqp), _dtype_id(x), B, N, _ptr(x.contiguous()),
         _ptr(u.contiguous()), _ptr(dt.contiguous()), _ptr(coef.contiguous()), _ptr(y),
         _ptr(disc), _stream(x))
    return y, disc


def equation_eval(eqp, what: int, x: torch.Tensor, u: torch.Tensor | None = None):
    """Row-wise Equation method on the device (equation.py:108-311)."""
    _require_gpu(x, u)
    _check_same(x, u)
    x = x.contiguous()
    B = x.shape[0]
    if what in (_lib.EVAL_DRIFT, _lib.EVAL_SIGMA, _lib.EVAL_V_GRAD):
        out = torch.empty(B, eqp.dim, dtype=x.dtype, device=x.device)
    elif what == _lib.EVAL_U_TRUE:
        out = torch.empty(B, eqp.control_dim, dtype=x.dtype, device=x.device)
    else:
        out = torch.empty(B, dtype=x.dtype, device=x.device)
    call("dpac_equation_eval", ctypes.byref(eqp), what, _dtype_id(x), B, _ptr(x),
         _ptr(None if u is None else u.contiguous()), _ptr(out), _stream(x))
    return out


class _VTrue(torch.autograd.Function):
    """V_true(x) with gradient V_grad_true(x) (cheat_value path, solver.py:223)."""

    @staticmethod
    def forward(ctx, x, eqp):
        ctx.save_for_backward(x)
        ctx.eqp = eqp
        return equation_eval(eqp, _lib.EVAL_V_TRUE, x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g.unsqueeze(1) * equation_eval(ctx.eqp, _lib.EVAL_V_GRAD, x), None


def v_true(eqp, x):
    return _VTrue.apply(x, eqp)


_ADAM_ARGS = {}


def adam_apply(vs, gs, ms, ss, alpha: float, beta_1: float, beta_2: float, eps: float):
    """One TF-form Adam step over parameter tensors vs with gradients gs and moments
    ms, ss (all on the GPU, one dtype): one dpac_adam_apply launch on the current
    stream.  The pointer arrays are cached per set of addresses (a replayed graph
    hands back the same gradient buffers every step)."""
    _require_gpu(*vs, *gs, *ms, *ss)
    _check_same(vs[0], *vs, *gs, *ms, *ss)
    key = tuple(t.data_ptr() for t in (*vs, *gs, *ms, *ss))
    args = _ADAM_ARGS.get(key)
    if args is None:
        for group in (gs, ms, ss):
            for v, t in zip(vs, group):
                if t.shape != v.shape or not t.is_contiguous():
                    raise ValueError("adam_apply: gradients and moments must match the "
                                     "parameters' shapes and be contiguous")
        if not all(v.is_contiguous() for v in vs):
            raise ValueError("adam_apply: parameters must be contiguous")
        n = len(vs)
        arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
        args = (n, (ctypes.c_int64 * n)(*[v.numel() for v in vs]), arr(vs), arr(gs), arr(ms), arr(ss))
        if len(_ADAM_ARGS) > 64:
            _ADAM_ARGS.clear()
        _ADAM_ARGS[key] = args
    n, numel, pv, pg, pm, ps = args
    call("dpac_adam_apply", _dtype_id(vs[0]), n, numel, pv, pg, pm, ps, float(alpha),
         float(beta_1), float(beta_2), float(eps), _stream(vs[0]))
