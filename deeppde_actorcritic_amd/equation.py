"""Equation classes with the reference's surface (equation.py:5-311), backed by libdpac.

Class names, constructor (`eqn_config`), attribute names and method signatures
follow the reference so `getattr(equation, eqn_name)(eqn_config)` (main.py:34)
keeps working; "EKN" (the name the shipped configs use) is an alias of `ekn`.

Two families of methods:
  * reference-layout methods (sample_*, propagate_*, w_tf, ...), accepting numpy
    arrays or tensors in the reference's layouts ([B,d], dw [B,d,N],
    x_smp [B,d,N+1]) — the drop-in surface; layout translation happens here;
  * device-native methods used by the solver (`sample_device`, `rollout`,
    `params`), in the step-major layouts of include/dpac.h.
All arithmetic on the device goes through libdpac; nothing here computes the
hot path in PyTorch.
"""
from __future__ import annotations

from typing import NamedTuple

import numpy as np
import torch
from scipy.stats import multivariate_normal as normal

from . import _lib, ops
from .config import torch_dtype

SCHEMES = {"naive": _lib.SCHEME_NAIVE, "adaptive": _lib.SCHEME_ADAPTIVE}
SAMPLE_TYPES = {"normal": _lib.SAMPLE_NORMAL, "bounded": _lib.SAMPLE_BOUNDED,
                "zero": _lib.SAMPLE_ZERO_X0}


class TrajectoryBatch(NamedTuple):
    """Device-native batch: x0 [B,d], dw [N,B,d], x_bdry [B,d]."""
    x0: torch.Tensor
    dw: torch.Tensor
    x_bdry: torch.Tensor


def _device():
    if not torch.cuda.is_available():
        raise _lib.DpacUnavailable("no ROCm GPU visible: the libdpac hot path has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def _as_dev(a, dtype=None):
    dtype = dtype or torch_dtype()
    if isinstance(a, torch.Tensor):
        return a.to(device=_device(), dtype=dtype)
    return torch.as_tensor(np.asarray(a), dtype=dtype, device=_device())


class Equation(object):
    """Base class for defining PDE related function (equation.py:5-142)."""

    eqn_id = None

    def __init__(self, eqn_config):
        self.dim = eqn_config.dim
        self.gamma = eqn_config.discount
        self.R = eqn_config.R
        self.control_dim = eqn_config.control_dim
        self.sigma_Up = np.sqrt(2.0)

    # ---- C-ABI parameter block ------------------------------------------------
    def params(self) -> _lib.EqnParams:
        cached = self.__dict__.get("_params_cache")
        if cached is not None:
            return cached
        p = _lib.EqnParams()
        p.eqn, p.dim, p.control_dim, p.reserved = self.eqn_id, self.dim, self.control_dim, 0
        p.gamma, p.R, p.sigma_up = float(self.gamma), float(self.R), float(self.sigma_Up)
        self._fill(p)
        self._params_cache = p
        return p

    def _fill(self, p):  # per-equation coefficients
        raise NotImplementedError

    # ---- host samplers, bit-identical to the reference (equation.py:13-44) ------
    def sample_normal(self, num_sample, N):
        r_Sample = np.random.uniform(low=0, high=self.R, size=[num_sample, 1])
        r = r_Sample ** (1 / self.dim) * (self.R ** ((self.dim - 1) / self.dim))
        angle = normal.rvs(size=[num_sample, self.dim])
        x0 = r * angle / np.sqrt(np.sum(angle ** 2, 1, keepdims=True))
        dw_sample = normal.rvs(size=[num_sample, self.dim, N])
        x_bdry = normal.rvs(size=[num_sample, self.dim])
        x_bdry = self.R * x_bdry / np.sqrt(np.sum(np.square(x_bdry), 1, keepdims=True))
        return x0, dw_sample, x_bdry

    def sample_bounded(self, num_sample, N):
        r_Sample = np.random.uniform(low=0, high=self.R, size=[num_sample, 1])
        r = r_Sample ** (1 / self.dim) * (self.R ** ((self.dim - 1) / self.dim))
        angle = normal.rvs(size=[num_sample, self.dim])
        x0 = r * angle / np.sqrt(np.sum(angle ** 2, 1, keepdims=True))
        k = np.random.randint(6, size=[num_sample, self.dim, N])
        dw_sample = np.floor((k - 1) / 4) * np.sqrt(3.0)
        x_bdry = normal.rvs(size=[num_sample, self.dim])
        x_bdry = self.R * x_bdry / np.sqrt(np.sum(np.square(x_bdry), 1, keepdims=True))
        return x0, dw_sample, x_bdry

    def sample0(self, num_sample, N):
        x0 = np.zeros(shape=[num_sample, self.dim]) + 0.01
        dw_sample = normal.rvs(size=[num_sample, self.dim, N])
        x_bdry = normal.rvs(size=[num_sample, self.dim])
        x_bdry = self.R * x_bdry / np.sqrt(np.sum(np.square(x_bdry), 1, keepdims=True))
        return x0, dw_sample, x_bdry

    # ---- device sampler (rocRAND Philox, keyed by global trajectory index) -----
    def sample_device(self, kind: str, num_sample: int, N: int, seed: int, traj_offset: int = 0,
                      dtype=None, out=None) -> TrajectoryBatch:
        x0, dw, xb = ops.sample(self.params(), SAMPLE_TYPES[kind], num_sample, N, seed,
                                traj_offset, dtype or torch_dtype(), _device(), out=out)
        return TrajectoryBatch(x0, dw, xb)

    @staticmethod
    def to_native(data, dtype=None) -> TrajectoryBatch:
        """Reference-layout (x0 [B,d], dw [B,d,N], x_bdry [B,d]) -> device-native batch."""
        if isinstance(data, TrajectoryBatch):
            return data
        x0, dw, xb = data
        dw = _as_dev(dw, dtype).permute(2, 0, 1).contiguous()
        return TrajectoryBatch(_as_dev(x0, dtype).contiguous(), dw, _as_dev(xb, dtype).contiguous())

    # ---- rollouts ---------------------------------------------------------------
    def rollout(self, scheme: str, x0, dw, T: float, N: int, NN_control=None, cheat=False,
                requires_grad=False):
        """Device-native rollout: returns x [N+1,B,d], dt [B,N], coef [B,N], u [N,B,c].

        cheat=True: one fused kernel with u = u_true (equation.py:54-55/87-88).
        NN control without gradients: one fused kernel evaluating the actor MLP on
        MFMA tiles inside the time loop (dpac_rollout_nn_fwd).  With gradients
        (the actor's BPTT): u_t = NN_control(x_t) between dpac_step_fwd launches.
        """
        sch = SCHEMES[scheme]
        eqp = self.params()
        if cheat:
            x, dt, coef, u, _, _ = ops.rollout_analytic(eqp, sch, x0, dw, T, N, want_u=True)
            return x, dt, coef, u
        B = x0.shape[0]
        if requires_grad:
            flag = ops.flag_init(eqp, sch, x0, T, N)
            xs, us, dts, coefs = [x0], [], [], []
            disc = torch.ones(B, dtype=x0.dtype, device=x0.device)
            y = torch.zeros_like(disc)
            x = x0
            for t in range(N):
                u = NN_control(x, False, need_grad=False)
                x, disc, y, dt, coef, flag = ops.sde_step(eqp, sch, T, N, x, u, dw[t], flag, disc, y)
                xs.append(x); us.append(u); dts.append(dt); coefs.append(coef)
            return torch.stack(xs), torch.stack(dts, 1), torch.stack(coefs, 1), torch.stack(us)
        if hasattr(NN_control, "fused_ok") and NN_control.fused_ok():  # one launch, MLP on MFMA
            x, dt, coef, u, _, _, _ = ops.rollout_nn(eqp, sch, x0, dw, T, N, NN_control.mlp_view())
            return x, dt, coef, u
        return rollout_nn_nograd(eqp, sch, x0, dw, T, N, NN_control)

    def _propagate(self, scheme, num_sample, x0, dw_sample, NN_control, training, T, N, cheat):
        x0 = _as_dev(x0).contiguous()
        dw = _as_dev(dw_sample).permute(2, 0, 1).contiguous()
        grad = (not cheat) and torch.is_grad_enabled()
        x, dt, coef, _ = self.rollout(scheme, x0, dw, T, N, NN_control, cheat, requires_grad=grad)
        # back to the reference layouts: x_smp [B,d,N+1], dt/coef [B,N]
        return x.permute(1, 2, 0), dt, coef

    def propagate_naive(self, num_sample, x0, dw_sample, NN_control, training, T, N, cheat):
        """equation.py:46-71 (same signature and return layouts)."""
        return self._propagate("naive", num_sample, x0, dw_sample, NN_control, training, T, N, cheat)

    def propagate_adaptive(self, num_sample, x0, dw_sample, NN_control, training, T, N, cheat):
        """equation.py:73-106 (same signature and return layouts)."""
        return self._propagate("adaptive", num_sample, x0, dw_sample, NN_control, training, T, N,
                               cheat)

    # ---- coefficients (device kernels; rows = samples) -------------------------
    def _eval(self, what, x, u=None):
        x = _as_dev(x)
        return ops.equation_eval(self.params(), what, x, None if u is None else _as_dev(u, x.dtype))

    def w_tf(self, x, u):
        """Running cost in control problems ([B,1])."""
        return self._eval(_lib.EVAL_W, x, u).unsqueeze(1)

    def Z_tf(self, x):
        """Terminal cost in control problems ([B,1])."""
        return self._eval(_lib.EVAL_Z, x).unsqueeze(1)

    def b_np(self, x):
        return np.sum(x ** 2, 1, keepdims=True) - (self.R ** 2)

    def b_tf(self, x):
        return self._eval(_lib.EVAL_B, x).unsqueeze(1)

    def V_true(self, x):
        """True value function ([B,1]); differentiable (gradient V_grad_true)."""
        return ops.v_true(self.params(), _as_dev(x)).unsqueeze(1)

    def u_true(self, x):
        return self._eval(_lib.EVAL_U_TRUE, x)

    def V_grad_true(self, x):
        return self._eval(_lib.EVAL_V_GRAD, x)

    def sigma(self, x, u, num_sample):
        """Dense [B,d,d] diffusion matrix, as the reference returns it."""
        return torch.diag_embed(self._eval(_lib.EVAL_SIGMA, x, u))

    def sigma_diag(self, x, u):
        return self._eval(_lib.EVAL_SIGMA, x, u)

    def drift(self, x, u):
        return self._eval(_lib.EVAL_DRIFT, x, u)

    def diffusion(self, x, u, dw, num_sample):
        return self.sigma_diag(x, u) * _as_dev(dw)


def rollout_nn_nograd(eqp, sch, x0, dw, T, N, NN_control, flag=None):
    """Critic-side rollout with the actor MLP as control and no graph: the step
    kernel writes x_{t+1}, dt_t, coef_t straight into the [N+1]/[N] buffers."""
    import ctypes
    B, d = x0.shape
    kw = dict(dtype=x0.dtype, device=x0.device)
    x = torch.empty(N + 1, B, d, **kw)
    u_all = torch.empty(N, B, eqp.control_dim, **kw)
    dt = torch.empty(N, B, **kw)
    coef = torch.empty(N, B, **kw)
    x[0].copy_(x0)
    if flag is None:
        flag = ops.flag_init(eqp, sch, x0, T, N)
    flag2 = torch.empty_like(flag)
    stream = ops._stream(x0)
    dtid = ops._dtype_id(x0)
    with torch.no_grad():
        for t in range(N):
            u_all[t].copy_(NN_control(x[t], False, need_grad=False))
            _lib.call("dpac_step_fwd", ctypes.byref(eqp), sch, dtid, B, N, float(T),
                      ops._ptr(x[t]), ops._ptr(u_all[t]), ops._ptr(dw[t]), ops._ptr(flag), None,
                      None, _lib.COST_CRITIC, ops._ptr(x[t + 1]), ops._ptr(flag2), None, None,
                      ops._ptr(dt[t]), ops._ptr(coef[t]), stream)
            flag, flag2 = flag2, flag
    # the step kernel emits per-step [B] vectors; present the [B, N] layout
    return x, dt.t().contiguous(), coef.t().contiguous(), u_all


class LQR(Equation):
    """linear quadratic regulator (equation.py:144-176)"""

    eqn_id = _lib.EQN_LQR

    def __init__(self, eqn_config):
        super(LQR, self).__init__(eqn_config)
        self.p = eqn_config.p
        self.q = eqn_config.q
        self.beta = eqn_config.beta
        self.k = (((self.gamma ** 2) * (self.q ** 2) + 4 * self.p * self.q * (self.beta ** 2)) ** 0.5
                  - self.q * self.gamma) / (self.beta ** 2) / 2

    def _fill(self, p):
        p.p, p.q, p.beta, p.k = float(self.p), float(self.q), float(self.beta), float(self.k)


class VDP(Equation):
    """Van Der Pol oscillator (equation.py:179-238)"""

    eqn_id = _lib.EQN_VDP

    def __init__(self, eqn_config):
        super(VDP, self).__init__(eqn_config)
        self.a = eqn_config.a
        self.epsl = eqn_config.epsilon
        self.q = eqn_config.q

    def _fill(self, p):
        p.a, p.epsilon, p.q = float(self.a), float(self.epsl), float(self.q)


class ekn(Equation):
    """Diffusive Eikonal equation (equation.py:240-276)"""

    eqn_id = _lib.EQN_EKN

    def __init__(self, eqn_config):
        super(ekn, self).__init__(eqn_config)
        self.a2 = eqn_config.a2
        self.a3 = eqn_config.a3
        self.epsl = 1 / 2 / self.a2 / self.dim

    def _fill(self, p):
        p.a2, p.a3 = float(self.a2), float(self.a3)


EKN = ekn  # the shipped configs say "EKN" (configs/ekn_d20.json:4); documented deviation


class LQR_var(Equation):
    """linear quadratic regulator with state-dependent diffusion (equation.py:278-311)"""

    eqn_id = _lib.EQN_LQR_VAR

    def __init__(self, eqn_config):
        super(LQR_var, self).__init__(eqn_config)
        self.k = (np.sqrt(5) - 1) / 2
        self.q = eqn_config.q
        self.beta = eqn_config.beta
        self.epsilon = eqn_config.epsilon

    def _fill(self, p):
        p.q, p.beta, p.epsilon, p.k = float(self.q), float(self.beta), float(self.epsilon), float(self.k)


def is_ekn(name: str) -> bool:
    return name in ("ekn", "EKN")
