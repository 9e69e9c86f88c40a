"""ORACLE (test infrastructure only): restatement of equation.py on torch-CPU / numpy.

Every TF op of the reference is replaced by the torch op with the same meaning,
in the same order, on float64 tensors (oracle.precision; float32 only for bench.py's CPU timing); gradients come from torch autograd (the
analogue of tf.GradientTape).  Tensor layouts are the reference's: x [B, d],
dw [B, d, N], x_smp [B, d, N+1], dt / coef [B, N].
"""
from __future__ import annotations

import numpy as np
import torch

from .precision import dtype as _dt
from scipy.stats import multivariate_normal as normal


def _t(a):
    return a if isinstance(a, torch.Tensor) else torch.as_tensor(np.asarray(a), dtype=_dt())


class Equation:
    """equation.py:5-142"""

    def __init__(self, eqn_config):
        self.dim = eqn_config.dim
        self.gamma = eqn_config.discount
        self.R = eqn_config.R
        self.control_dim = eqn_config.control_dim

    # ---- samplers (equation.py:13-44), same numpy/scipy call sequence ----
    def sample_normal(self, num_sample, N):
        r_Sample = np.random.uniform(low=0, high=self.R, size=[num_sample, 1])
        r = r_Sample ** (1 / self.dim) * (self.R ** ((self.dim - 1) / self.dim))
        angle = normal.rvs(size=[num_sample, self.dim])
        norm = np.sqrt(np.sum(angle ** 2, 1, keepdims=True))
        x0 = r * angle / norm
        dw_sample = normal.rvs(size=[num_sample, self.dim, N])
        x_bdry = normal.rvs(size=[num_sample, self.dim])
        norm = np.sqrt(np.sum(np.square(x_bdry), 1, keepdims=True))
        x_bdry = self.R * x_bdry / norm
        return x0, dw_sample, x_bdry

    def sample_bounded(self, num_sample, N):
        r_Sample = np.random.uniform(low=0, high=self.R, size=[num_sample, 1])
        r = r_Sample ** (1 / self.dim) * (self.R ** ((self.dim - 1) / self.dim))
        angle = normal.rvs(size=[num_sample, self.dim])
        norm = np.sqrt(np.sum(angle ** 2, 1, keepdims=True))
        x0 = r * angle / norm
        dw_sample = np.random.randint(6, size=[num_sample, self.dim, N])
        dw_sample = np.floor((dw_sample - 1) / 4) * np.sqrt(3.0)
        x_bdry = normal.rvs(size=[num_sample, self.dim])
        norm = np.sqrt(np.sum(np.square(x_bdry), 1, keepdims=True))
        x_bdry = self.R * x_bdry / norm
        return x0, dw_sample, x_bdry

    def sample0(self, num_sample, N):
        x0 = np.zeros(shape=[num_sample, self.dim]) + 0.01
        dw_sample = normal.rvs(size=[num_sample, self.dim, N])
        x_bdry = normal.rvs(size=[num_sample, self.dim])
        norm = np.sqrt(np.sum(np.square(x_bdry), 1, keepdims=True))
        x_bdry = self.R * x_bdry / norm
        return x0, dw_sample, x_bdry

    # ---- rollouts ----
    def propagate_naive(self, num_sample, x0, dw_sample, NN_control, training, T, N, cheat):
        """equation.py:46-71"""
        x0, dw_sample = _t(x0), _t(dw_sample)
        delta_t = T / N
        sqrt_delta_t = np.sqrt(delta_t)
        xs = [x0]
        coefs = []
        x_i = x0
        flag = torch.ones(num_sample, dtype=_dt())
        for i in range(N):
            u_i = self.u_true(x_i) if cheat else NN_control(x_i, training, need_grad=False)
            delta_x = (self.drift(x_i, u_i) * delta_t
                       + self.diffusion(x_i, u_i, dw_sample[:, :, i], num_sample) * sqrt_delta_t)
            x_next = x_i + delta_x
            Exit = self.b_tf(x_next)
            Exit = torch.ceil((torch.sign(Exit) + 1) / 2).reshape(num_sample)
            coef_i = flag * (1 - Exit)
            coefs.append(coef_i)
            x_i = x_i + delta_x * coef_i.reshape(num_sample, 1)
            xs.append(x_i)
            flag = flag * (1 - Exit)
        dt = torch.ones(num_sample, N, dtype=_dt()) * delta_t
        return torch.stack(xs, 2), dt, torch.stack(coefs, 1)

    def propagate_adaptive(self, num_sample, x0, dw_sample, NN_control, training, T, N, cheat):
        """equation.py:73-106"""
        x0, dw_sample = _t(x0), _t(dw_sample)
        delta_t = T / N
        xs, coefs, dts = [x0], [], []
        x_i = x0
        x0_norm = torch.sqrt(torch.sum(x0 ** 2, 1))
        layer = self.sigma_Up * np.sqrt(3 * self.dim * delta_t)
        temp = torch.sign(self.R - x0_norm - layer) + torch.sign(self.R - x0_norm)
        flag = torch.ones(num_sample, dtype=_dt()) + torch.floor(temp / 2)
        for i in range(N):
            xi_norm = torch.sqrt(torch.sum(x_i ** 2, 1))
            dt_i = ((2 * flag - (flag ** 2)) * ((self.R - xi_norm) ** 2)
                    / (3 * self.dim * self.sigma_Up ** 2) + (flag ** 2 - 2 * flag + 1) * delta_t)
            # tf.maximum: gradient to the first argument where dt_i >= bound (ties included)
            bound = delta_t * 1e-4
            dt_i = torch.where(dt_i >= bound, dt_i, torch.full_like(dt_i, bound))
            u_i = self.u_true(x_i) if cheat else NN_control(x_i, training, need_grad=False)
            delta_x = (self.drift(x_i, u_i) * dt_i.reshape(num_sample, 1)
                       + self.diffusion(x_i, u_i, dw_sample[:, :, i], num_sample)
                       * torch.sqrt(dt_i).reshape(num_sample, 1))
            x_next = x_i + delta_x
            x_next_norm = torch.sqrt(torch.sum(x_next ** 2, 1))
            temp = torch.sign(self.R - x_next_norm - layer) + torch.sign(self.R - x_next_norm)
            new_flag = (torch.ones(num_sample, dtype=_dt()) + torch.floor(temp / 2)) * torch.sign(flag)
            coef_i = torch.sign(flag) * torch.sign(new_flag)
            coefs.append(coef_i)
            dts.append(dt_i)
            x_i = x_i + delta_x * coef_i.reshape(num_sample, 1)
            xs.append(x_i)
            flag = new_flag
        return torch.stack(xs, 2), torch.stack(dts, 1), torch.stack(coefs, 1)

    def b_np(self, x):
        return np.sum(x ** 2, 1, keepdims=True) - (self.R ** 2)

    def b_tf(self, x):
        return torch.sum(x ** 2, 1, keepdim=True) - (self.R ** 2)

    def diffusion(self, x, u, dw, num_sample):
        # tf.linalg.matvec(sigma, dw) with the dense [B, d, d] sigma (equation.py:176 etc.)
        return torch.einsum("bij,bj->bi", self.sigma(x, u, num_sample), dw)


class LQR(Equation):
    """equation.py:144-176"""

    def __init__(self, eqn_config):
        super().__init__(eqn_config)
        self.p = eqn_config.p
        self.q = eqn_config.q
        self.beta = eqn_config.beta
        self.k = (((self.gamma ** 2) * (self.q ** 2) + 4 * self.p * self.q * (self.beta ** 2)) ** 0.5
                  - self.q * self.gamma) / (self.beta ** 2) / 2
        self.sigma_Up = np.sqrt(2.0)

    def w_tf(self, x, u):
        return torch.sum(self.p * torch.square(x) + self.q * torch.square(u), 1, keepdim=True) - 2 * self.k * self.dim

    def Z_tf(self, x):
        return 0 * torch.sum(x, 1, keepdim=True) + self.k * (self.R ** 2)

    def V_true(self, x):
        return torch.sum(torch.square(x), 1, keepdim=True) * self.k

    def u_true(self, x):
        return -self.beta * self.k / self.q * x

    def V_grad_true(self, x):
        return 2 * self.k * x

    def sigma(self, x, u, num_sample):
        return np.sqrt(2.0) * torch.ones(num_sample, 1, 1, dtype=_dt()) * torch.eye(self.dim, dtype=_dt())

    def drift(self, x, u):
        return self.beta * u


class VDP(Equation):
    """equation.py:179-238"""

    def __init__(self, eqn_config):
        super().__init__(eqn_config)
        self.a = eqn_config.a
        self.epsl = eqn_config.epsilon
        self.q = eqn_config.q
        self.sigma_Up = np.sqrt(2.0)

    def _split(self, x):
        d = self.control_dim
        x1, x2 = x[:, 0:d], x[:, d:self.dim]
        px1 = torch.cat([x1[:, 1:d], x1[:, 0:1]], 1)
        px2 = torch.cat([x2[:, 1:d], x2[:, 0:1]], 1)
        nx1 = torch.cat([x1[:, d - 1:d], x1[:, 0:d - 1]], 1)
        nx2 = torch.cat([x2[:, d - 1:d], x2[:, 0:d - 1]], 1)
        return x1, x2, px1, px2, nx1, nx2

    def w_tf(self, x, u):
        x1, x2, px1, px2, nx1, nx2 = self._split(x)
        dv1 = 2 * self.a * x1 - self.epsl * (px1 + nx1)
        dv2 = 2 * self.a * x2 - self.epsl * (px2 + nx2)
        temp = (-self.gamma * self.epsl * (x1 * px1 + x2 * px2) + (dv2 ** 2) / 4 / self.q - x2 * dv1
                - ((1 - x1 ** 2) * x2 - x1) * dv2)
        return (torch.sum(temp + self.q * (u ** 2), 1, keepdim=True)
                + self.gamma * self.a * torch.sum(x ** 2, 1, keepdim=True) - 2 * self.a * self.dim)

    def Z_tf(self, x):
        return self.V_true(x)

    def V_true(self, x):
        x1, x2, px1, px2, _, _ = self._split(x)
        return (self.a * torch.sum(x ** 2, 1, keepdim=True)
                - self.epsl * torch.sum(x1 * px1 + x2 * px2, 1, keepdim=True))

    def u_true(self, x):
        _, x2, _, px2, _, nx2 = self._split(x)
        return -(2 * self.a * x2 - self.epsl * (px2 + nx2)) / 2 / self.q

    def V_grad_true(self, x):
        x1, x2, px1, px2, nx1, nx2 = self._split(x)
        return torch.cat([2 * self.a * x1 - self.epsl * (px1 + nx1),
                          2 * self.a * x2 - self.epsl * (px2 + nx2)], 1)

    def sigma(self, x, u, num_sample):
        return np.sqrt(2.0) * torch.ones(num_sample, 1, 1, dtype=_dt()) * torch.eye(self.dim, dtype=_dt())

    def drift(self, x, u):
        x_1 = x[:, 0:self.control_dim]
        x_2 = x[:, self.control_dim:self.dim]
        return torch.cat([x_2, (1 - x_1 ** 2) * x_2 - x_1 + u], 1)


class ekn(Equation):
    """equation.py:240-276"""

    def __init__(self, eqn_config):
        super().__init__(eqn_config)
        self.a2 = eqn_config.a2
        self.a3 = eqn_config.a3
        self.epsl = 1 / 2 / self.a2 / self.dim
        self.sigma_Up = np.sqrt(2.0)

    def w_tf(self, x, u):
        return 0 * torch.sum(x, 1, keepdim=True) + 1

    def Z_tf(self, x):
        return self.V_true(x)

    def V_true(self, x):
        x_norm = torch.sum(x ** 2, 1, keepdim=True) ** 0.5
        return self.a3 * x_norm ** 3 - self.a2 * x_norm ** 2

    def u_true(self, x):
        x_norm = torch.sum(x ** 2, 1, keepdim=True) ** 0.5
        return x / x_norm

    def V_grad_true(self, x):
        x_norm = torch.sum(x ** 2, 1, keepdim=True) ** 0.5
        return (3 * self.a3 * x_norm - 2 * self.a2) * x

    def sigma(self, x, u, num_sample):
        return np.sqrt(2.0) * torch.ones(num_sample, 1, 1, dtype=_dt()) * torch.eye(self.dim, dtype=_dt())

    def drift(self, x, u):
        x_norm = torch.sum(x ** 2, 1, keepdim=True) ** 0.5
        c = 3 * (self.dim + 1) * self.a3 / 2 / self.a2 / self.dim / (2 * self.a2 - 3 * self.a3 * x_norm)
        return c * u


class LQR_var(Equation):
    """equation.py:278-311"""

    def __init__(self, eqn_config):
        super().__init__(eqn_config)
        self.k = (np.sqrt(5) - 1) / 2
        self.q = eqn_config.q
        self.beta = eqn_config.beta
        self.epsilon = eqn_config.epsilon
        self.sigma_Up = np.sqrt(2.0)

    def w_tf(self, x, u):
        temp = torch.sum(self.k ** 2 * (self.beta + 2 * self.epsilon) ** 2 * x ** 2
                         / (self.q + 2 * self.k * self.epsilon ** 2 * x ** 2), 1, keepdim=True)
        return temp + torch.sum(self.gamma * self.k * torch.square(x) + self.q * torch.square(u), 1, keepdim=True) - 2 * self.k * self.dim

    def Z_tf(self, x):
        return 0 * torch.sum(x, 1, keepdim=True) + self.k * (self.R ** 2)

    def V_true(self, x):
        return torch.sum(torch.square(x), 1, keepdim=True) * self.k

    def u_true(self, x):
        return -(self.beta + 2 * self.epsilon) * x / (self.q / self.k + 2 * self.epsilon ** 2 * x ** 2)

    def V_grad_true(self, x):
        return 2 * self.k * x

    def sigma(self, x, u, num_sample):
        return np.sqrt(2.0) * torch.diag_embed(1 + self.epsilon * x * u)

    def drift(self, x, u):
        return self.beta * u


EKN = ekn  # configs name the class "EKN" (configs/ekn_d20.json:4); the reference has only `ekn`


def make(eqn_config):
    return {"LQR": LQR, "VDP": VDP, "ekn": ekn, "EKN": ekn, "LQR_var": LQR_var}[eqn_config.eqn_name](eqn_config)
