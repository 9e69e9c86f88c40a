"""ORACLE (test infrastructure only): restatement of solver.py on torch-CPU float64.

Keras semantics are written out explicitly:
inference-mode BatchNormalization with moving mean 0 / variance 1 and eps 1e-6,
`y + relu(y)` activation, bias-free hidden Dense layers, TF-form Adam and
PiecewiseConstantDecay.  Weights are plain tensors so tests can load the
product's initial weights and compare step by step.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .precision import dtype as _dt

DELTA_CLIP = 50.0  # solver.py:5
BN_EPS = 1e-6      # solver.py:242


class DeepNN:
    """solver.py:227-278.  params: bn_gamma[L+2], bn_beta[L+2], W[L+1], b (last layer)."""

    def __init__(self, config, AC, params=None):
        self.AC = AC
        self.d = config.eqn_config.control_dim
        self.eqn = config.eqn_config.eqn_name
        self.dim = config.eqn_config.dim
        hid = config.net_config.num_hiddens_actor if AC == "actor" else config.net_config.num_hiddens_critic
        if AC == "critic":
            out = 1
        elif AC == "critic_grad":
            out = self.dim
        elif AC == "actor" and self.eqn in ("ekn", "EKN"):
            out = self.d + 1
        else:
            out = self.d
        self.sizes = [self.dim] + list(hid) + [out]
        self.params = params

    def __call__(self, x, training=False, need_grad=False):
        p = self.params
        L = len(self.sizes) - 2
        inv = lambda i: torch.rsqrt(torch.tensor(1.0 + BN_EPS, dtype=_dt())) * p["bn_gamma"][i]
        y = x * inv(0) + p["bn_beta"][0]
        for i in range(L):
            y = y @ p["W"][i]
            y = y * inv(i + 1) + p["bn_beta"][i + 1]
            y = y + torch.relu(y)
        y = y @ p["W"][L] + p["b"]
        y = y * inv(L + 1) + p["bn_beta"][L + 1]
        if self.AC == "actor" and self.eqn in ("ekn", "EKN"):
            norm_y = torch.sum(y[:, 0:self.d] ** 2, 1, keepdim=True) ** 0.5
            y = y[:, 0:self.d] / (1e-15 + torch.relu(y[:, self.d:self.d + 1]) + norm_y)
        return y

    def trainable(self):
        p = self.params
        return list(p["bn_gamma"]) + list(p["bn_beta"]) + list(p["W"]) + [p["b"]]


def init_params(sizes, gen: torch.Generator):
    """Keras initialisers: BN gamma U(0.1,0.5), beta N(0,0.1); Dense glorot_uniform; bias 0."""
    L = len(sizes) - 2
    bn_dims = [sizes[0]] + list(sizes[1:-1]) + [sizes[-1]]
    g = [torch.rand(n, generator=gen, dtype=_dt()) * 0.4 + 0.1 for n in bn_dims]
    b = [torch.randn(n, generator=gen, dtype=_dt()) * 0.1 for n in bn_dims]
    W = []
    for i in range(L + 1):
        lim = np.sqrt(6.0 / (sizes[i] + sizes[i + 1]))
        W.append((torch.rand(sizes[i], sizes[i + 1], generator=gen, dtype=_dt()) * 2 - 1) * lim)
    return {"bn_gamma": g, "bn_beta": b, "W": W, "b": torch.zeros(sizes[-1], dtype=_dt())}


class CriticModel:
    """solver.py:138-191"""

    def __init__(self, config, bsde, params_value=None, params_grad=None):
        self.eqn_config = config.eqn_config
        self.train_config = config.train_config
        self.bsde = bsde
        self.NN_value = DeepNN(config, "critic", params_value)
        self.NN_value_grad = DeepNN(config, "critic_grad", params_grad)
        self.gamma = config.eqn_config.discount
        self.propagate = bsde.propagate_naive if self.train_config.scheme == "naive" else bsde.propagate_adaptive

    def control(self, x, cheat_control, model_actor):
        if not cheat_control:
            return model_actor.NN_control(x, training=False, need_grad=False)
        return self.bsde.u_true(x)

    def __call__(self, inputs, model_actor, training, cheat_control):
        x0, dw, x_bdry = [torch.as_tensor(np.asarray(a), dtype=_dt()) if not isinstance(a, torch.Tensor) else a
                          for a in inputs]
        num_sample = dw.shape[0]
        y = 0
        discount = 1
        N = self.eqn_config.num_time_interval_critic
        x, dt, coef = self.propagate(num_sample, x0, dw, model_actor.NN_control, training,
                                     self.eqn_config.total_time_critic, N, cheat_control)
        for t in range(N):
            u = self.control(x[:, :, t], cheat_control, model_actor)
            w = self.bsde.w_tf(x[:, :, t], u)
            delta_y_drift = w * discount
            delta_y_drift_coef = coef[:, t:t + 1] * dt[:, t:t + 1]
            y = y + delta_y_drift * delta_y_drift_coef
            if self.train_config.TD_type == "TD1":
                dd = torch.einsum("bij,bj->bi", self.bsde.sigma(x[:, :, t], u, num_sample), dw[:, :, t])
                dd = torch.sum(dd * self.NN_value_grad(x[:, :, t], training, need_grad=False), 1, keepdim=True)
                dd = dd * discount
                y = y - dd * (coef[:, t:t + 1] * torch.sqrt(dt[:, t:t + 1]))
            discount = discount * torch.exp(-self.gamma * dt[:, t:t + 1] * coef[:, t:t + 1])
        delta = (self.NN_value(x[:, :, 0], training, need_grad=False) - y
                 - self.NN_value(x[:, :, -1], training, need_grad=False) * discount)
        delta_bdry = self.NN_value(x_bdry, training, need_grad=False) - self.bsde.Z_tf(x_bdry)
        return delta, delta_bdry


class ActorModel:
    """solver.py:193-224"""

    def __init__(self, config, bsde, params=None):
        self.eqn_config = config.eqn_config
        self.bsde = bsde
        self.NN_control = DeepNN(config, "actor", params)
        self.gamma = config.eqn_config.discount
        self.propagate = bsde.propagate_naive if config.train_config.scheme == "naive" else bsde.propagate_adaptive

    def __call__(self, inputs, model_critic, training, cheat_value, cheat_control):
        x0, dw, x_bdry = [torch.as_tensor(np.asarray(a), dtype=_dt()) if not isinstance(a, torch.Tensor) else a
                          for a in inputs]
        num_sample = dw.shape[0]
        y = 0
        N = self.eqn_config.num_time_interval_actor
        x, dt, coef = self.propagate(num_sample, x0, dw, self.NN_control, training,
                                     self.eqn_config.total_time_actor, N, cheat_control)
        discount = 1
        for t in range(N):
            if not cheat_control:
                w = self.bsde.w_tf(x[:, :, t], self.NN_control(x[:, :, t], training, need_grad=False))
            else:
                w = self.bsde.w_tf(x[:, :, t], self.bsde.u_true(x[:, :, t]))
            y = y + coef[:, t:t + 1] * w * dt[:, t:t + 1] * discount
            discount = discount * torch.exp(-self.gamma * dt[:, t:t + 1] * coef[:, t:t + 1])
        if not cheat_value:
            y = y + model_critic.NN_value(x[:, :, -1], training, need_grad=False) * discount
        else:
            y = y + self.bsde.V_true(x[:, :, -1]) * discount
        return y


def huber(delta):
    """solver.py:76-77"""
    return torch.mean(torch.where(torch.abs(delta) < DELTA_CLIP, torch.square(delta),
                                  2 * DELTA_CLIP * torch.abs(delta) - DELTA_CLIP ** 2))


class PiecewiseConstantDecay:
    """tf.keras.optimizers.schedules.PiecewiseConstantDecay (solver.py:16-19)."""

    def __init__(self, boundaries, values):
        self.boundaries, self.values = list(boundaries), list(values)

    def __call__(self, step):
        for b, v in zip(self.boundaries, self.values):
            if step <= b:
                return v
        return self.values[-1]


class TFAdam:
    """tf.keras Adam (solver.py:20-21): ResourceApplyAdam update, eps outside the sqrt."""

    def __init__(self, schedule, beta_1=0.9, beta_2=0.999, epsilon=1e-8):
        self.schedule, self.b1, self.b2, self.eps = schedule, beta_1, beta_2, epsilon
        self.iterations = 0
        self.slots = {}

    def apply_gradients(self, grads_and_vars):
        lr = self.schedule(self.iterations)
        t = self.iterations + 1
        b1p, b2p = self.b1 ** t, self.b2 ** t
        alpha = lr * np.sqrt(1 - b2p) / (1 - b1p)
        for g, v in grads_and_vars:
            if g is None:
                continue
            m, s = self.slots.setdefault(id(v), (torch.zeros_like(v), torch.zeros_like(v)))
            m += (g - m) * (1 - self.b1)
            s += (g * g - s) * (1 - self.b2)
            with torch.no_grad():
                v -= (m * alpha) / (torch.sqrt(s) + self.eps)
        self.iterations += 1


class ActorCriticSolver:
    """solver.py:7-136 (single process, host numpy sampling)."""

    def __init__(self, config, bsde, params=None):
        self.eqn_config = config.eqn_config
        self.net_config = config.net_config
        self.train_config = config.train_config
        self.bsde = bsde
        p = params or {}
        self.model_critic = CriticModel(config, bsde, p.get("critic"), p.get("critic_grad"))
        self.model_actor = ActorModel(config, bsde, p.get("actor"))
        nc = self.net_config
        self.optimizer_critic = TFAdam(PiecewiseConstantDecay(nc.lr_boundaries_critic, nc.lr_values_critic))
        self.optimizer_actor = TFAdam(PiecewiseConstantDecay(nc.lr_boundaries_actor, nc.lr_values_actor))
        self.sample = bsde.sample_normal if self.train_config.sample_type == "normal" else bsde.sample_bounded
        self.cheat_value_in_actor = self.train_config.train == "actor"
        self.cheat_control_in_critic = self.train_config.train == "critic"

    def loss_critic(self, inputs, training, cheat_control):
        delta, delta_bdry = self.model_critic(inputs, self.model_actor, training, cheat_control)
        return (huber(delta) + huber(delta_bdry)) * 100

    def loss_actor(self, inputs, training, cheat_value, cheat_control):
        return torch.mean(self.model_actor(inputs, self.model_critic, training, cheat_value, cheat_control))

    def critic_vars(self):
        return self.model_critic.NN_value.trainable() + self.model_critic.NN_value_grad.trainable()

    def actor_vars(self):
        return self.model_actor.NN_control.trainable()

    def grad_critic(self, inputs, training, cheat_control):
        vs = self.critic_vars()
        for v in vs:
            v.requires_grad_(True)
        loss = self.loss_critic(inputs, training, cheat_control)
        return list(torch.autograd.grad(loss, vs, allow_unused=True)), loss

    def grad_actor(self, inputs, training, cheat_value, cheat_control):
        vs = self.actor_vars()
        for v in vs:
            v.requires_grad_(True)
        loss = self.loss_actor(inputs, training, cheat_value, cheat_control)
        return list(torch.autograd.grad(loss, vs, allow_unused=True)), loss

    def train_step_critic(self, data):
        g, _ = self.grad_critic(data, False, self.cheat_control_in_critic)
        self.optimizer_critic.apply_gradients(zip(g, self.critic_vars()))

    def train_step_actor(self, data):
        g, _ = self.grad_actor(data, False, self.cheat_value_in_actor, False)
        self.optimizer_actor.apply_gradients(zip(g, self.actor_vars()))

    def err_value(self, inputs):
        x0 = torch.as_tensor(inputs[0], dtype=_dt())
        with torch.no_grad():
            e = torch.sum(torch.square(self.bsde.V_true(x0) - self.model_critic.NN_value(x0)))
            return torch.sqrt(e / torch.sum(torch.square(self.bsde.V_true(x0))))

    def err_control(self, inputs):
        x0 = torch.as_tensor(inputs[0], dtype=_dt())
        with torch.no_grad():
            e = torch.sum(torch.square(self.bsde.u_true(x0) - self.model_actor.NN_control(x0)))
            return torch.sqrt(e / torch.sum(torch.square(self.bsde.u_true(x0))))

    def err_value_grad(self, inputs):
        x0 = torch.as_tensor(inputs[0], dtype=_dt())
        with torch.no_grad():
            e = torch.sum(torch.square(self.bsde.V_grad_true(x0) - self.model_critic.NN_value_grad(x0)))
            return torch.sqrt(e / torch.sum(torch.square(self.bsde.V_grad_true(x0))))

    def err_value_infty(self, inputs):
        x0 = torch.as_tensor(inputs[0], dtype=_dt())
        with torch.no_grad():
            return torch.max(torch.abs(self.bsde.V_true(x0) - self.model_critic.NN_value(x0)))

    def err_cost(self, inputs):
        x0 = torch.as_tensor(inputs[0], dtype=_dt())
        with torch.no_grad():
            y = self.model_actor(inputs, self.model_critic, False, False, False)
            return torch.mean(y - self.model_critic.NN_value(x0))

    def train(self):
        """solver.py:36-71"""
        start_time = time.time()
        hist = []
        nc, ec = self.net_config, self.eqn_config
        vc = self.sample(nc.valid_size, ec.num_time_interval_critic)
        va = self.sample(nc.valid_size, ec.num_time_interval_actor)
        vcost = self.bsde.sample0(nc.valid_size, ec.num_time_interval_actor)
        with torch.no_grad():
            true_loss_actor = float(self.loss_actor(va, False, True, True))
        for step in range(nc.num_iterations + 1):
            if step % nc.logging_frequency == 0:
                with torch.no_grad():
                    lc = float(self.loss_critic(vc, False, False))
                    la = float(self.loss_actor(va, False, False, False))
                row = [step, lc, la, float(self.err_value(vc)), float(self.err_value_infty(vc)),
                       float(self.err_control(va)), float(self.err_value_grad(vc)),
                       float(self.err_cost(vcost)), time.time() - start_time]
                hist.append(row)
            if step == nc.num_iterations:
                hist.append([0, 0.0, true_loss_actor, 0.0, 0.0, 0.0, 0.0, 0.0, time.time() - start_time])
            if self.train_config.train in ("actor-critic", "critic"):
                self.train_step_critic(self.sample(nc.batch_size, ec.num_time_interval_critic))
            if self.train_config.train in ("actor-critic", "actor"):
                self.train_step_actor(self.sample(nc.batch_size, ec.num_time_interval_actor))
        return np.array(hist)
