"""Actor-critic solver with the reference's surface (solver.py:7-278).

`ActorCriticSolver(config, bsde).train()` returns the same 7-tuple as the
reference (solver.py:71).  The hot path — rollouts, running cost, TD target
assembly and the per-step backward — runs in libdpac (HIP, gfx950), and so do
the MLPs on the GPU path (fused into the actor's rollout and BPTT, row-parallel
kernels for the critic's V and G networks, parameter gradients) and the Adam
update; PyTorch-ROCm holds the parameters, streams, HIP graphs and the
torch.distributed exchange.  The PyTorch forms of DeepNN stay as test references
(ops.ROW_MLP / ops.BPTT_MODE / ops.PARAM_GRADS).

Deliberate differences from the reference: the actor MLP is
evaluated once per step and its output reused for the cost (the reference
evaluates it twice on identical inputs, equation.py:57 + solver.py:167/215);
the critic's G network runs as one batched [N*B, d] pass instead of N calls.
Both give the same values and gradients.
"""
from __future__ import annotations

import contextlib
import logging
import os
import time

import numpy as np
import torch
from torch import nn

from . import _lib, ops
from .config import set_floatx, torch_dtype
from .equation import SAMPLE_TYPES, SCHEMES, Equation, TrajectoryBatch, is_ekn
from .parallel import SingleProcess

DELTA_CLIP = 50.0  # solver.py:5
BN_EPS = 1e-6      # solver.py:242


# ---------------------------------------------------------------------------
# Networks
# ---------------------------------------------------------------------------
class DeepNN(nn.Module):
    """solver.py:227-278: bn -> (dense -> bn -> y+relu(y)) * L -> dense -> bn.

    BatchNormalization is always called with training=False in the reference
    (solver.py:101,106,155), i.e. an affine map with the initial moving
    statistics (mean 0, variance 1): y = x * gamma/sqrt(1+eps) + beta.
    """

    def __init__(self, config, AC, generator=None, dtype=None, device=None):
        super().__init__()
        self.AC = AC
        ec, nc = config.eqn_config, config.net_config
        self.d = ec.control_dim
        self.eqn = ec.eqn_name
        dim = ec.dim
        hid = list(nc.num_hiddens_actor if AC == "actor" else nc.num_hiddens_critic)
        if AC == "critic":
            out = 1
        elif AC == "critic_grad":
            out = dim
        elif AC == "actor" and is_ekn(self.eqn):
            out = self.d + 1
        else:
            out = self.d
        self.sizes = [dim] + hid + [out]
        self.ekn_head = AC == "actor" and is_ekn(self.eqn)
        dtype = dtype or torch_dtype()
        gen = generator if generator is not None else torch.Generator().manual_seed(0)
        bn_dims = [dim] + hid + [out]
        mk = lambda t: nn.Parameter(t.to(dtype=dtype, device=device))
        # Keras initialisers (solver.py:243-244; Dense defaults glorot_uniform / zeros)
        self.bn_gamma = nn.ParameterList(
            [mk(torch.rand(n, generator=gen, dtype=torch.float64) * 0.4 + 0.1) for n in bn_dims])
        self.bn_beta = nn.ParameterList(
            [mk(torch.randn(n, generator=gen, dtype=torch.float64) * 0.1) for n in bn_dims])
        Ws = []
        for i in range(len(self.sizes) - 1):
            lim = np.sqrt(6.0 / (self.sizes[i] + self.sizes[i + 1]))
            Ws.append(mk((torch.rand(self.sizes[i], self.sizes[i + 1], generator=gen,
                                     dtype=torch.float64) * 2 - 1) * lim))
        self.W = nn.ParameterList(Ws)
        self.b = mk(torch.zeros(out, dtype=torch.float64))
        self.register_buffer("bn_rs", torch.rsqrt(torch.tensor(1.0 + BN_EPS, dtype=dtype)).to(device),
                             persistent=False)

    def forward(self, x, training=False, need_grad=False, const_params=False):
        """x [rows, d], or [S, R, d] for a stack of S batches (e.g. the critic's G over
        all N steps): then every product is a batched GEMM over S with the weight
        broadcast, so autograd forms the weight gradients as S partial products and
        a sum instead of one GEMM with a 10^5-long reduction.  const_params: the
        parameters are not differentiated (kernel path: no parameter-gradient work)."""
        if x.is_cuda and ops.ROW_MLP == "kernel" and self.fused_ok():
            y = ops.row_mlp(self, x, const_params)  # hand-written MFMA kernels (dpac_mlp_rows_*)
            return self._ekn(y) if self.ekn_head else y
        rs = self.bn_rs
        g, bt, W = self.bn_gamma, self.bn_beta, self.W
        L = len(self.sizes) - 2
        if x.dim() == 3:
            S = x.shape[0]
            mm = lambda a, w: torch.bmm(a, w.unsqueeze(0).expand(S, -1, -1))
            mm_bias = lambda b, a, w: torch.baddbmm(b, a, w.unsqueeze(0).expand(S, -1, -1))
        else:
            mm, mm_bias = torch.mm, torch.addmm
        y = torch.addcmul(bt[0], x, rs * g[0])
        for i in range(L):
            y = mm(y, W[i])
            y = torch.addcmul(bt[i + 1], y, rs * g[i + 1])
            y = y + torch.relu(y)
        y = mm_bias(self.b, y, W[L])
        y = torch.addcmul(bt[L + 1], y, rs * g[L + 1])
        return self._ekn(y) if self.ekn_head else y

    def _ekn(self, y):
        """The Eikonal actor head, solver.py:272-274."""
        d = self.d
        norm_y = torch.sum(y[..., 0:d] ** 2, -1, keepdim=True) ** 0.5
        return y[..., 0:d] / (1e-15 + torch.relu(y[..., d:d + 1]) + norm_y)

    def fused_ok(self) -> bool:
        """Whether dpac_rollout_nn_fwd can run this network (layer and width limits)."""
        return 1 <= len(self.sizes) - 2 <= _lib.MLP_MAX_HIDDEN and max(self.sizes) <= _lib.MLP_MAX_WIDTH

    @torch.no_grad()
    def mlp_prepared(self):
        """(view, weight_t, weight_t_km) of mlp_prepare with the backward images too: one
        launch for a forward over rows and its backward (ops.row_mlp_backward(prepared=))."""
        return ops.mlp_prepare([g.detach() for g in self.bn_gamma], [bt.detach() for bt in self.bn_beta],
                               [w.detach() for w in self.W], self.b.detach(), self.ekn_head, True)

    @torch.no_grad()
    def mlp_view(self):
        """This network as dpac_rollout_nn_fwd reads it (BN scale = rs * gamma, the same
        product forward() forms)."""
        if not self.bn_rs.is_cuda:
            rs = self.bn_rs
            return ops.MlpView([rs * g for g in self.bn_gamma], [bt.detach() for bt in self.bn_beta],
                               [w.detach() for w in self.W], self.b.detach(), self.ekn_head)
        view, _, _ = ops.mlp_prepare([g.detach() for g in self.bn_gamma], [bt.detach() for bt in self.bn_beta],
                                     [w.detach() for w in self.W], self.b.detach(), self.ekn_head, False)
        return view

    def trainable_variables(self):
        return list(self.bn_gamma) + list(self.bn_beta) + list(self.W) + [self.b]

    def export_params(self):
        c = lambda t: t.detach().to("cpu", torch.float64).clone()
        return {"bn_gamma": [c(t) for t in self.bn_gamma], "bn_beta": [c(t) for t in self.bn_beta],
                "W": [c(t) for t in self.W], "b": c(self.b)}

    @torch.no_grad()
    def load_params(self, p):
        for dst, src in zip(self.trainable_variables(),
                            list(p["bn_gamma"]) + list(p["bn_beta"]) + list(p["W"]) + [p["b"]]):
            dst.copy_(torch.as_tensor(src).to(dst))


class CriticModel(nn.Module):
    """solver.py:138-191: returns (delta, delta_bdry), each [B, 1]."""

    def __init__(self, config, bsde, generator=None, dtype=None, device=None):
        super().__init__()
        self.eqn_config, self.net_config, self.train_config = (
            config.eqn_config, config.net_config, config.train_config)
        self.bsde = bsde
        self.NN_value = DeepNN(config, "critic", generator, dtype, device)
        self.NN_value_grad = DeepNN(config, "critic_grad", generator, dtype, device)
        self.gamma = config.eqn_config.discount
        self.scheme = self.train_config.scheme
        self.td = _lib.TD1 if self.train_config.TD_type == "TD1" else _lib.TD2

    def forward(self, inputs, model_actor, training, cheat_control, G_fn=None):
        """G_fn(x[:N]) -> G [N, B, d] replaces NN_value_grad when given (the split
        critic step evaluates it with saves and makes it a leaf of the tape)."""
        x0, dw, x_bdry = Equation.to_native(inputs, self.NN_value.bn_rs.dtype)
        N = self.eqn_config.num_time_interval_critic
        T = self.eqn_config.total_time_critic
        B, d = x0.shape
        with torch.no_grad():  # the actor is fixed during the critic step
            x, dt, coef, u = self.bsde.rollout(self.scheme, x0, dw, T, N,
                                               model_actor.NN_control, cheat=cheat_control)
        G = None
        if self.td == _lib.TD1:
            G = (G_fn(x[:N]) if G_fn is not None    # [N, B, d], batched over the N steps
                 else self.NN_value_grad(x[:N], training))
        y, disc = ops.td_assemble(self.bsde.params(), self.td, x, u, dw, dt, coef, G,
                                  cost_order=_lib.COST_CRITIC)
        V = self.NN_value(torch.cat([x[0], x[N], x_bdry]), training)[:, 0]
        delta = V[:B] - y - V[B:2 * B] * disc                      # solver.py:189
        delta_bdry = V[2 * B:] - self.bsde.Z_tf(x_bdry)[:, 0]      # solver.py:190
        return delta.unsqueeze(1), delta_bdry.unsqueeze(1)


class ActorModel(nn.Module):
    """solver.py:193-224: returns the pathwise discounted cost y, [B, 1]."""

    def __init__(self, config, bsde, generator=None, dtype=None, device=None):
        super().__init__()
        self.eqn_config, self.net_config, self.train_config = (
            config.eqn_config, config.net_config, config.train_config)
        self.bsde = bsde
        self.NN_control = DeepNN(config, "actor", generator, dtype, device)
        self.gamma = config.eqn_config.discount
        self.scheme = SCHEMES[self.train_config.scheme]

    def forward(self, inputs, model_critic, training, cheat_value, cheat_control):
        x0, dw, x_bdry = Equation.to_native(inputs, self.NN_control.bn_rs.dtype)
        N = self.eqn_config.num_time_interval_actor
        T = self.eqn_config.total_time_actor
        eqp = self.bsde.params()
        B = x0.shape[0]
        if cheat_control:  # analytic control: one fused rollout + cost kernel
            x, _, _, _, y, disc = ops.rollout_analytic(eqp, self.scheme, x0, dw, T, N,
                                                       cost_order=_lib.COST_ACTOR)
            xN = x[N]
        elif self.NN_control.fused_ok():
            # fused NN rollout forward + manual BPTT backward (ops._ActorRolloutNN)
            y, disc, xN = ops.actor_rollout_nn(eqp, self.scheme, x0, dw, T, N, self.NN_control)
        else:
            flag = ops.flag_init(eqp, self.scheme, x0, T, N)
            disc = torch.ones(B, dtype=x0.dtype, device=x0.device)
            y = torch.zeros_like(disc)
            xN = x0
            for t in range(N):  # propagate (equation.py:83-105) fused with solver.py:213-219
                u = self.NN_control(xN, training)
                xN, disc, y, _, _, flag = ops.sde_step(eqp, self.scheme, T, N, xN, u, dw[t], flag,
                                                       disc, y, _lib.COST_ACTOR)
        if cheat_value:
            term = ops.v_true(eqp, xN)
        else:
            # the actor's tape watches only the actor (solver.py:95): V's parameters
            # are constants here
            term = model_critic.NN_value(xN, training, const_params=True)[:, 0]
        return (y + term * disc).unsqueeze(1)  # solver.py:220-223


# ---------------------------------------------------------------------------
# Optimizer (tf.keras Adam + PiecewiseConstantDecay, solver.py:16-21)
# ---------------------------------------------------------------------------
class PiecewiseConstantDecay:
    def __init__(self, boundaries, values):
        if len(values) != len(boundaries) + 1:
            raise ValueError("values must have one more entry than boundaries")
        self.boundaries, self.values = list(boundaries), list(values)

    def __call__(self, step):
        for b, v in zip(self.boundaries, self.values):
            if step <= b:
                return v
        return self.values[-1]


def tf_adam_scalars(lr, t, b1, b2, dtype):
    """ResourceApplyAdam's scalars in the variables' dtype T, as TF forms them (Keras
    Adam casts lr, beta_1, beta_2 to T, beta_i_power = pow(beta_i, t) in T; the op computes
    alpha = lr * sqrt(T(1) - beta2_power) / (T(1) - beta1_power) and T(1) - beta_i in T):
    (alpha, 1 - b1, 1 - b2) as Python floats holding T values."""
    f = np.float32 if dtype == torch.float32 else np.float64
    one, b1t, b2t = f(1), f(b1), f(b2)
    b1p, b2p = np.power(b1t, f(t)), np.power(b2t, f(t))
    alpha = f(lr) * np.sqrt(one - b2p) / (one - b1p)
    return float(alpha), float(one - b1t), float(one - b2t)


class TFAdam:
    """Adam with TensorFlow's update (ResourceApplyAdam):
        alpha = lr * sqrt(1 - b2^t) / (1 - b1^t)
        m += (g - m)(1 - b1);  v += (g^2 - v)(1 - b2);  var -= m*alpha / (sqrt(v) + eps)
    every scalar formed in the variables' dtype (tf_adam_scalars);
    lr = schedule(iterations) before the increment, t = iterations + 1.  None
    gradients are skipped (Keras filters them), iterations still advance."""

    def __init__(self, schedule, beta_1=0.9, beta_2=0.999, epsilon=1e-8):
        self.schedule, self.b1, self.b2, self.eps = schedule, beta_1, beta_2, epsilon
        self.iterations = 0
        self.state = {}

    @torch.no_grad()
    def apply_gradients(self, grads_and_vars, advance=True):
        """advance=False leaves `iterations` unchanged, so one optimizer step can be
        applied in parts (disjoint variable sets, same lr and t)."""
        lr = self.schedule(self.iterations)
        t = self.iterations + 1
        gs, vs, ms, ss = [], [], [], []
        for g, v in grads_and_vars:
            if g is None:
                continue
            st = self.state.get(v)
            if st is None:
                st = self.state[v] = (torch.zeros_like(v), torch.zeros_like(v))
            gs.append(g); vs.append(v); ms.append(st[0]); ss.append(st[1])
        if gs:
            alpha, omb1, omb2 = tf_adam_scalars(lr, t, self.b1, self.b2, vs[0].dtype)
        if gs and gs[0].is_cuda:  # one dpac_adam_apply launch (same arithmetic, same order)
            ops.adam_apply([v.data for v in vs], [g.detach().contiguous() for g in gs], ms, ss, alpha,
                           self.b1, self.b2, self.eps)
        elif gs:
            torch._foreach_add_(ms, torch._foreach_mul(torch._foreach_sub(gs, ms), omb1))
            g2 = torch._foreach_mul(gs, gs)
            torch._foreach_add_(ss, torch._foreach_mul(torch._foreach_sub(g2, ss), omb2))
            den = torch._foreach_add(torch._foreach_sqrt(ss), self.eps)
            torch._foreach_sub_(vs, torch._foreach_div(torch._foreach_mul(ms, alpha), den))
        if advance:
            self.iterations += 1

    def state_dict(self):
        return {"iterations": self.iterations}


# HIP-graph captures are thread-local: with a torch.distributed "nccl" (RCCL) process group
# alive, its watchdog thread queries events concurrently, and under the default global
# capture mode such a query invalidates an ongoing capture ("operation failed due to a
# previous error during capture", seen intermittently in round 3's RCCL test).
_CAPTURE_MODE = "thread_local"


class _GradGraph:
    """One gradient evaluation (forward + backward, no optimizer step) captured as a
    HIP graph over static input buffers.  Replaying it after copying a fresh batch
    in replaces the ~10^3 kernel launches of a step (the actor's reverse time loop,
    the critic's G network and TD assembly) with one graph launch; the optimizer
    still runs eagerly on the returned gradients, whose buffers the next replay
    overwrites.  Parameters are updated in place, so every replay sees the
    current weights."""

    def __init__(self, fn, batch: TrajectoryBatch):
        self.static = TrajectoryBatch(*[t.clone() for t in batch])
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up outside the capture (allocator, autograd)
            for _ in range(2):
                fn(self.static)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode=_CAPTURE_MODE):
            self.out = fn(self.static)

    def __call__(self, batch: TrajectoryBatch):
        for dst, src in zip(self.static, batch):
            dst.copy_(src)
        self.graph.replay()
        return list(self.out)


def _capture_redo(fns):
    """The deferred range-guard fallbacks a capture collected (ops.deferred_fallbacks) as one
    HIP graph, or None when there are none: no-op kernels while the split-fp16 status word
    is clear, the exact-f32 recomputation of their chains once it is set."""
    if not fns:
        return None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
        for f in fns:
            f()
    return g


class _SplitActorGraphs:
    """The actor step as two HIP graphs: the fused forward rollout with its backward
    saves (replayed on a side stream, so it runs beside the critic step: it reads only
    the actor's parameters, which the critic step does not change) and the gradient
    from those saves (after the critic update, which the terminal value V(x_N) needs;
    solver.py:67-70 order).  The backward graph reads the forward graph's outputs in
    place: nothing is copied between them."""

    def __init__(self, fwd_fn, bwd_fn, batch: TrajectoryBatch, side, defer=None):
        """defer: a context manager factory yielding the list the backward's deferred guard
        fallbacks go to (ActorCriticSolver._deferring); they become the graph g_redo."""
        self.static = TrajectoryBatch(*[t.clone() for t in batch])
        self.side = side
        defer = defer or (lambda: contextlib.nullcontext([]))
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up outside the capture (allocator, autograd)
            for _ in range(2):
                with defer() as fns:
                    bwd_fn(fwd_fn(self.static))
                for f in fns:
                    f()
        torch.cuda.current_stream().wait_stream(side)
        self.g_fwd, self.g_bwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fwd, capture_error_mode=_CAPTURE_MODE):
            self.fwd = fwd_fn(self.static)
        with torch.cuda.graph(self.g_bwd, capture_error_mode=_CAPTURE_MODE):
            with defer() as self.redo_fns:
                self.out = bwd_fn(self.fwd)
            if not GUARD_DEFER_JOIN:  # the fallbacks at the chain's end, in the same graph
                for f in self.redo_fns:
                    f()
        self.g_redo = _capture_redo(self.redo_fns) if GUARD_DEFER_JOIN else None

    def launch_forward(self, batch: TrajectoryBatch):
        """On the side stream, after the work queued so far on the current stream."""
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            for dst, src in zip(self.static, batch):
                if dst.data_ptr() != src.data_ptr():  # drawn in place by prefetch_samples: no copy
                    dst.copy_(src)
            self.g_fwd.replay()

    def grads(self):
        """The gradients (valid once redo() has run after them)."""
        torch.cuda.current_stream().wait_stream(self.side)
        self.g_bwd.replay()
        return list(self.out)

    def redo(self):
        """The backward's deferred guard fallbacks, on the current stream (DPAC_GUARD_DEFER=join;
        otherwise they ended the backward graph)."""
        if self.g_redo is not None:
            self.g_redo.replay()


class _SplitCriticGraphs:
    """The critic step as three HIP graphs, split at the G network's output: the head
    (rollout, G forward with saves, TD assembly, V forward, the loss's gradient at V's
    output and at G's TD1 dots), V's backward (its parameter gradients), and the G
    network's backward (input-gradient chain + parameter gradients).  The G backward reads
    only the head's outputs, so it is launched on a side stream as soon as the head is done:
    it runs beside V's backward, V's Adam step and the actor's terminal V(x_N) (a chain of
    small kernels that leaves most CUs idle) and then beside the actor's BPTT, which needs
    the updated V only (solver.py:221), not G."""

    def __init__(self, head_fn, v_fn, back_fn, batch: TrajectoryBatch, side, defer=None):
        """defer: as _SplitActorGraphs's, for the G backward (graph g_redo)."""
        self.static = TrajectoryBatch(*[t.clone() for t in batch])
        self.side = side
        defer = defer or (lambda: contextlib.nullcontext([]))
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up outside the capture (allocator, autograd)
            for _ in range(2):
                h = head_fn(self.static)
                v_fn(h[0])
                with defer() as fns:
                    back_fn((None,) + tuple(h[1]))
                for f in fns:
                    f()
        torch.cuda.current_stream().wait_stream(side)
        self.g_head, self.g_v, self.g_back = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_head, capture_error_mode=_CAPTURE_MODE):
            self.head_out = head_fn(self.static)
        with torch.cuda.graph(self.g_v, capture_error_mode=_CAPTURE_MODE):
            self.v_out = v_fn(self.head_out[0])
        with torch.cuda.graph(self.g_back, capture_error_mode=_CAPTURE_MODE):
            with defer() as self.redo_fns:
                self.back_out = back_fn((None,) + tuple(self.head_out[1]))
            if not GUARD_DEFER_JOIN:  # the fallbacks at the chain's end, on the side stream
                for f in self.redo_fns:
                    f()
        self.g_redo = _capture_redo(self.redo_fns) if GUARD_DEFER_JOIN else None

    def head(self, batch: TrajectoryBatch):
        """The head graph on the current stream."""
        for dst, src in zip(self.static, batch):
            if dst.data_ptr() != src.data_ptr():  # drawn in place by prefetch_samples: no copy
                dst.copy_(src)
        self.g_head.replay()

    def grads_v(self):
        """V's parameter gradients (current stream, after head())."""
        self.g_v.replay()
        return list(self.v_out)

    def launch_back(self, after: torch.cuda.Event):
        """G's parameter gradients, replayed on the side stream once `after` (recorded
        behind head()) has passed; use them on the side stream (valid once redo() has run)."""
        self.side.wait_event(after)
        with torch.cuda.stream(self.side):
            self.g_back.replay()
        return list(self.back_out)

    def redo(self):
        """The G backward's deferred guard fallbacks, on the current stream after it has waited
        for the side stream (DPAC_GUARD_DEFER=join; otherwise they ended the backward graph)."""
        if self.g_redo is not None:
            self.g_redo.replay()


# DPAC_GRAPH_SETS=2: train_iteration alternates two sets of the split graphs and prefetch_samples
# draws the next iteration's samples into the idle set's static inputs (no copies in front of the
# graphs; round 5); 1: one set, the samples copied in (round 4's path).  "auto" (default, round 6):
# two sets while a rank's batch is at most GRAPH_SETS_MAX_ROWS trajectories, one above it — a set
# holds its own graph pools (the G network's saves over N x B rows, the actor's rollout saves), so
# the second set costs 18 GB at lqr_var_d20's 16 384 trajectories on one GPU (45.4 vs 27.5 GB peak)
# for 0.4 % of the iteration (22.06 vs 22.16 ms), while at 2 048 the copies it saves are a visible
# part of a 3 ms iteration (profiles/r06_call5_pg_early_and_graph_sets.txt).  Both give bitwise the
# same parameters (tests/test_gpu_training.py).
_GS_ENV = os.environ.get("DPAC_GRAPH_SETS", "auto")
GRAPH_SETS = _GS_ENV if _GS_ENV == "auto" else int(_GS_ENV)
if GRAPH_SETS not in ("auto", 1, 2):
    raise ValueError(f"DPAC_GRAPH_SETS must be auto, 1 or 2, got {_GS_ENV!r}")
GRAPH_SETS_MAX_ROWS = 8192


def graph_sets(rows: int) -> int:
    """The graph sets train_iteration alternates for a rank batch of `rows` trajectories."""
    if GRAPH_SETS == "auto":
        return 2 if rows <= GRAPH_SETS_MAX_ROWS else 1
    return GRAPH_SETS

# DPAC_GUARD_DEFER=1 (default): the split graphs' backward chains (the actor's BPTT and its
# parameter gradients, G's row backward and parameter gradients) launch their range-guard
# fallbacks not behind each split-fp16 launch but at the end of the chain, in the chain's own
# graph on its own stream (ops.deferred_fallbacks, dpac.h guard_phase; round 6).  Each chain's
# fallbacks follow every split-fp16 launch of that chain, so whichever launch sets the device's
# sticky status word — this chain's or the other's — the chain is recomputed in exact f32 before
# its gradients are read.  "join": one redo graph after the two chains have joined (round 6's
# first form: on the critical path, ~60 us of no-op launches and graph gaps per iteration);
# 0: inline, behind each launch (rounds 4-5).
_GD_ENV = os.environ.get("DPAC_GUARD_DEFER", "1")
GUARD_DEFER = _GD_ENV != "0"
GUARD_DEFER_JOIN = _GD_ENV == "join"

# DPAC_SAMPLE_STREAM: "gside" (default, round 6: prefetch_samples draws on the G backward's side
# stream, behind G's chain; 2.900 vs 2.906 ms per lqr_d20 iteration at B = 2048, and the
# iteration then holds three of the box's four hardware queues, leaving one to RCCL's stream at
# N > 1) or "own" (a stream of its own, rounds 4-5)
SAMPLE_STREAM = os.environ.get("DPAC_SAMPLE_STREAM", "gside")

# DPAC_GBACK=late (default): the critic's G backward is launched on its side stream after V's
# update and the actor's BPTT are queued, so it runs beside the BPTT and the actor's
# parameter gradients; "early": right after the critic head, beside V's backward, V's Adam
# step and the actor's terminal V(x_N) too.  Both measure the same and give
# bitwise the same parameters (tests/test_gpu_training.py).
GBACK = os.environ.get("DPAC_GBACK", "late")
if GBACK not in ("early", "late"):
    raise ValueError(f"DPAC_GBACK must be 'early' or 'late', got {GBACK!r}")


def _huber_grad(delta):
    """d/d delta of the per-sample Huber term of solver.py:76-77."""
    return torch.where(torch.abs(delta) < DELTA_CLIP, 2 * delta, (2 * DELTA_CLIP) * torch.sign(delta))


def _huber_mean(delta):
    """solver.py:76-77 (quadratic inside |delta| < 50, linear outside)."""
    a = torch.abs(delta)
    return torch.mean(torch.where(a < DELTA_CLIP, torch.square(delta), 2 * DELTA_CLIP * a - DELTA_CLIP ** 2))


# ---------------------------------------------------------------------------
# Solver
# ---------------------------------------------------------------------------
class ActorCriticSolver(object):
    """solver.py:7-136.

    Extra keyword arguments (all optional; defaults reproduce the reference):
      seed     -- seeds the weight initialisers and the device sampler (the
                  reference is unseeded); with data parallelism
                  rank 0's seed is used on every rank, drawn or given;
      sampler  -- "device" (rocRAND Philox on the GPU, default) or "host" (the
                  reference's numpy/scipy stream on numpy's global RandomState,
                  bit-identical inputs: seed it with np.random.seed, as the
                  reference would be);
      parallel -- a parallel.DataParallel for multi-GPU data parallelism;
      graphs   -- capture each training step's gradient evaluation as a HIP graph
                  (default: on with the device sampler; results are identical).
    """

    def __init__(self, config, bsde, seed=None, sampler=None, parallel=None, device=None,
                 graphs=None):
        self.eqn_config = config.eqn_config
        self.net_config = config.net_config
        self.train_config = config.train_config
        self.bsde = bsde
        set_floatx(self.net_config.dtype)
        self.dtype = torch_dtype(self.net_config.dtype)
        if not torch.cuda.is_available():
            raise _lib.DpacUnavailable("ActorCriticSolver needs a ROCm GPU (libdpac has no CPU path)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        _lib.load()
        _lib.ensure_dim(bsde.params())  # a dimension outside the main build: its plugin, built on demand
        self.par = parallel or SingleProcess()
        # one seed for every rank: the Philox stream is keyed by global trajectory index,
        # so the shards of a batch are its rows whatever the world size
        self.seed = self.par.broadcast_int(seed if seed is not None else np.random.randint(0, 2 ** 31 - 1),
                                          device=self.device)
        self.sampler = sampler or self.train_config.get("sampler", "device")
        if self.sampler not in ("device", "host"):
            raise ValueError("sampler must be 'device' or 'host'")
        gen = torch.Generator().manual_seed(self.seed)
        self.model_critic = CriticModel(config, bsde, gen, self.dtype, self.device)
        self.model_actor = ActorModel(config, bsde, gen, self.dtype, self.device)
        self.par.broadcast_(self.critic_variables() + self.actor_variables())
        nc = self.net_config
        self.optimizer_critic = TFAdam(PiecewiseConstantDecay(nc.lr_boundaries_critic, nc.lr_values_critic),
                                       epsilon=1e-8)
        self.optimizer_actor = TFAdam(PiecewiseConstantDecay(nc.lr_boundaries_actor, nc.lr_values_actor),
                                      epsilon=1e-8)
        self.x = None
        self.gamma = self.eqn_config.discount
        st = self.train_config.sample_type
        if st not in ("normal", "bounded"):
            raise ValueError(f"sample_type must be 'normal' or 'bounded', got {st!r}")
        self.sample_type = st
        if self.train_config.train == "actor-critic":
            self.cheat_value_in_actor = False
            self.cheat_control_in_critic = False
        elif self.train_config.train == "critic":
            self.cheat_control_in_critic = True
            self.cheat_value_in_actor = False
        elif self.train_config.train == "actor":
            self.cheat_value_in_actor = True
            self.cheat_control_in_critic = False
        else:
            raise ValueError(f"unknown train mode {self.train_config.train!r}")
        self._calls = 0
        self._next_samples = None  # (spec, critic batch, actor batch, ready event)
        self._sample_side = None
        self.hip_graphs = (self.sampler == "device") if graphs is None else bool(graphs)
        self._graphs = {}
        self._side = None
        self._side_g = None
        # the split actor / critic graphs, two sets per shape used alternately (round 5): the
        # next iteration's samples are drawn straight into the idle set's static inputs
        self._gsets = {}          # (B, N_critic, N_actor) -> [(actor graphs, critic graphs)] * 2
        self._parity = 0          # the set the next train_iteration uses
        self._set_done = [None, None]  # event after the last iteration that used each set
        self._consts = {}  # constant operands of the graphs (never written)
        self._redo_sink = None  # a list while a split graph's capture collects deferred fallbacks

    @contextlib.contextmanager
    def _deferring(self):
        """Collect the guarded backward chains' deferred fallbacks (ops.deferred_fallbacks) of
        the enclosed actor_grads_from / critic_G_back calls: yields the list."""
        prev, self._redo_sink = self._redo_sink, []
        try:
            yield self._redo_sink
        finally:
            self._redo_sink = prev

    def _defer(self):
        return self._deferring if GUARD_DEFER else None

    # ---- variables ---------------------------------------------------------
    def critic_variables(self):
        return self.model_critic.NN_value.trainable_variables() + self.model_critic.NN_value_grad.trainable_variables()

    def actor_variables(self):
        return self.model_actor.NN_control.trainable_variables()

    # ---- sampling (this rank's shard of every batch) -------------------------
    def sample(self, num_sample, N, kind=None, out=None):
        """This rank's shard of a fresh batch; out (device sampler only): a TrajectoryBatch to
        draw into (the same numbers)."""
        kind = kind or self.sample_type
        off, cnt = self.par.shard(num_sample)
        if self.sampler == "host":
            fn = {"normal": self.bsde.sample_normal, "bounded": self.bsde.sample_bounded,
                  "zero": self.bsde.sample0}[kind]
            x0, dw, xb = fn(num_sample, N)
            return Equation.to_native((x0[off:off + cnt], dw[off:off + cnt], xb[off:off + cnt]), self.dtype)
        self._calls += 1
        key = (self.seed * 0x9E3779B1 + self._calls) & 0xFFFFFFFFFFFFFFFF
        if out is None:
            return self.bsde.sample_device(kind, cnt, N, key, off, self.dtype)
        return self.bsde.sample_device(kind, cnt, N, key, off, self.dtype, out=out)

    def sample_iteration(self, num_sample, N_critic, N_actor):
        """The (critic, actor) samples of one training iteration (solver.py:67-70): the pair
        prefetch_samples() drew on a side stream if it matches, else drawn now.

        With two graph sets (graph_sets) the prefetched pair IS the static input of a set:
        the next prefetch_samples() into that set (two iterations later) overwrites it in
        place.  A caller that keeps a batch beyond its train_iteration must clone it."""
        spec = (num_sample, N_critic, N_actor)
        nxt, self._next_samples = self._next_samples, None
        if nxt is None or nxt[0] != spec:
            return self.sample(num_sample, N_critic), self.sample(num_sample, N_actor)
        _, dc, da, ready = nxt
        cur = torch.cuda.current_stream()
        cur.wait_event(ready)
        for t in (*dc, *da):  # made on the side stream, used on this one
            t.record_stream(cur)
        return dc, da

    def prefetch_samples(self, num_sample, N_critic, N_actor):
        """Draw the next iteration's (critic, actor) pair on a side stream (device sampler;
        the samples do not depend on the parameters), after the current iteration's work is
        queued, so sampling leaves the critical path.  As long as no other sample() call
        comes before the next sample_iteration() the Philox keys are those of drawing in
        place."""
        if self.sampler != "device":
            return
        if self._sample_side is None:
            # SAMPLE_STREAM "gside": the G backward's side stream (once it exists), so a training
            # iteration uses three streams of its own and a fourth hardware queue stays free for
            # RCCL's stream at N > 1 (the box runs 4 queues per process)
            if SAMPLE_STREAM == "gside" and self._side_g is not None:
                self._sample_side = self._side_g
            else:
                self._sample_side = torch.cuda.Stream()
        # the next iteration's graph set (train_iteration alternates two): its static inputs are
        # drawn into in place, once the iteration that last read them is done, so the next
        # iteration copies nothing in (round 5); otherwise fresh buffers
        two = graph_sets(self.par.shard(num_sample)[1]) == 2
        gset = self._gsets.get((num_sample, N_critic, N_actor)) if two else None
        gset = gset[self._parity] if gset else None
        with torch.cuda.stream(self._sample_side):
            if gset is not None:
                sg, cg = gset
                if self._set_done[self._parity] is not None:
                    torch.cuda.current_stream().wait_event(self._set_done[self._parity])
                dc = self.sample(num_sample, N_critic, out=cg.static)
                da = self.sample(num_sample, N_actor, out=sg.static)
            else:  # fresh buffers: nothing to wait for
                dc, da = self.sample(num_sample, N_critic), self.sample(num_sample, N_actor)
            ready = torch.cuda.Event()
            ready.record()
        self._next_samples = ((num_sample, N_critic, N_actor), dc, da, ready)

    # ---- losses ------------------------------------------------------------
    def loss_critic(self, inputs, training, cheat_control):
        delta, delta_bdry = self.model_critic(inputs, self.model_actor, training, cheat_control)
        return (_huber_mean(delta) + _huber_mean(delta_bdry)) * 100  # solver.py:73-78

    def loss_actor(self, inputs, training, cheat_value, cheat_control):
        y = self.model_actor(inputs, self.model_critic, training, cheat_value, cheat_control)
        return torch.mean(y)  # solver.py:80-83

    def grad_critic(self, inputs, training, cheat_control):
        vs = self.critic_variables()
        loss = self.loss_critic(inputs, training, cheat_control)
        return list(torch.autograd.grad(loss, vs, allow_unused=True))

    def grad_actor(self, inputs, training, cheat_value, cheat_control):
        vs = self.actor_variables()
        loss = self.loss_actor(inputs, training, cheat_value, cheat_control)
        return list(torch.autograd.grad(loss, vs, allow_unused=True))

    def _global(self, data, total):
        return data.x0.shape[0], total

    def _grads(self, kind, fn, data):
        """fn(batch) -> gradients, through a captured HIP graph when enabled."""
        data = Equation.to_native(data, self.dtype)
        if not self.hip_graphs:
            return fn(data)
        key = (kind, tuple(data.dw.shape))
        graph = self._graphs.get(key)
        if graph is None:
            graph = self._graphs[key] = _GradGraph(fn, data)
        return graph(data)

    def train_step_critic(self, train_data, total=None):
        g = self._grads("critic", lambda d: self.grad_critic(
            d, training=False, cheat_control=self.cheat_control_in_critic), train_data)
        cnt = train_data[0].shape[0]
        g = self.par.allreduce_grads(g, cnt, total or cnt * self.par.world)
        self.optimizer_critic.apply_gradients(zip(g, self.critic_variables()))

    # ---- the actor step split around the critic step (overlap) ---------------
    def _actor_split_ok(self):
        return (self.hip_graphs and self.train_config.train == "actor-critic"
                and self.model_actor.NN_control.fused_ok() and ops.BPTT_MODE == "fused")

    def actor_forward(self, data):
        """The actor's rollout with saves (solver.py:207-219 forward), no autograd."""
        ma, ec = self.model_actor, self.eqn_config
        d = Equation.to_native(data, self.dtype)
        return ops.actor_rollout_saves(self.bsde.params(), ma.scheme, d.x0, d.dw, ec.total_time_actor,
                                       ec.num_time_interval_actor, ma.NN_control)

    def actor_grads_from(self, fwd):
        """grad_actor from actor_forward's outputs: loss = mean(y + V(x_N)*disc_N)
        (solver.py:80-83, 220-223) differentiated by hand at (y, disc_N, x_N), then the
        BPTT kernels; V's parameters are constants (the tape watches the actor)."""
        y, disc, xN, saved = fwd
        B = y.shape[0]
        eqp = self.bsde.params()
        if self.cheat_value_in_actor:
            term = ops.equation_eval(eqp, _lib.EVAL_V_TRUE, xN)
            gV = ops.equation_eval(eqp, _lib.EVAL_V_GRAD, xN)
        elif ops.ROW_MLP == "kernel" and self.model_critic.NN_value.fused_ok():
            # V(x_N) and dV/dx_N (V's parameters are constants here): the row kernels
            Vnet = self.model_critic.NN_value
            with torch.no_grad():
                xN = xN.contiguous()
                prep = Vnet.mlp_prepared()  # forward and backward images, one launch
                v, zV = ops.mlp_rows(prep[0], xN, save=True)
                gV, _ = ops.row_mlp_backward(Vnet.bn_rs, [p.detach() for p in Vnet.trainable_variables()],
                                             xN, zV, torch.ones_like(v), True, False, prepared=prep)
            term = v[:, 0]
        else:
            xl = xN.detach().requires_grad_(True)
            with torch.enable_grad():
                v = self.model_critic.NN_value(xl, False, const_params=True)[:, 0]
                gV, = torch.autograd.grad(v.sum(), xl)
            term = v.detach()
        key = ("g_y", B, y.dtype, y.device)
        g_y = self._consts.get(key)
        if g_y is None:  # made in the warm-up before a graph capture: the graph reads it, no fill kernel
            g_y = self._consts[key] = torch.full_like(y, 1.0 / B)
        g_disc = term / B
        g_xN = gV * (disc / B).unsqueeze(1)
        net = self.model_actor.NN_control
        ec = self.eqn_config
        with ops.deferred_fallbacks(self._redo_sink):  # the BPTT -> parameter gradients chain
            return ops.actor_bptt_grads(eqp, self.model_actor.scheme, ec.total_time_actor,
                                        ec.num_time_interval_actor, net.ekn_head, net.bn_rs,
                                        net.trainable_variables(), saved, g_y, g_disc, g_xN)

    # ---- the critic step split at the G network (its backward beside the BPTT) ----
    def _critic_split_ok(self):
        mc = self.model_critic
        return (self._actor_split_ok() and mc.td == _lib.TD1 and ops.ROW_MLP == "kernel"
                and mc.NN_value_grad.fused_ok() and not mc.NN_value_grad.ekn_head)

    def critic_front(self, data):
        """grad_critic split at the G network, without autograd (critic_head + critic_grads_v).
        Returns (gradients of V's variables, then the G backward's inputs: dL/d(TD1 dot)
        [N*B] (fused) or dL/dG [N*B, d], G's input rows, G's saves[, u rows, dw rows])."""
        vstate, back = self.critic_head(data)
        return (self.critic_grads_v(vstate), *back)

    def critic_head(self, data):
        """The rollout, G = NN_value_grad(x_t) over the N*B rows with saves (solver.py:179),
        the TD1 target (solver.py:166-187), V at (x_0, x_N, x_bdry) with saves, then the loss
        100*(mean h(delta) + mean h(delta_bdry)) (solver.py:73-78, 189-190) differentiated by
        hand at V's output and at G: h'(z) = 2z inside |z| < 50, 100 sign(z) outside;
        dL/dV(x_0) = g, dL/dV(x_N) = -g*disc, dL/dy = -g, dL/dV(x_bdry) = g_bdry.
        Returns ((V's rows, V's saves, dL/dV, V's prepared images), the G backward's inputs)."""
        mc, ec = self.model_critic, self.eqn_config
        d = Equation.to_native(data, self.dtype)
        N, T = ec.num_time_interval_critic, ec.total_time_critic
        B = d.x0.shape[0]
        eqp = self.bsde.params()
        Gnet, Vnet = mc.NN_value_grad, mc.NN_value
        with torch.no_grad():
            x, dt, coef, u = self.bsde.rollout(mc.scheme, d.x0, d.dw, T, N, self.model_actor.NN_control,
                                               cheat=self.cheat_control_in_critic)
            rows = x[:N].reshape(N * B, -1)
            fused = ops.CRITIC_TD1 == "fused"
            if fused:  # G never written, only its TD1 dots
                u_rows, dw_rows = u.reshape(N * B, -1), d.dw.reshape(N * B, -1)
                gdot, zG, *mG = ops.mlp_rows_td1(eqp, Gnet.mlp_view(), rows, u_rows, dw_rows, save=True,
                                                 mask=ops.ROW_MASK)
                mG = mG[0] if mG else None  # the sign-bit mask, or None (DPAC_ROW_MASK=0, float64)
                y, disc = ops.td_assemble_gdot(eqp, x, u, dt, coef, gdot.view(N, B),
                                               cost_order=_lib.COST_CRITIC)
            else:
                G, zG, *mG = ops.mlp_rows(Gnet.mlp_view(), rows, save=True, mask=ops.ROW_MASK)
                mG = mG[0] if mG else None
                y, disc = ops.td_assemble(eqp, mc.td, x, u, d.dw, dt, coef, G.view(N, B, -1),
                                          cost_order=_lib.COST_CRITIC)
            xv = torch.cat([x[0], x[N], d.x_bdry])
            prepV = Vnet.mlp_prepared()  # V's forward and backward images, one launch
            Vout, zV = ops.mlp_rows(prepV[0], xv, save=True)
            # delta = V(x_0) - y - V(x_N) disc, delta_b = V(x_bdry) - Z_tf(x_bdry)
            # (solver.py:189-190) and the Huber gradient, one launch
            g_out, neg_g = ops.critic_loss_grad(Vout, y, disc, self.bsde.Z_tf(d.x_bdry), 100.0 / B, DELTA_CLIP)
            if fused:
                g_gdot = ops.td_assemble_bwd_gdot(eqp, dt, coef, neg_g)
                back = (g_gdot.reshape(N * B), rows, zG, mG, u_rows, dw_rows)
            else:
                gG = ops.td_assemble_bwd(eqp, x, u, d.dw, dt, coef, neg_g)
                back = (gG.reshape(N * B, -1), rows, zG, mG)
        return (xv, zV, g_out, prepV), back

    def critic_grads_v(self, vstate):
        """Gradients of V's variables from critic_head's (rows, saves, dL/dV, V's prepared
        images)."""
        xv, zV, g_out, prepV = vstate
        Vnet = self.model_critic.NN_value
        with torch.no_grad():
            _, gV = ops.row_mlp_backward(Vnet.bn_rs, Vnet.trainable_variables(), xv, zV, g_out,
                                         False, True, prepared=prepV)
        return gV

    def critic_G_back(self, front):
        """G's parameter gradients from critic_front's outputs (dpac_mlp_rows_bwd[_td1] +
        dpac_mlp_param_grads, on their own scratch buffer: they run beside the BPTT)."""
        net = self.model_critic.NN_value_grad
        with torch.no_grad(), ops.deferred_fallbacks(self._redo_sink):  # row backward -> gradients
            if len(front) == 7:  # fused TD1: dL/dG formed from dL/dgdot in the prologue
                _, g_gdot, rows, z, m, u_rows, dw_rows = front
                return ops.row_mlp_backward_td1(self.bsde.params(), net.bn_rs,
                                                net.trainable_variables(), rows, z, u_rows,
                                                dw_rows, g_gdot, True, ws_tag=1, mask=m)
            _, gG, rows, z, m = front
            _, grads = ops.row_mlp_backward(net.bn_rs, net.trainable_variables(), rows, z, gG,
                                            False, True, ws_tag=1, mask=m)
        return grads

    def train_iteration(self, data_critic, data_actor, total=None):
        """One iteration of solver.py:67-70 (critic step, then actor step).  With HIP
        graphs the actor's forward rollout runs on a side stream during the critic step;
        under TD1 the critic's G-network backward runs on a second side stream beside the
        actor's BPTT (which reads V, not G).  Two gradient all-reduces per iteration (SURVEY
        §8(e)): V's half of the critic step (the actor's terminal V(x_N) needs the updated V,
        solver.py:221), then the actor's gradients and G's half in one flattened exchange (G
        is next read by the following iteration's critic step)."""
        if not self._actor_split_ok():
            self.train_step_critic(data_critic, total)
            self.train_step_actor(data_actor, total)
            return
        da = Equation.to_native(data_actor, self.dtype)
        if self._side is None:
            self._side = torch.cuda.Stream()
        if not self._critic_split_ok():
            key = ("actor_split", tuple(da.dw.shape))
            sg = self._graphs.get(key)
            if sg is None:
                sg = self._graphs[key] = _SplitActorGraphs(self.actor_forward, self.actor_grads_from,
                                                           da, self._side, self._defer())
            sg.launch_forward(da)
            self.train_step_critic(data_critic, total)
            cg = None
        else:
            dc = Equation.to_native(data_critic, self.dtype)
            if self._side_g is None:
                self._side_g = torch.cuda.Stream()
            spec = (dc.x0.shape[0] * self.par.world if total is None else total, dc.dw.shape[0], da.dw.shape[0])
            sets = self._gsets.setdefault(spec, [None, None])
            p = self._parity
            if sets[p] is None:
                sets[p] = (_SplitActorGraphs(self.actor_forward, self.actor_grads_from, da, self._side,
                                             self._defer()),
                           _SplitCriticGraphs(self.critic_head, self.critic_grads_v, self.critic_G_back, dc,
                                              self._side_g, self._defer()))
            sg, cg = sets[p]
            sg.launch_forward(da)
            ccnt = dc.x0.shape[0]
            ctot = total or ccnt * self.par.world
            cg.head(dc)
            head_done = torch.cuda.Event()
            head_done.record()
            if GBACK == "early":  # G's backward beside V's update and the actor's terminal V
                gG = cg.launch_back(head_done)
            gV = self.par.allreduce_grads(cg.grads_v(), ccnt, ctot)
            # one Adam step of the critic in two parts: V now (the actor reads it), G after the
            # actor's exchange (same lr and t: advance=False here)
            self.optimizer_critic.apply_gradients(
                zip(gV, self.model_critic.NN_value.trainable_variables()), advance=False)
        g = sg.grads()  # the actor's terminal V(x_N), BPTT and parameter gradients
        cnt = da.x0.shape[0]
        atot = total or cnt * self.par.world
        if cg is None:
            sg.redo()
            g = self.par.allreduce_grads(g, cnt, atot)
            self.optimizer_actor.apply_gradients(zip(g, self.actor_variables()))
            return
        if GBACK != "early":
            gG = cg.launch_back(head_done)
        torch.cuda.current_stream().wait_stream(cg.side)  # G's gradients, made on the side stream
        sg.redo()  # DPAC_GUARD_DEFER=join: both chains' range-guard fallbacks (no-ops unless a split
        cg.redo()  # operand overflowed); by default each chain's graph ends with its own
        g, gG = self.par.allreduce_grads_multi([(g, cnt, atot), (gG, ccnt, ctot)])
        self.optimizer_actor.apply_gradients(zip(g, self.actor_variables()))
        self.optimizer_critic.apply_gradients(zip(gG, self.model_critic.NN_value_grad.trainable_variables()))
        done = torch.cuda.Event()  # every reader of this set's static inputs is behind this point
        done.record()
        self._set_done[self._parity] = done
        self._parity = (self._parity + 1) % graph_sets(ccnt)

    def train_step_actor(self, train_data, total=None):
        g = self._grads("actor", lambda d: self.grad_actor(
            d, training=False, cheat_value=self.cheat_value_in_actor, cheat_control=False), train_data)
        cnt = train_data[0].shape[0]
        g = self.par.allreduce_grads(g, cnt, total or cnt * self.par.world)
        self.optimizer_actor.apply_gradients(zip(g, self.actor_variables()))

    # ---- metrics (solver.py:109-136), reduced over ranks ---------------------
    def _mean(self, local_mean, cnt, total):
        return self.par.sum(local_mean * (cnt / total))

    @torch.no_grad()
    def err_value(self, inputs, total=None):
        x0 = Equation.to_native(inputs, self.dtype).x0
        vt = self.bsde.V_true(x0)
        num = self.par.sum(torch.sum(torch.square(vt - self.model_critic.NN_value(x0))))
        den = self.par.sum(torch.sum(torch.square(vt)))
        return torch.sqrt(num / den)

    @torch.no_grad()
    def err_control(self, inputs, total=None):
        x0 = Equation.to_native(inputs, self.dtype).x0
        ut = self.bsde.u_true(x0)
        num = self.par.sum(torch.sum(torch.square(ut - self.model_actor.NN_control(x0))))
        den = self.par.sum(torch.sum(torch.square(ut)))
        return torch.sqrt(num / den)

    @torch.no_grad()
    def err_value_grad(self, inputs, total=None):
        x0 = Equation.to_native(inputs, self.dtype).x0
        gt = self.bsde.V_grad_true(x0)
        num = self.par.sum(torch.sum(torch.square(gt - self.model_critic.NN_value_grad(x0))))
        den = self.par.sum(torch.sum(torch.square(gt)))
        return torch.sqrt(num / den)

    @torch.no_grad()
    def err_value_infty(self, inputs, total=None):
        x0 = Equation.to_native(inputs, self.dtype).x0
        return self.par.max(torch.max(torch.abs(self.bsde.V_true(x0) - self.model_critic.NN_value(x0))))

    @torch.no_grad()
    def err_cost(self, inputs, total=None):
        data = Equation.to_native(inputs, self.dtype)
        y = self.model_actor(data, self.model_critic, False, False, False)
        y0 = self.model_critic.NN_value(data.x0)
        cnt = data.x0.shape[0]
        return self._mean(torch.mean(y - y0), cnt, total or cnt * self.par.world)

    @torch.no_grad()
    def _valid_loss_critic(self, data, total):
        cnt = data.x0.shape[0]
        delta, delta_bdry = self.model_critic(data, self.model_actor, False, False)
        local = (_huber_mean(delta) + _huber_mean(delta_bdry)) * 100
        return self._mean(local, cnt, total)

    @torch.no_grad()
    def _valid_loss_actor(self, data, total, cheat_value=False, cheat_control=False):
        cnt = data.x0.shape[0]
        local = self.loss_actor(data, False, cheat_value, cheat_control)
        return self._mean(local, cnt, total)

    # ---- training loop (solver.py:36-71) -------------------------------------
    def train(self):
        start_time = time.time()
        training_history = []
        nc, ec = self.net_config, self.eqn_config
        V = nc.valid_size
        valid_data_critic = self.sample(V, ec.num_time_interval_critic)
        valid_data_actor = self.sample(V, ec.num_time_interval_actor)
        valid_data_cost = self.sample(V, ec.num_time_interval_actor, kind="zero")
        true_loss_actor = float(self._valid_loss_actor(valid_data_actor, V, True, True))
        x0 = y = true_y = z = true_z = grad_y = None
        for step in range(nc.num_iterations + 1):
            if step % nc.logging_frequency == 0:
                loss_critic = float(self._valid_loss_critic(valid_data_critic, V))
                loss_actor = float(self._valid_loss_actor(valid_data_actor, V))
                err_value = float(self.err_value(valid_data_critic))
                err_control = float(self.err_control(valid_data_actor))
                err_value_grad = float(self.err_value_grad(valid_data_critic))
                err_value_infty = float(self.err_value_infty(valid_data_critic))
                err_cost = float(self.err_cost(valid_data_cost, V))
                elapsed_time = time.time() - start_time
                training_history.append([step, loss_critic, loss_actor, err_value, err_value_infty,
                                         err_control, err_value_grad, err_cost, elapsed_time])
                if nc.verbose and self.par.rank == 0:
                    logging.info(
                        "step: %5u, loss_critic: %.4e, loss_actor: %.4e, err_value: %.4e, "
                        "err_value_infty: %.4e, err_control: %.4e, err_value_grad: %.4e, "
                        "err_cost: %.4e, elapsed time: %3u" % (
                            step, loss_critic, loss_actor, err_value, err_value_infty, err_control,
                            err_value_grad, err_cost, elapsed_time))
            if step == nc.num_iterations:
                with torch.no_grad():  # solver.py:63-66 on the whole validation set
                    xv = valid_data_critic.x0
                    g = lambda t: self.par.gather_rows(t, V).cpu().numpy()  # global row order
                    x0 = g(xv)
                    y = g(self.model_critic.NN_value(xv))
                    true_y = g(self.bsde.V_true(xv))
                    grad_y = g(self.model_critic.NN_value_grad(xv))
                    z = g(self.model_actor.NN_control(xv))
                    true_z = g(self.bsde.u_true(xv))
                if self.par.rank == 0:
                    print("true loss actor: ", true_loss_actor)
                training_history.append([0, 0.0, true_loss_actor, 0.0, 0.0, 0.0, 0.0, 0.0, elapsed_time])
            if self.train_config.train == "actor-critic":
                # both samples first, in the reference's order (critic, then actor)
                dc, da = self.sample_iteration(nc.batch_size, ec.num_time_interval_critic,
                                               ec.num_time_interval_actor)
                self.train_iteration(dc, da, nc.batch_size)
                self.prefetch_samples(nc.batch_size, ec.num_time_interval_critic,
                                      ec.num_time_interval_actor)
            elif self.train_config.train == "critic":
                self.train_step_critic(self.sample(nc.batch_size, ec.num_time_interval_critic), nc.batch_size)
            else:
                self.train_step_actor(self.sample(nc.batch_size, ec.num_time_interval_actor), nc.batch_size)
        return np.array(training_history), x0, y, true_y, z, true_z, grad_y
