"""Generate the committed golden fixtures under tests/golden/.

Run in the development container (needs /root/reference, read-only):

    python tests/golden/make_golden.py

1. sampler_*.npz — outputs of the REFERENCE's own sampler methods
   (equation.py:7-44: Equation.__init__, sample_normal, sample_bounded, sample0),
   executed here with their real dependencies (numpy, scipy.stats).  The methods
   are taken from /root/reference/equation.py by AST and run unchanged; the rest
   of that file needs TensorFlow, which is not installed, and is not executed.
   Nothing of the reference is stored: only seeds, sizes and the arrays it drew.
2. rollout_*.npz — oracle (oracle/equations.py) outputs for small cheat-control
   rollouts of every equation x scheme, plus the critic/actor cost loops; used as
   regression vectors for the oracle and as fixed inputs/outputs for GPU parity.
"""
from __future__ import annotations

import ast
import os
import sys

import numpy as np
import scipy.stats
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = os.environ.get("DPAC_REFERENCE", "/root/reference")

from oracle import equations as oeq  # noqa: E402
from tests.helpers import eqn_config  # noqa: E402

SAMPLER_CASES = [  # (seed, dim, R, num_sample, N)
    (1234, 4, 1.0, 6, 3),
    (7, 5, 1.0, 5, 4),
    (2024, 20, 1.0, 3, 2),
    (99, 10, 2.0, 4, 3),
]


def reference_sampler_class():
    """The reference's Equation class restricted to its numpy/scipy-only methods."""
    path = os.path.join(REF, "equation.py")
    tree = ast.parse(open(path).read(), filename=path)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Equation")
    keep = {"__init__", "sample_normal", "sample_bounded", "sample0", "b_np"}
    body = [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name in keep]
    mod = ast.Module(body=[ast.ClassDef(name="Equation", bases=[], keywords=[], body=body,
                                        decorator_list=[])], type_ignores=[])
    ns = {"np": np, "normal": scipy.stats.multivariate_normal, "object": object}
    exec(compile(ast.fix_missing_locations(mod), path, "exec"), ns)
    return ns["Equation"]


class _Cfg(dict):
    __getattr__ = dict.__getitem__


def make_sampler_fixtures():
    Ref = reference_sampler_class()
    for seed, dim, R, B, N in SAMPLER_CASES:
        eq = Ref(_Cfg(dim=dim, discount=1.0, R=R, control_dim=dim))
        out = {"seed": seed, "dim": dim, "R": R, "num_sample": B, "N": N}
        for name in ("sample_normal", "sample_bounded", "sample0"):
            np.random.seed(seed)
            x0, dw, xb = getattr(eq, name)(B, N)
            out[f"{name}_x0"], out[f"{name}_dw"], out[f"{name}_x_bdry"] = x0, dw, xb
        # two successive calls (the training loop's RNG sequence: critic then actor batch)
        np.random.seed(seed)
        a = eq.sample_normal(B, N)
        b = eq.sample_normal(B, N)
        out["seq_x0_1"], out["seq_dw_2"] = a[0], b[1]
        np.savez(os.path.join(HERE, f"sampler_d{dim}_s{seed}.npz"), **out)


ROLLOUT_CASES = [  # (eqn, dim, control_dim, scheme, sample_type)
    ("LQR", 5, 5, "naive", "normal"),
    ("LQR", 5, 5, "adaptive", "normal"),
    ("LQR", 20, 20, "adaptive", "bounded"),
    ("VDP", 4, 2, "naive", "normal"),
    ("VDP", 4, 2, "adaptive", "normal"),
    ("EKN", 5, 5, "adaptive", "normal"),
    ("EKN", 5, 5, "naive", "bounded"),
    ("LQR_var", 5, 5, "adaptive", "normal"),
    ("LQR_var", 20, 20, "naive", "normal"),
]


def make_rollout_fixtures(B=8, N=6, T=0.2):
    for i, (name, d, c, scheme, st) in enumerate(ROLLOUT_CASES):
        cfg = eqn_config(name, d, c, T=T, N=N)
        eq = oeq.make(cfg)
        np.random.seed(100 + i)
        x0, dw, xb = (eq.sample_normal if st == "normal" else eq.sample_bounded)(B, N)
        prop = eq.propagate_naive if scheme == "naive" else eq.propagate_adaptive
        x, dt, coef = prop(B, x0, dw, None, False, T, N, True)
        # critic-order and actor-order cost loops with the analytic control (solver.py:166-187, 213-219)
        y_c = torch.zeros(B, 1, dtype=torch.float64)
        y_a = torch.zeros(B, 1, dtype=torch.float64)
        disc = torch.ones(B, 1, dtype=torch.float64)
        for t in range(N):
            u = eq.u_true(x[:, :, t])
            w = eq.w_tf(x[:, :, t], u)
            y_c = y_c + (w * disc) * (coef[:, t:t + 1] * dt[:, t:t + 1])
            y_a = y_a + coef[:, t:t + 1] * w * dt[:, t:t + 1] * disc
            disc = disc * torch.exp(-cfg.discount * dt[:, t:t + 1] * coef[:, t:t + 1])
        np.savez(os.path.join(HERE, f"rollout_{i}_{name}_d{d}_{scheme}.npz"),
                 eqn=name, dim=d, control_dim=c, scheme=scheme, T=T, N=N, x0=x0, dw=dw, x_bdry=xb,
                 x=x.numpy(), dt=dt.numpy(), coef=coef.numpy(), y_critic=y_c.numpy()[:, 0],
                 y_actor=y_a.numpy()[:, 0], disc=disc.numpy()[:, 0])


if __name__ == "__main__":
    make_sampler_fixtures()
    make_rollout_fixtures()
    print("fixtures written to", HERE)
