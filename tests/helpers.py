"""Shared test helpers: reference-schema configs for every equation family."""
from __future__ import annotations

import numpy as np

from deeppde_actorcritic_amd.config import munchify

EQN_COEFFS = {  # per-equation eqn_config keys, values of the shipped configs
    "LQR": {"p": 1.0, "q": 1.0, "beta": 1.0},                 # configs/lqr_d20.json:12-14
    "VDP": {"a": 1.0, "epsilon": 0.1, "q": 1.0},              # configs/vdp_d20.json:12-14
    "EKN": {"a2": 1.2, "a3": 0.2},                            # configs/ekn_d20.json:12-13
    "ekn": {"a2": 1.2, "a3": 0.2},
    "LQR_var": {"q": 1.0, "beta": 1.0, "epsilon": 0.01},      # configs/lqr_var_d20.json:12-14
}


# the reference's configs/lqr_d5.json, restated verbatim (the reference tree does not travel to
# the GPU box): BASELINE configs[0] is this file with TD2, the naive scheme and batch 256
SHIPPED_LQR_D5 = {
    "eqn_config": {"_comment": "linear quadratic regulator", "eqn_name": "LQR",
                   "total_time_critic": 0.2, "total_time_actor": 0.2, "dim": 5, "control_dim": 5,
                   "num_time_interval_critic": 50, "num_time_interval_actor": 50, "discount": 1.0,
                   "p": 1.0, "q": 1.0, "beta": 1.0, "R": 1.0},
    "net_config": {"num_hiddens_critic": [200, 200], "num_hiddens_actor": [200, 200],
                   "lr_values_critic": [1e-3, 1e-4, 1e-5], "lr_boundaries_critic": [20000, 30000],
                   "lr_values_actor": [1e-3, 1e-4, 1e-5], "lr_boundaries_actor": [20000, 30000],
                   "num_iterations": 40000, "batch_size": 1024, "valid_size": 1024,
                   "logging_frequency": 100, "dtype": "float64", "verbose": True},
    "train_config": {"sample_type": "normal", "scheme": "adaptive", "TD_type": "TD1",
                     "train": "actor-critic"},
}


def eqn_config(name, dim, control_dim=None, T=0.2, N=10, discount=None, R=1.0):
    if control_dim is None:
        control_dim = dim // 2 if name == "VDP" else dim
    if discount is None:
        discount = 0.0 if name in ("EKN", "ekn") else 1.0
    cfg = {"_comment": "test", "eqn_name": name, "total_time_critic": T, "total_time_actor": T,
           "dim": dim, "control_dim": control_dim, "num_time_interval_critic": N,
           "num_time_interval_actor": N, "discount": discount, "R": R}
    cfg.update(EQN_COEFFS[name])
    return munchify(cfg)


def full_config(name, dim, control_dim=None, T=0.2, N=10, hidden=(16, 16), batch=32, valid=32,
                iters=2, scheme="adaptive", td="TD1", train="actor-critic", sample="normal",
                dtype="float64", log_freq=1):
    return munchify({
        "eqn_config": dict(eqn_config(name, dim, control_dim, T, N)),
        "net_config": {"num_hiddens_critic": list(hidden), "num_hiddens_actor": list(hidden),
                       "lr_values_critic": [1e-3, 1e-4, 1e-5], "lr_boundaries_critic": [30000, 40000],
                       "lr_values_actor": [1e-3, 1e-4, 1e-5], "lr_boundaries_actor": [30000, 40000],
                       "num_iterations": iters, "batch_size": batch, "valid_size": valid,
                       "logging_frequency": log_freq, "dtype": dtype, "verbose": False},
        "train_config": {"sample_type": sample, "scheme": scheme, "TD_type": td, "train": train},
    })


def rel_close(a, b, rtol):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.max(np.abs(a - b) / (1.0 + np.abs(b))) <= rtol
