"""Config loading and global numeric settings.

Replaces the reference's `munch.munchify` attribute access (main.py:31-33) and
`tf.keras.backend.set_floatx` (main.py:35).  The JSON schema is the reference's
(`configs/*.json`: eqn_config / net_config / train_config) and is accepted
verbatim; optional keys this build adds are listed in DESIGN.md §6.
"""
from __future__ import annotations

import json

import torch


class AttrDict(dict):
    """dict with attribute access, recursively (a stand-in for munch.Munch)."""

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def __setattr__(self, name, value):
        self[name] = value

    def __delattr__(self, name):
        try:
            del self[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def __dir__(self):  # like Munch: the keys (main.py:47-48 dumps dir(config))
        return list(self.keys())

    def get_opt(self, name, default=None):
        return self.get(name, default)


def munchify(obj):
    if isinstance(obj, dict):
        return AttrDict({k: munchify(v) for k, v in obj.items()})
    if isinstance(obj, (list, tuple)):
        return type(obj)(munchify(v) for v in obj)
    return obj


def unmunchify(obj):
    if isinstance(obj, dict):
        return {k: unmunchify(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [unmunchify(v) for v in obj]
    return obj


def load_config(path: str) -> AttrDict:
    with open(path) as f:
        return munchify(json.load(f))


# eqn_config of the reference's BASELINE configs (configs/*.json values restated)
BASELINE_EQN_CONFIGS = {
    "lqr_d20": {"_comment": "linear quadratic regulator", "eqn_name": "LQR", "dim": 20, "control_dim": 20,
                "discount": 1.0, "p": 1.0, "q": 1.0, "beta": 1.0, "R": 1.0},
    "ekn_d20": {"_comment": "Diffusive Eikonal equation", "eqn_name": "EKN", "dim": 20, "control_dim": 20,
                "discount": 0, "a2": 1.2, "a3": 0.2, "R": 1.0},
    "lqr_var_d20": {"_comment": "linear quadratic regulator", "eqn_name": "LQR_var", "dim": 20,
                    "control_dim": 20, "discount": 1.0, "q": 1.0, "beta": 1.0, "epsilon": 0.01, "R": 1.0},
    "vdp_d20": {"_comment": "Van Der Pol oscillator", "eqn_name": "VDP", "dim": 20, "control_dim": 10,
                "discount": 1.0, "a": 1.0, "epsilon": 0.1, "q": 1.0, "R": 1.0},
}


def baseline_config(iters, log_freq, dtype, batch, valid, name="lqr_d20"):
    """A full config of one BASELINE case (T = 0.2, N = 100, 3x200 MLPs, adaptive, TD1,
    normal sampling, actor-critic: the reference's configs/*_d20.json), with the
    iteration count, logging frequency, dtype and batch sizes given."""
    eqn = dict(BASELINE_EQN_CONFIGS[name], total_time_critic=0.2, total_time_actor=0.2,
               num_time_interval_critic=100, num_time_interval_actor=100)
    return munchify({
        "eqn_config": eqn,
        "net_config": {"num_hiddens_critic": [200, 200, 200], "num_hiddens_actor": [200, 200, 200],
                       "lr_values_critic": [1e-3, 1e-4, 1e-5], "lr_boundaries_critic": [30000, 40000],
                       "lr_values_actor": [1e-3, 1e-4, 1e-5], "lr_boundaries_actor": [30000, 40000],
                       "num_iterations": iters, "batch_size": batch, "valid_size": valid,
                       "logging_frequency": log_freq, "dtype": dtype, "verbose": False},
        "train_config": {"sample_type": "normal", "scheme": "adaptive", "TD_type": "TD1",
                         "train": "actor-critic"},
    })


_FLOATX = {"float32": torch.float32, "float64": torch.float64}
_state = {"floatx": "float32"}


def set_floatx(name: str) -> None:
    """Global compute dtype, as tf.keras.backend.set_floatx (main.py:35)."""
    if name not in _FLOATX:
        raise ValueError(f"unsupported dtype {name!r}; expected one of {sorted(_FLOATX)}")
    _state["floatx"] = name


def floatx() -> str:
    return _state["floatx"]


def torch_dtype(name: str | None = None) -> torch.dtype:
    return _FLOATX[name or _state["floatx"]]
