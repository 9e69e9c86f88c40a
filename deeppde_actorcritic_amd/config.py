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
