"""ctypes binding of libdpac (include/dpac.h).

The library is built in-tree (``make lib`` or ``__graft_entry__.build()``) and is
loaded from this package directory.  There is no fallback: if the shared object
is missing or fails to load, every device op raises :class:`DpacUnavailable`.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPAC_LIB", os.path.join(_HERE, "libdpac.so"))

# constants mirrored from include/dpac.h
ABI_VERSION = 8  # DPAC_ABI_VERSION: load() refuses a library built from another header
DPAC_OK, DPAC_EINVAL, DPAC_EUNSUP = 0, -1, -2
F32, F64 = 0, 1
EQN_LQR, EQN_VDP, EQN_EKN, EQN_LQR_VAR = 0, 1, 2, 3
SCHEME_NAIVE, SCHEME_ADAPTIVE = 0, 1
TD1, TD2, TD1_GDOT = 1, 2, 3
COST_CRITIC, COST_ACTOR = 0, 1
SAMPLE_NORMAL, SAMPLE_BOUNDED, SAMPLE_ZERO_X0 = 0, 1, 2
X3_FELL_BACK = 1  # dpac_mlp.status bit: a split-fp16 operand left the split range (dpac.h)
GUARD_INLINE, GUARD_SPLIT_ONLY, GUARD_FALLBACK_ONLY = 0, 1, 2  # dpac_mlp.guard_phase (dpac.h)
(EVAL_DRIFT, EVAL_SIGMA, EVAL_W, EVAL_Z, EVAL_V_TRUE, EVAL_U_TRUE, EVAL_V_GRAD,
 EVAL_B) = range(8)


class DpacUnavailable(RuntimeError):
    """libdpac.so is missing or could not be loaded (no CPU fallback exists)."""


class DpacError(RuntimeError):
    def __init__(self, func: str, code: int, msg: str):
        super().__init__(f"{func} failed with status {code}: {msg}")
        self.code = code


class EqnParams(ctypes.Structure):
    """dpac_eqn_params (include/dpac.h)."""

    _fields_ = [
        ("eqn", ctypes.c_int32), ("dim", ctypes.c_int32), ("control_dim", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("gamma", ctypes.c_double), ("R", ctypes.c_double), ("sigma_up", ctypes.c_double),
        ("p", ctypes.c_double), ("q", ctypes.c_double), ("beta", ctypes.c_double),
        ("k", ctypes.c_double), ("a", ctypes.c_double), ("epsilon", ctypes.c_double),
        ("a2", ctypes.c_double), ("a3", ctypes.c_double),
    ]


MLP_MAX_HIDDEN, MLP_MAX_WIDTH = 4, 256


class Mlp(ctypes.Structure):
    """dpac_mlp (include/dpac.h): the actor MLP of dpac_rollout_nn_fwd."""

    _fields_ = [
        ("n_hidden", ctypes.c_int32), ("ekn_head", ctypes.c_int32),
        ("width", ctypes.c_int32 * (MLP_MAX_HIDDEN + 2)),
        ("bn_scale", ctypes.c_void_p * (MLP_MAX_HIDDEN + 2)),
        ("bn_shift", ctypes.c_void_p * (MLP_MAX_HIDDEN + 2)),
        ("weight", ctypes.c_void_p * (MLP_MAX_HIDDEN + 1)),
        ("bias", ctypes.c_void_p),
        ("weight_km", ctypes.c_void_p * (MLP_MAX_HIDDEN + 1)),
        ("weight_x3", ctypes.c_void_p * (MLP_MAX_HIDDEN + 1)),
        ("weight_t_x3", ctypes.c_void_p * (MLP_MAX_HIDDEN + 1)),
        ("status", ctypes.c_void_p),
        ("guard_phase", ctypes.c_int32),
    ]


_P = ctypes.c_void_p
_I32, _I64, _U64, _D = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
_EQ = ctypes.POINTER(EqnParams)

# name -> argtypes (restype int unless listed in _RESTYPES)
SIGNATURES = {
    "dpac_abi_version": [],
    "dpac_last_error": [],
    "dpac_supported": [_EQ],
    "dpac_sample": [_EQ, _I32, _I32, _I64, _I32, _U64, _I64, _P, _P, _P, _P],
    "dpac_rollout_fwd": [_EQ, _I32, _I32, _I64, _I32, _D, _P, _P, _U64, _I64, _I32, _P, _P, _P,
                         _P, _I32, _P, _P, _P],
    "dpac_flag_init": [_EQ, _I32, _I32, _I64, _I32, _D, _P, _P, _P],
    "dpac_step_fwd": [_EQ, _I32, _I32, _I64, _I32, _D, _P, _P, _P, _P, _P, _P, _I32, _P, _P, _P,
                      _P, _P, _P, _P],
    "dpac_step_bwd": [_EQ, _I32, _I32, _I64, _I32, _D, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P,
                      _P, _P, _P],
    "dpac_td_assemble_fwd": [_EQ, _I32, _I32, _I32, _I64, _I32, _P, _P, _P, _U64, _I64, _I32, _P,
                             _P, _P, _P, _P, _P],
    "dpac_td_assemble_bwd": [_EQ, _I32, _I64, _I32, _P, _P, _P, _U64, _I64, _I32, _P, _P, _P, _P,
                             _P],
    "dpac_td_assemble_bwd_gdot": [_EQ, _I32, _I64, _I32, _P, _P, _P, _P, _P],
    "dpac_actor_cost_fwd": [_EQ, _I32, _I64, _I32, _P, _P, _P, _P, _P, _P, _P],
    "dpac_equation_eval": [_EQ, _I32, _I32, _I64, _P, _P, _P, _P],
    "dpac_rollout_nn_fwd": [_EQ, _I32, _I32, _I64, _I32, _D, ctypes.POINTER(Mlp), _P, _P, _P, _P,
                            _P, _P, _I32, _P, _P, _P, _P, _P, _P],
    "dpac_rollout_nn_bwd": [_EQ, _I32, _I32, _I64, _I32, _D, ctypes.POINTER(Mlp),
                            ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p), _P, _P,
                            _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "dpac_rollout_nn_mask_tile_bytes": [ctypes.POINTER(Mlp)],
    "dpac_rollout_nn_mask_bytes": [ctypes.POINTER(Mlp), _I32, _I64, _I32],
    "dpac_rollout_nn_fwd_masked": [_EQ, _I32, _I32, _I64, _I32, _D, ctypes.POINTER(Mlp), _P, _P, _P, _P,
                                   _P, _P, _I32, _P, _P, _P, _P, _P, _P, ctypes.POINTER(_I32), _P],
    "dpac_rollout_nn_bwd_masked": [_EQ, _I32, _I32, _I64, _I32, _D, ctypes.POINTER(Mlp),
                                   ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p), _P, _P,
                                   _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "dpac_mlp_rows_fwd": [_I32, _I64, ctypes.POINTER(Mlp), _P, _I64, _P, _P, _P],
    "dpac_mlp_rows_bwd": [_I32, _I64, ctypes.POINTER(Mlp), ctypes.POINTER(ctypes.c_void_p),
                          ctypes.POINTER(ctypes.c_void_p), _P, _P, _P, _P, _P],
    "dpac_mlp_rows_fwd_td1": [_EQ, _I32, _I64, ctypes.POINTER(Mlp), _P, _I64, _P, _P, _P, _P, _P],
    "dpac_mlp_rows_bwd_td1": [_EQ, _I32, _I64, ctypes.POINTER(Mlp), ctypes.POINTER(ctypes.c_void_p),
                              ctypes.POINTER(ctypes.c_void_p), _P, _P, _I64, _P, _P, _P, _P, _P, _P],
    "dpac_mlp_rows_mask_bytes": [ctypes.POINTER(Mlp), _I32, _I64],
    "dpac_mlp_rows_fwd_masked": [_I32, _I64, ctypes.POINTER(Mlp), _P, _I64, _P, _P, _P, ctypes.POINTER(_I32), _P],
    "dpac_mlp_rows_bwd_masked": [_I32, _I64, ctypes.POINTER(Mlp), ctypes.POINTER(ctypes.c_void_p),
                                 ctypes.POINTER(ctypes.c_void_p), _P, _P, _P, _P, _P, _P],
    "dpac_mlp_rows_fwd_td1_masked": [_EQ, _I32, _I64, ctypes.POINTER(Mlp), _P, _I64, _P, _P, _P, _P, _P,
                                     ctypes.POINTER(_I32), _P],
    "dpac_mlp_rows_bwd_td1_masked": [_EQ, _I32, _I64, ctypes.POINTER(Mlp), ctypes.POINTER(ctypes.c_void_p),
                                     ctypes.POINTER(ctypes.c_void_p), _P, _P, _P, _I64, _P, _P, _P, _P, _P, _P],
    "dpac_mlp_param_grads_workspace": [_I32, _I64, ctypes.POINTER(Mlp)],
    "dpac_mlp_param_grads": [_I32, _I64, ctypes.POINTER(Mlp), _D, _P, _I64, _P, _P, _P, _I64, _P,
                             _P],
    "dpac_mlp_prepare": [_I32, ctypes.POINTER(Mlp), _D, _P, _P, _P, _P, _P, _P, _P],
    "dpac_critic_loss_grad": [_I32, _I64, _P, _P, _P, _P, _D, _D, _P, _P, _P],
    "dpac_adam_apply": [_I32, _I32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_void_p),
                        ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                        ctypes.POINTER(ctypes.c_void_p), _D, _D, _D, _D, _P],
}
_RESTYPES = {"dpac_abi_version": ctypes.c_int32, "dpac_last_error": ctypes.c_char_p,
             "dpac_supported": ctypes.c_int32, "dpac_mlp_param_grads_workspace": ctypes.c_int64,
             "dpac_rollout_nn_mask_tile_bytes": ctypes.c_int32, "dpac_rollout_nn_mask_bytes": ctypes.c_int64,
             "dpac_mlp_rows_mask_bytes": ctypes.c_int64}

_lock = threading.Lock()
_lib = None
_load_error = None


def load() -> ctypes.CDLL:
    """Load libdpac.so once; raise DpacUnavailable with the reason if impossible."""
    global _lib, _load_error
    with _lock:
        if _lib is not None:
            return _lib
        if _load_error is not None:
            raise DpacUnavailable(_load_error)
        if not os.path.exists(LIB_PATH):
            _load_error = (f"{LIB_PATH} not found: build it with `make lib` or "
                           "`python -c 'import __graft_entry__ as g; g.build()'`")
            raise DpacUnavailable(_load_error)
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the host
            _load_error = f"failed to load {LIB_PATH}: {e}"
            raise DpacUnavailable(_load_error) from e
        # check the version before binding anything: a library built from another header
        # (e.g. a stale DPAC_LIB build) would take shifted arguments
        try:
            ver_fn = lib.dpac_abi_version
        except AttributeError as e:
            _load_error = f"{LIB_PATH} does not export dpac_abi_version: not a libdpac build"
            raise DpacUnavailable(_load_error) from e
        ver_fn.argtypes, ver_fn.restype = [], ctypes.c_int32
        ver = int(ver_fn())
        if ver != ABI_VERSION:
            _load_error = (f"{LIB_PATH} has DPAC_ABI_VERSION {ver}, these bindings need {ABI_VERSION}: "
                           "rebuild it with `make lib`")
            raise DpacUnavailable(_load_error)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        for path in dim_plugins():
            try:  # its instantiations register into libdpac's dispatch table as it loads
                _plugins.append(ctypes.CDLL(path))
            except OSError as e:  # pragma: no cover - depends on the host
                _load_error = f"failed to load the dimension plugin {path}: {e}"
                raise DpacUnavailable(_load_error) from e
        _lib = lib
        return lib


_plugins = []


def dim_plugins():
    """The dimension plugins beside libdpac.so (libdpac_d<D>.so, `make ext EXT_DIMS=...`): the
    equation kernels compiled for state dimensions outside the main build's (4, 5, 10, 20)."""
    d = os.path.dirname(LIB_PATH)
    return sorted(os.path.join(d, f) for f in os.listdir(d)
                  if f.startswith("libdpac_d") and f.endswith(".so"))


def build_dim_plugin(*dims) -> None:
    """Compile and load the dimension plugins for `dims` (hipcc; a few minutes per dimension),
    e.g. for a config whose dim has no kernel instantiation (DPAC_EUNSUP)."""
    import subprocess
    root = os.path.dirname(_HERE)
    # `plugins`, not `ext`: only the plugin objects, linked against the libdpac.so in place (this
    # process has it loaded; `ext` would rebuild it wherever its objects are missing)
    subprocess.run(["make", "-C", root, "-j8", "plugins", "EXT_DIMS=" + ",".join(str(int(d)) for d in dims)],
                   check=True)
    return _load_new_plugins()


# Run-time state dimensions (round 6): the kernels are templates over d
# (register-resident state), so a dimension outside the main build runs once its plugin exists.
# ensure_dim() compiles that plugin on demand (hipcc, the same sources and flags as `make ext`)
# the first time a solver meets the dimension, under a file lock so that the ranks of a
# data-parallel job build it once; DPAC_AUTO_PLUGIN=0 turns this off (the calls then return
# DPAC_EUNSUP with the remedy in the message).
AUTO_PLUGIN = os.environ.get("DPAC_AUTO_PLUGIN", "1") != "0"
MAX_PLUGIN_DIM = 32  # register-resident state (kMaxRegDim in the kernels' static checks)


def ensure_dim(eqp, auto=None) -> bool:
    """Whether libdpac has kernels for eqp's (equation, dimension), after building and loading
    the dimension plugin on demand (AUTO_PLUGIN, 1 <= dim <= MAX_PLUGIN_DIM)."""
    lib = load()
    if lib.dpac_supported(ctypes.byref(eqp)):
        return True
    d = int(eqp.dim)
    if not (AUTO_PLUGIN if auto is None else auto) or not 1 <= d <= MAX_PLUGIN_DIM:
        return False
    import fcntl
    lock_dir = os.path.join(os.path.dirname(_HERE), "build")
    os.makedirs(lock_dir, exist_ok=True)
    with open(os.path.join(lock_dir, f".plugin_d{d}.lock"), "w") as fh:
        fcntl.flock(fh, fcntl.LOCK_EX)  # another rank may be building it: wait, then load
        try:
            if not any(os.path.basename(q) == f"libdpac_d{d}.so" for q in dim_plugins()):
                build_dim_plugin(d)
            else:  # built by another rank meanwhile
                _load_new_plugins()
        finally:
            fcntl.flock(fh, fcntl.LOCK_UN)
    return bool(lib.dpac_supported(ctypes.byref(eqp)))


def _load_new_plugins():
    """Load the plugins beside libdpac.so that this process has not loaded yet."""
    lib = load()
    have = {os.path.realpath(p._name) for p in _plugins}
    for path in dim_plugins():
        if os.path.realpath(path) not in have:
            _plugins.append(ctypes.CDLL(path))
    return lib


def call(name: str, *args) -> None:
    """Call an entry point and raise DpacError on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != DPAC_OK:
        msg = lib.dpac_last_error()
        text = msg.decode() if msg else ""
        if rc == DPAC_EUNSUP and "no kernel instantiation for dim" in text:
            text += (" (build a dimension plugin: `make ext EXT_DIMS=<dim>` or "
                     "deeppde_actorcritic_amd._lib.build_dim_plugin(<dim>))")
        raise DpacError(name, rc, text)


def exported_symbols() -> list:
    return list(SIGNATURES)
