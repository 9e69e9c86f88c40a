"""CPU: libdpac.so loads, exports every entry point of include/dpac.h, and its
host-side validation rejects bad arguments before any device work."""
import ctypes
import os
import re

import pytest

from deeppde_actorcritic_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dpac.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dpac_[a-z0-9_]+)\s*\(", txt)))


def header_defines():
    out = {}
    for m in re.finditer(r"#define\s+(DPAC_[A-Z0-9_]+)\s+\(?(-?\d+)\)?", open(HEADER).read()):
        out[m.group(1)] = int(m.group(2))
    return out


def test_library_loads_and_exports_every_header_symbol():
    lib = _lib.load()
    fns = header_functions()
    assert len(fns) >= 12
    for name in fns:
        assert hasattr(lib, name), f"libdpac.so does not export {name}"
    assert sorted(_lib.exported_symbols()) == fns, "ctypes signature table out of sync with dpac.h"


def test_nm_shows_exports():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in header_functions():
        assert re.search(rf"\bT {name}$", out, re.M), name


def test_constants_match_header():
    d = header_defines()
    assert d["DPAC_ABI_VERSION"] == _lib.load().dpac_abi_version()
    pairs = {"DPAC_F32": _lib.F32, "DPAC_F64": _lib.F64, "DPAC_EQN_LQR": _lib.EQN_LQR,
             "DPAC_EQN_VDP": _lib.EQN_VDP, "DPAC_EQN_EKN": _lib.EQN_EKN,
             "DPAC_EQN_LQR_VAR": _lib.EQN_LQR_VAR, "DPAC_SCHEME_NAIVE": _lib.SCHEME_NAIVE,
             "DPAC_SCHEME_ADAPTIVE": _lib.SCHEME_ADAPTIVE, "DPAC_TD1": _lib.TD1, "DPAC_TD2": _lib.TD2,
             "DPAC_TD1_GDOT": _lib.TD1_GDOT,
             "DPAC_COST_CRITIC": _lib.COST_CRITIC, "DPAC_COST_ACTOR": _lib.COST_ACTOR,
             "DPAC_SAMPLE_NORMAL": _lib.SAMPLE_NORMAL, "DPAC_SAMPLE_BOUNDED": _lib.SAMPLE_BOUNDED,
             "DPAC_SAMPLE_ZERO_X0": _lib.SAMPLE_ZERO_X0, "DPAC_EVAL_B": _lib.EVAL_B,
             "DPAC_EVAL_V_GRAD": _lib.EVAL_V_GRAD, "DPAC_EINVAL": _lib.DPAC_EINVAL,
             "DPAC_EUNSUP": _lib.DPAC_EUNSUP, "DPAC_X3_FELL_BACK": _lib.X3_FELL_BACK,
             "DPAC_GUARD_INLINE": _lib.GUARD_INLINE, "DPAC_GUARD_SPLIT_ONLY": _lib.GUARD_SPLIT_ONLY,
             "DPAC_GUARD_FALLBACK_ONLY": _lib.GUARD_FALLBACK_ONLY}
    for k, v in pairs.items():
        assert d[k] == v, k


def test_struct_layout():
    # 4 int32 + 11 doubles, no padding surprises
    assert ctypes.sizeof(_lib.EqnParams) == 16 + 11 * 8


def _params(eqn=_lib.EQN_LQR, dim=20, cdim=20):
    p = _lib.EqnParams()
    p.eqn, p.dim, p.control_dim = eqn, dim, cdim
    p.gamma, p.R, p.sigma_up, p.p, p.q, p.beta, p.k = 1.0, 1.0, 2 ** 0.5, 1.0, 1.0, 1.0, 0.618
    return p


def test_supported_dims():
    lib = _lib.load()
    for d in (4, 5, 10, 20):
        assert lib.dpac_supported(ctypes.byref(_params(dim=d, cdim=d))) == 1
    assert lib.dpac_supported(ctypes.byref(_params(_lib.EQN_VDP, 20, 10))) == 1
    assert lib.dpac_supported(ctypes.byref(_params(_lib.EQN_VDP, 20, 20))) == 0  # needs d == 2c
    assert lib.dpac_supported(ctypes.byref(_params(_lib.EQN_LQR, 20, 10))) == 0  # needs c == d
    assert lib.dpac_supported(ctypes.byref(_params(dim=7, cdim=7))) == 1         # the d = 7 plugin
    assert lib.dpac_supported(ctypes.byref(_params(dim=9, cdim=9))) == 0         # not compiled
    bad = _params()
    bad.eqn = 9
    assert lib.dpac_supported(ctypes.byref(bad)) == 0
    assert lib.dpac_supported(None) == 0


def _net(d_in, d_out, hidden=32):
    """A dpac_mlp with dummy (never dereferenced) pointers: host validation only."""
    n = _lib.Mlp()
    n.n_hidden = 1
    n.width[0], n.width[1], n.width[2] = d_in, hidden, d_out
    for i in range(3):
        n.bn_scale[i] = n.bn_shift[i] = 0x1000
    n.weight[0] = n.weight[1] = 0x1000
    n.bias = 0x1000
    return n


def test_validation_without_gpu():
    """Bad arguments are rejected on the host with DPAC_EINVAL and a message."""
    p = _params()
    dummy = ctypes.c_void_p(0x1000)
    cases = [
        # bad scheme
        ("dpac_rollout_fwd", (ctypes.byref(p), 7, _lib.F32, 16, 10, 0.2, dummy, dummy, 0, 0, 0, dummy,
                              dummy, dummy, None, 0, None, None, None), "scheme"),
        # zero batch
        ("dpac_rollout_fwd", (ctypes.byref(p), 1, _lib.F32, 0, 10, 0.2, dummy, dummy, 0, 0, 0, dummy,
                              dummy, dummy, None, 0, None, None, None), "num_sample"),
        # missing x
        ("dpac_rollout_fwd", (ctypes.byref(p), 1, _lib.F32, 16, 10, 0.2, dummy, dummy, 0, 0, 0, None,
                              dummy, dummy, None, 0, None, None, None), "x"),
        # y without disc
        ("dpac_rollout_fwd", (ctypes.byref(p), 1, _lib.F32, 16, 10, 0.2, dummy, dummy, 0, 0, 0, dummy,
                              dummy, dummy, None, 0, dummy, None, None), "disc"),
        # bad dtype
        ("dpac_td_assemble_fwd", (ctypes.byref(p), 1, 0, 5, 16, 10, dummy, dummy, dummy, 0, 0, 0, dummy,
                                  dummy, dummy, dummy, dummy, None), "dtype"),
        # TD1 without G
        ("dpac_td_assemble_fwd", (ctypes.byref(p), 1, 0, 0, 16, 10, dummy, dummy, dummy, 0, 0, 0, dummy,
                                  dummy, None, dummy, dummy, None), "G"),
        ("dpac_step_fwd", (ctypes.byref(p), 1, 0, 16, 10, 0.2, dummy, dummy, dummy, dummy, None, None, 0,
                           dummy, dummy, None, None, None, None, None), "alias"),
        ("dpac_sample", (ctypes.byref(p), 5, 0, 16, 10, 1, 0, dummy, dummy, dummy, None), "sample_type"),
        ("dpac_equation_eval", (ctypes.byref(p), 99, 0, 16, dummy, dummy, dummy, None), "eval"),
        # fused TD1: the G network's widths must be d
        ("dpac_mlp_rows_fwd_td1", (ctypes.byref(p), 0, 64, ctypes.byref(_net(20, 16)), dummy, 20, dummy,
                                   dummy, dummy, None, None), "output width"),
        ("dpac_mlp_rows_fwd_td1", (ctypes.byref(p), 0, 64, ctypes.byref(_net(20, 20)), dummy, 20, dummy,
                                   dummy, None, None, None), "gdot"),
        ("dpac_mlp_rows_bwd_td1", (ctypes.byref(p), 0, 64, ctypes.byref(_net(20, 20)), None, None, dummy,
                                   dummy, 20, dummy, dummy, dummy, dummy, None, None), "weight_t"),
        ("dpac_td_assemble_bwd_gdot", (ctypes.byref(p), 0, 16, 10, dummy, dummy, None, dummy, None),
         "g_y"),
        ("dpac_td_assemble_fwd", (ctypes.byref(p), _lib.TD1_GDOT, 0, 0, 16, 10, dummy, dummy, None, 0, 0,
                                  0, dummy, dummy, None, dummy, dummy, None), "G"),
    ]
    for name, args, word in cases:
        with pytest.raises(_lib.DpacError) as ei:
            _lib.call(name, *args)
        assert ei.value.code == _lib.DPAC_EINVAL, (name, ei.value)
        assert word.lower() in str(ei.value).lower(), (name, str(ei.value))


def test_unsupported_dim_is_eunsup():
    p = _params(dim=9, cdim=9)  # neither the main build (4, 5, 10, 20) nor a plugin (7)
    d = ctypes.c_void_p(0x1000)
    with pytest.raises(_lib.DpacError) as ei:
        _lib.call("dpac_flag_init", ctypes.byref(p), 1, 0, 16, 10, 0.2, d, d, None)
    assert ei.value.code == _lib.DPAC_EUNSUP


def test_fused_td1_rejects_eikonal_head():
    """The fused TD1 G network (dpac_mlp_rows_fwd_td1 / _bwd_td1) refuses an Eikonal head at the
    C boundary, not only in the solver (_critic_split_ok)."""
    p = _params(_lib.EQN_EKN, 20, 20)
    p.a2, p.a3 = 1.2, 0.2
    d = ctypes.c_void_p(0x1000)
    net = _net(20, 20)
    net.ekn_head = 1
    with pytest.raises(_lib.DpacError) as ei:
        _lib.call("dpac_mlp_rows_fwd_td1", ctypes.byref(p), 0, 64, ctypes.byref(net), d, 20, d, d, d,
                  None, None)
    assert ei.value.code == _lib.DPAC_EINVAL and "eikonal" in str(ei.value).lower()
    with pytest.raises(_lib.DpacError) as ei:
        _lib.call("dpac_mlp_rows_bwd_td1", ctypes.byref(p), 0, 64, ctypes.byref(net), (ctypes.c_void_p * 2)(d, d),
                  None, d, d, 20, d, d, d, d, None, None)
    assert ei.value.code == _lib.DPAC_EINVAL


def _actor_shape_net(L=3, d=20, h=200, km=True):
    """A dpac_mlp with the actor shape of the shipped configs (dummy pointers)."""
    n = _lib.Mlp()
    n.n_hidden = L
    n.width[0] = d
    for i in range(1, L + 1):
        n.width[i] = h
    n.width[L + 1] = d
    for i in range(L + 2):
        n.bn_scale[i] = n.bn_shift[i] = 0x1000
    for i in range(L + 1):
        n.weight[i] = 0x1000
        n.weight_km[i] = 0x1000 if km else None
    n.bias = 0x1000
    return n


def test_mask_bytes_query(monkeypatch):
    """dpac_rollout_nn_mask_bytes mirrors the forward's kernel choice: a mask only for float
    16-row tiles (B > 1024 or DPAC_NN_TILE=16) on the actor-shape fast path."""
    lib = _lib.load()
    monkeypatch.delenv("DPAC_NN_TILE", raising=False)
    monkeypatch.delenv("DPAC_NN_FAST", raising=False)
    q = lambda net, dt, B, N: lib.dpac_rollout_nn_mask_bytes(ctypes.byref(net), dt, B, N)
    net = _actor_shape_net()
    tile = lib.dpac_rollout_nn_mask_tile_bytes(ctypes.byref(net))
    assert tile == 13 * 64 * 3
    assert q(net, _lib.F32, 2048, 100) == 100 * 128 * tile
    assert q(net, _lib.F32, 1030, 7) == 7 * 65 * tile
    assert q(net, _lib.F32, 1024, 100) == 0          # 4-row tiles
    assert q(net, _lib.F64, 4096, 100) == 0          # float only
    assert q(_actor_shape_net(km=False), _lib.F32, 4096, 100) == 0  # no k-major images
    assert q(_actor_shape_net(h=64), _lib.F32, 4096, 100) == 0      # not 13 column tiles
    monkeypatch.setenv("DPAC_NN_TILE", "16")
    assert q(net, _lib.F32, 100, 10) == 10 * 7 * tile
    monkeypatch.setenv("DPAC_NN_FAST", "0")
    assert q(net, _lib.F32, 4096, 10) == 0
    assert q(net, _lib.F32, 0, 10) == -1 and q(net, 7, 16, 10) == -1


def test_abi_version_mismatch_is_refused(tmp_path):
    """_lib.load() refuses a library whose dpac_abi_version differs from the bindings' (a stale
    build would take shifted arguments), before binding any entry point."""
    import subprocess
    import sys
    src = tmp_path / "old.c"
    src.write_text("int dpac_abi_version(void) { return 1; }\n")
    so = tmp_path / "libold.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    code = ("from deeppde_actorcritic_amd import _lib\n"
            "try:\n    _lib.load()\nexcept _lib.DpacUnavailable as e:\n    print('REFUSED', e)\n")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                         env=dict(os.environ, DPAC_LIB=str(so)))
    assert "REFUSED" in out.stdout and "DPAC_ABI_VERSION 1" in out.stdout, out.stdout + out.stderr


def test_dimension_plugin_registers_d7():
    """libdpac_d7.so (make ext, built by __graft_entry__.build()) adds the d = 7 kernels to the
    dispatch table as _lib.load() loads it; a dimension with neither the main build nor a plugin
    is reported as DPAC_EUNSUP with the remedy in the message (host-side, no GPU)."""
    from deeppde_actorcritic_amd import equation as peq
    from tests.helpers import full_config
    lib = _lib.load()
    assert any(p.endswith("libdpac_d7.so") for p in _lib.dim_plugins())
    for name in ("LQR", "EKN", "LQR_var"):
        assert lib.dpac_supported(getattr(peq, name)(full_config(name, 7).eqn_config).params()) == 1
    p9 = peq.LQR(full_config("LQR", 9).eqn_config).params()
    assert lib.dpac_supported(p9) == 0
    with pytest.raises(_lib.DpacError) as ei:
        _lib.call("dpac_flag_init", ctypes.byref(p9), _lib.SCHEME_ADAPTIVE, _lib.F64, 4, 10, 0.2, None, None, None)
    assert ei.value.code == _lib.DPAC_EUNSUP and "make ext" in str(ei.value)


def test_ensure_dim_builds_the_plugin_on_demand(monkeypatch, tmp_path):
    """Round 6: a solver meeting a dimension without kernels has its plugin
    compiled on demand (`make ext EXT_DIMS=<d>`, under a lock file so data-parallel ranks build it
    once) and loaded; DPAC_AUTO_PLUGIN=0 (auto=False) leaves it unsupported, and dimensions above
    MAX_PLUGIN_DIM are refused.  Host-side: the build command is captured, not run."""
    import subprocess
    from deeppde_actorcritic_amd import equation as peq
    from tests.helpers import full_config
    built = []

    class FakeLib:
        def dpac_supported(self, eq_ref):
            return 1 if built else 0
    monkeypatch.setattr(_lib, "load", lambda: FakeLib())
    monkeypatch.setattr(_lib, "_load_new_plugins", lambda: FakeLib())
    monkeypatch.setattr(subprocess, "run", lambda cmd, check: built.append(cmd))
    p9 = peq.LQR(full_config("LQR", 9).eqn_config).params()
    assert _lib.ensure_dim(p9, auto=False) is False and not built
    assert _lib.ensure_dim(p9, auto=True) is True
    assert len(built) == 1 and built[0][-2:] == ["plugins", "EXT_DIMS=9"]
    assert _lib.ensure_dim(p9, auto=True) is True and len(built) == 1  # supported now: no rebuild
    built.clear()
    p40 = peq.LQR(full_config("LQR", 40).eqn_config).params()
    assert _lib.ensure_dim(p40, auto=True) is False and not built
