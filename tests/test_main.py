"""main.py as the reference's drop-in CLI (main.py:20-68): the configs/*.json schema is
accepted verbatim and the run writes the reference's three log files."""
import json
import os

import numpy as np
import pytest

import main as dpac_main
from deeppde_actorcritic_amd.config import load_config
from tests.helpers import SHIPPED_LQR_D5

# the reference's configs/lqr_d5.json verbatim; the test run overrides only num_iterations
# (--num_iterations 200, logged at 0, 100, 200)
LQR_D5 = SHIPPED_LQR_D5


def write_config(tmp_path, cfg):
    path = tmp_path / "lqr_d5.json"
    path.write_text(json.dumps(cfg))
    return str(path)


def test_config_schema_accepted_verbatim(tmp_path):
    cfg = load_config(write_config(tmp_path, LQR_D5))
    assert cfg.eqn_config.eqn_name == "LQR" and cfg.eqn_config.dim == 5
    assert cfg.net_config.num_hiddens_actor == [200, 200] and cfg.net_config.dtype == "float64"
    assert cfg.train_config.TD_type == "TD1"
    a = dpac_main.parse_args(["--config_path", "x.json", "--exp_name", "e"])
    assert a.config_path == "x.json" and a.exp_name == "e" and a.log_dir == "./logs"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_main_writes_reference_logs(tmp_path, dtype):
    path = write_config(tmp_path, LQR_D5)
    logs = tmp_path / "logs"
    hist = dpac_main.main(["--config_path", path, "--exp_name", "lqr_d5", "--log_dir", str(logs),
                           "--num_iterations", "200", "--dtype", dtype, "--seed", "3"])
    char = "normal_adaptive_TD1_actor-critic"
    files = sorted(os.listdir(logs))
    assert files == sorted(["lqr_d5_config.json", f"lqr_d5_{char}.csv", f"lqr_d5_{char}_hist.csv"])
    h = np.loadtxt(logs / f"lqr_d5_{char}.csv", delimiter=",", skiprows=1)
    assert h.shape == (4, 9) and np.array_equal(h[:3, 0], [0, 100, 200])  # 3 logs + true-loss row
    assert np.all(np.isfinite(h)) and h[2, 3] < h[0, 3]  # err_value decreases from init
    f = np.loadtxt(logs / f"lqr_d5_{char}_hist.csv", delimiter=",", skiprows=1)
    assert f.shape == (1024, 5 + 1 + 1 + 5 + 5)  # valid_size rows
    assert np.allclose(hist[:, 1:8], h[:, 1:8], rtol=1e-5, atol=1e-12)  # CSV keeps 6 digits (%.5e)
    saved = json.loads((logs / "lqr_d5_config.json").read_text())
    assert saved["net_config"]["num_iterations"] == 200 and saved["eqn_config"] == LQR_D5["eqn_config"]
