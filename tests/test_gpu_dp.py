"""GPU: the multi-rank product path equals the single-process path (float64).

Launches tests/dp_equality.py as a child process under torch.distributed.run with two gloo
ranks sharing cuda:0 (RCCL needs one GPU per rank; the box has one).  Each rank runs the
product solver's train_iteration (HIP graphs, split critic step, three all-reduces per
iteration) and train(); rank 0 compares parameters, history and the final arrays with a
single-process run on the whole batch (see that script's docstring).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_training_equals_single_process(tmp_path):
    out = tmp_path / "dp.json"
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dp_equality.py"), "--out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["ok"] and len(res["cases"]) == 3
    for c in res["cases"]:
        assert c["params_max_rel_diff"] <= 1e-12 and c["history_max_rel_diff"] <= 1e-12
        assert c["final_arrays_rows"] == c["batch"]
