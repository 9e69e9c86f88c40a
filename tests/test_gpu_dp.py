"""GPU: the multi-rank product path equals the single-process path (float64).

Launches tests/dp_equality.py as a child process under torch.distributed.run with two gloo
ranks sharing cuda:0 (RCCL needs one GPU per rank; the box has one).  Each rank runs the
product solver's train_iteration (HIP graphs, split critic step, two gradient all-reduces
per iteration: V's, then the actor's and G's in one exchange) and train(); rank 0 compares parameters, history and the final arrays with a
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


def test_rccl_single_rank_path_equals_single_process(tmp_path):
    """The same script on RCCL ("nccl" backend) with one rank on cuda:0: every collective the
    data-parallel product path issues (broadcast of the seed on a device tensor, the gradient
    all-reduces on the current and the side stream inside the training step, the metric
    reductions, the device all-gather of the final arrays) executes on RCCL, and the results
    equal the process-group-free path."""
    out = tmp_path / "dp_nccl.json"
    env = dict(os.environ, OMP_NUM_THREADS="4", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dp_equality.py"), "--backend", "nccl", "--out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["ok"] and res["world"] == 1 and res["backend"].startswith("nccl")
    for c in res["cases"]:
        assert c["params_max_rel_diff"] <= 1e-12 and c["history_max_rel_diff"] <= 1e-12
        assert c["final_arrays_rows"] == c["batch"]
