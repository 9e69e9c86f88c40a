"""bench.py's N-rank launch path.

`python bench.py --gpus N` with N > 1 and no launcher around it starts torch.distributed.run
as a child process, before any GPU call, and relays rank 0's JSON line; every rank checks
that WORLD_SIZE equals --gpus.  The CPU tests run here (no GPU: the ranks must refuse and the
parent must return their failure); the GPU test rehearses two ranks on the one-GPU box over
gloo and reads the line.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env.update(OMP_NUM_THREADS="2", **kw)
    return env


def test_gpus_n_without_launcher_spawns_ranks_and_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check of the launcher's failure path")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-variants", "--no-cpu-baseline"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert "launching 2 ranks" in r.stderr
    assert "torch.distributed.run" in r.stderr and "--nproc-per-node 2" in r.stderr
    assert "2 ranks on this node need 2 GPUs, 0 visible" in r.stderr
    assert r.stdout.strip() == ""  # no JSON line from a failed run


def test_world_size_must_equal_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1", "--warmup", "0",
                        "--no-variants", "--no-cpu-baseline"], cwd=ROOT,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "--gpus 4 but the launcher started WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_bench_gpus_2_gloo_rehearsal_reports_two_ranks():
    """Two ranks sharing cuda:0 over gloo, launched by bench.py itself."""
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--steps", "5", "--warmup", "2",
                        "--no-cpu-baseline", "--no-train"], cwd=ROOT,
                       env=_env(DPAC_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0"),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [s for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 8192
    assert out["dist"]["world"] == 2 and out["dist"]["backend"] == "gloo"
    assert out["dist"]["launcher"] == "torch.distributed.run"
    assert out["value"] > 0 and out["roofline"]["frac"] > 0
    assert out["dist"]["note"].startswith("ranks share a GPU")
    # strong scaling: the global batch stays 4096, split 2048 + 2048
    st = out["strong_scaling"]
    assert st["scaling"] == "strong" and st["global_batch"] == 4096
    assert st["batch_per_gpu"] == 2048 and st["batch_per_rank"] == [2048, 2048]
    assert st["value"] > 0 and st["ms_per_step"] > 0 and 0 < st["roofline"]["frac"] < 1
    assert st["roofline"]["peak"] == 2 * 8000.0
    sp = out["speedup_vs_1"]
    assert sp["one_gpu_value"] > 0
    assert abs(sp["weak"] - out["value"] / sp["one_gpu_value"]) < 1e-9 * sp["weak"]
    assert abs(sp["strong"] - st["value"] / sp["one_gpu_value"]) < 1e-9 * sp["strong"]
    print("gloo rehearsal line:", json.dumps({k: out[k] for k in ("value", "n_gpus", "ms_per_step",
                                                                  "speedup_vs_1")}))
