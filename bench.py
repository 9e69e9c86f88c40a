"""Benchmark of the hot path: the fused SDE rollout on the BASELINE synthetic shape.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One "step" = one launch of dpac_rollout_fwd over one batch: LQR (p=q=beta=gamma=R=1),
d = c = 20, B = 4096 trajectories per GPU, N = 200 steps, T = 0.2, adaptive
scheme, analytic control (the reference's propagate_adaptive with cheat=True,
equation.py:73-106), increments dw already resident in HBM, writing x [N+1,B,d],
dt [B,N] and coef [B,N] — the canonical rollout of SURVEY.md §8(d).
Trajectories shard across ranks by global index (weak scaling, no collective on
the data path).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "SDE trajectory-steps/sec (batch×horizon) at d=20; value-fn rel-L2 vs analytic"
B_PER_GPU, DIM, HORIZON, T_TOTAL = 4096, 20, 200, 0.2
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak
MFMA_F32_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (f32-in MFMA) dense peak
BYTES_PER_TRAJ_STEP_F32 = (2 * DIM + 2) * 4  # read dw[d] + write x[d] + dt + coef


def lqr_config():
    from deeppde_actorcritic_amd.config import munchify
    return munchify({"_comment": "synthetic", "eqn_name": "LQR", "total_time_critic": T_TOTAL,
                     "total_time_actor": T_TOTAL, "dim": DIM, "control_dim": DIM,
                     "num_time_interval_critic": HORIZON, "num_time_interval_actor": HORIZON,
                     "discount": 1.0, "p": 1.0, "q": 1.0, "beta": 1.0, "R": 1.0})


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def time_launches(launch, steps, warmup, world):
    """Warm up, then time exactly `steps` back-to-back launches between
    barrier+synchronize pairs.  A HIP event pair on the launch stream (torch's
    current stream, which every launch here uses) brackets the same launches:
    per-launch time = event span / steps, i.e. kernel time plus the dispatch gap
    between consecutive launches (rocprofv3's per-kernel average excludes it)."""
    for _ in range(warmup):
        launch()
    torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    start.record()
    for _ in range(steps):
        launch()
    end.record()
    torch.cuda.synchronize()
    barrier(world)
    wall = time.perf_counter() - t0
    per_launch_ms = start.elapsed_time(end) / steps
    return wall, per_launch_ms


def training_iteration(dtype, iters=8, warmup=3):
    """End-to-end lqr_d20 training iteration (critic step + actor step, solver.py:67-70)
    on on-device samples, the reference's shape: B=2048, N=100, 3x200 MLPs, TD1."""
    from deeppde_actorcritic_amd import equation as peq
    from deeppde_actorcritic_amd import solver as psol
    from deeppde_actorcritic_amd.config import baseline_config as lqr_d20
    cfg = lqr_d20(iters, 10 ** 9, "float32" if dtype == torch.float32 else "float64", 2048, 2048)
    sp = psol.ActorCriticSolver(cfg, peq.LQR(cfg.eqn_config), seed=1, sampler="device")
    B, N = 2048, cfg.eqn_config.num_time_interval_critic
    def iteration():  # solver.train's loop body: both samples, critic step, actor step
        dc, da = sp.sample_iteration(B, N, N)
        sp.train_iteration(dc, da)
        sp.prefetch_samples(B, N, N)  # the next pair, on a side stream
    for _ in range(warmup):
        iteration()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        iteration()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1e3
    return {"ms_per_iteration": ms, "batch": B, "horizon": N, "mlp": "20-200-200-200-20",
            "note": "critic + actor step, HIP-graph replay, fused NN rollouts; side streams: the "
                    "actor's forward rollout beside the critic step, the critic's G-network "
                    "backward beside the actor's BPTT"}


def training_dp(dtype, world, iters=5, warmup=3):
    """lqr_var_d20 (BASELINE configs[3]: global batch 16384, TD1, N=100, 3x200 MLPs,
    state-dependent diffusion) trained data-parallel over the ranks: each rank samples and
    rolls out its contiguous shard of every batch, and each optimiser step all-reduces the
    flattened gradient once over RCCL (parallel.DataParallel, solver.train_iteration).
    Strong scaling: the global batch is fixed."""
    from deeppde_actorcritic_amd import equation as peq
    from deeppde_actorcritic_amd import solver as psol
    from deeppde_actorcritic_amd.parallel import DataParallel
    from deeppde_actorcritic_amd.config import baseline_config as lqr_d20
    Bg, N = 16384, 100
    cfg = lqr_d20(iters, 10 ** 9, "float32" if dtype == torch.float32 else "float64", Bg, Bg,
                  name="lqr_var_d20")
    par = DataParallel() if world > 1 else None
    sp = psol.ActorCriticSolver(cfg, peq.LQR_var(cfg.eqn_config), seed=1, sampler="device", parallel=par)

    def iteration():  # solver.train's loop body on this rank's shards
        dc, da = sp.sample_iteration(Bg, N, N)
        sp.train_iteration(dc, da, Bg)
        sp.prefetch_samples(Bg, N, N)
    for _ in range(warmup):
        iteration()
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(iters):
        iteration()
    torch.cuda.synchronize()
    barrier(world)
    wall = max_over_ranks(time.perf_counter() - t0, world)
    ms = wall / iters * 1e3
    return {"config": "lqr_var_d20", "global_batch": Bg, "batch_per_gpu": Bg // world, "horizon": N,
            "ms_per_iteration": ms, "traj_steps_per_s": 2 * Bg * N / (ms * 1e-3), "scaling": "strong",
            "collective": (f"one all-reduce ({torch.distributed.get_backend()}; nccl = RCCL over xGMI) of "
                           "the flattened gradients per optimiser step") if world > 1 else None}


def max_over_ranks(v, world):
    if world == 1:
        return v
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(seconds=10.0):
    """Oracle (torch-CPU float64 restatement of equation.py:73-106, cheat=True) on the
    same workload shape, timed on the host cores (bounded to ~`seconds`)."""
    from oracle import equations as oeq
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    eq = oeq.LQR(lqr_config())
    np.random.seed(1234)
    x0, dw, _ = eq.sample_normal(B_PER_GPU, HORIZON)
    x0t, dwt = torch.as_tensor(x0), torch.as_tensor(dw)
    reps, t0 = 0, time.perf_counter()
    while True:
        eq.propagate_adaptive(B_PER_GPU, x0t, dwt, None, False, T_TOTAL, HORIZON, True)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 50:
            break
    return {"value": reps * B_PER_GPU * HORIZON / el, "unit": "traj-steps/s", "cores": threads,
            "kind": "port",
            "sample": f"{reps} x oracle propagate_adaptive(cheat=True), fp64, B={B_PER_GPU}, d={DIM}, "
                      f"N={HORIZON} ({el:.1f} s)"}


def pmc_traffic(key):
    """HBM bytes per launch measured by rocprofv3 PMC passes (profiles/pmc_*.json), if present."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        return d.get(key, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--scheme", choices=["adaptive", "naive"], default="adaptive")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--no-train", action="store_true", help="skip the training-iteration variant")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        # one rank per GPU; DPAC_DIST_BACKEND=gloo lets ranks share a GPU (rehearsal only)
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
        dist.init_process_group(os.environ.get("DPAC_DIST_BACKEND", "nccl"))
    else:
        torch.cuda.set_device(0)

    from deeppde_actorcritic_amd import _lib, ops
    from deeppde_actorcritic_amd.equation import LQR
    lib = _lib.load()
    eqp = LQR(lqr_config()).params()
    dtype = torch.float32 if args.dtype == "f32" else torch.float64
    esize = 4 if dtype == torch.float32 else 8
    scheme = _lib.SCHEME_ADAPTIVE if args.scheme == "adaptive" else _lib.SCHEME_NAIVE
    B, N, d = B_PER_GPU, HORIZON, DIM
    off = rank * B  # this rank's global trajectories [rank*B, rank*B + B)
    x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=1234, traj_offset=off, dtype=dtype,
                           device="cuda")
    x = torch.empty(N + 1, B, d, dtype=dtype, device="cuda")
    dt = torch.empty(B, N, dtype=dtype, device="cuda")
    coef = torch.empty(B, N, dtype=dtype, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = ctypes.c_void_p
    fn = lib.dpac_rollout_fwd

    def make_launch(dw_ptr):
        a = (ctypes.byref(eqp), scheme, _lib.F32 if dtype == torch.float32 else _lib.F64, B, N, T_TOTAL,
             P(x0.data_ptr()), dw_ptr, 1234, off, _lib.SAMPLE_NORMAL, P(x.data_ptr()), P(dt.data_ptr()),
             P(coef.data_ptr()), None, _lib.COST_CRITIC, None, None, stream)

        def launch():
            rc = fn(*a)
            if rc:
                raise _lib.DpacError("dpac_rollout_fwd", rc, lib.dpac_last_error().decode())
        return launch

    wall, per_launch_ms = time_launches(make_launch(P(dw.data_ptr())), args.steps, args.warmup, world)
    wall = max_over_ranks(wall, world)
    per_launch_ms = max_over_ranks(per_launch_ms, world)
    ms_per_step = wall / args.steps * 1e3
    value = world * B * N * args.steps / wall
    algo_bytes = B * N * (2 * d + 2) * esize
    achieved = algo_bytes / (per_launch_ms * 1e-3) / 1e9
    key = f"rollout_{args.scheme}_{args.dtype}_B{B}_N{N}_d{d}"
    traffic = pmc_traffic(key)
    out = {
        "metric": METRIC, "value": value, "unit": "traj-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic",
        "config": {"workload": f"canonical rollout, LQR d=20 synthetic: B={B}/GPU, horizon N={N}, "
                               f"T={T_TOTAL}, {args.scheme} scheme, analytic control, dw resident in HBM",
                   "batch_per_gpu": B, "global_batch": B * world, "dim": d, "horizon": N,
                   "scheme": args.scheme, "parallelism": f"dp{world} (trajectory shards)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "dpac::k_rollout", "algorithmic_bytes_per_launch": algo_bytes,
                     "avg_launch_ms": per_launch_ms},
    }
    if not args.no_variants:
        variants = {}
        # in-kernel Philox increments (dw not read): 4*(d+2) B per traj-step
        wall2, pl2 = time_launches(make_launch(None), max(20, args.steps // 4), 5, world)
        variants["rollout_inkernel_philox"] = {
            "traj_steps_per_s": world * B * N * max(20, args.steps // 4) / max_over_ranks(wall2, world),
            "avg_launch_ms": pl2, "hbm_GBps_algorithmic": B * N * (d + 2) * esize / (pl2 * 1e-3) / 1e9}
        # TD1 target assembly over the rolled-out batch: reads x,u,dw,G,dt,coef
        u = torch.zeros(N, B, d, dtype=dtype, device="cuda")
        G = torch.randn(N, B, d, dtype=dtype, device="cuda")
        y = torch.empty(B, dtype=dtype, device="cuda")
        disc = torch.empty(B, dtype=dtype, device="cuda")
        tfn = lib.dpac_td_assemble_fwd
        targs = (ctypes.byref(eqp), _lib.TD1, _lib.COST_CRITIC, _lib.F32 if dtype == torch.float32 else _lib.F64,
                 B, N, P(x.data_ptr()), P(u.data_ptr()), P(dw.data_ptr()), 0, 0, 0, P(dt.data_ptr()),
                 P(coef.data_ptr()), P(G.data_ptr()), P(y.data_ptr()), P(disc.data_ptr()), stream)

        def td_launch():
            rc = tfn(*targs)
            if rc:
                raise _lib.DpacError("dpac_td_assemble_fwd", rc, lib.dpac_last_error().decode())
        k3 = max(20, args.steps // 4)
        wall3, pl3 = time_launches(td_launch, k3, 5, world)
        variants["td1_assembly"] = {
            "traj_steps_per_s": world * B * N * k3 / max_over_ranks(wall3, world), "avg_launch_ms": pl3,
            "hbm_GBps_algorithmic": B * N * (3 * d + d + 2) * esize / (pl3 * 1e-3) / 1e9}
        # fused NN-control rollout: actor MLP d-200-200-200-d on MFMA inside the time loop
        from deeppde_actorcritic_amd import solver as psol
        from deeppde_actorcritic_amd.config import baseline_config as lqr_d20
        cfg_nn = lqr_d20(1, 1, "float32" if dtype == torch.float32 else "float64", B, B)
        net = psol.DeepNN(cfg_nn, "actor", torch.Generator().manual_seed(0), dtype, "cuda")
        view = net.mlp_view()
        nn_out = {}

        def nn_launch():
            nn_out["r"] = ops.rollout_nn(eqp, scheme, x0, dw, T_TOTAL, N, view, want_u=False)
        k4 = max(5, args.steps // 20)
        wall4, pl4 = time_launches(nn_launch, k4, 2, world)
        widths = [d, 200, 200, 200, d]
        flops = 2 * sum(widths[i] * widths[i + 1] for i in range(4)) * B * N
        tfs = flops / (pl4 * 1e-3) / 1e12
        variants["rollout_nn_fused"] = {
            "traj_steps_per_s": world * B * N * k4 / max_over_ranks(wall4, world), "avg_launch_ms": pl4,
            "mlp": "-".join(map(str, widths)),
            "roofline": {"bound": "mfma", "achieved": tfs, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": tfs / MFMA_F32_PEAK_TFS, "kernel": "dpac::k_rollout_nn"}}
        if world == 1 and not args.no_train:
            variants["training_lqr_d20"] = training_iteration(dtype)
        if not args.no_train:
            variants["training_dp_lqr_var_d20"] = training_dp(dtype, world)
        out["variants"] = variants
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
