"""Benchmark of the hot path: the fused SDE rollout on the BASELINE synthetic shape.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Both forms run N ranks: without a launcher around it, `--gpus N > 1` starts
torch.distributed.run as a child process (before any GPU call) and relays rank 0's line.
Every rank checks WORLD_SIZE == --gpus and, on RCCL, one GPU per rank.

One "step" = one launch of dpac_rollout_fwd over one batch: LQR (p=q=beta=gamma=R=1),
d = c = 20, B = 4096 trajectories per GPU, N = 200 steps, T = 0.2, adaptive
scheme, analytic control (the reference's propagate_adaptive with cheat=True,
equation.py:73-106), increments dw already resident in HBM, writing x [N+1,B,d],
dt [B,N] and coef [B,N] — the canonical rollout of SURVEY.md §8(d).
The timed launches rotate over 5 batches (buffer sets of 138 MB each, 690 MB in all), so
a launch's inputs and outputs are not resident in the 256 MiB Infinity Cache from the
previous launch: `value` and `roofline` are HBM figures, both from the same wall clock
(barrier + synchronize on both sides of the K launches); the HIP event pair over the same
launches is reported beside it (roofline.event_pair).  The single-set loop (everything
MALL-resident) is the variant `rollout_mall_resident`, run only with --mall: it launches the
same kernel, and without it every launch of the headline kernel in a default run is a cold
one, so a rocprofv3 summary of the driver's command averages exactly the headline's launches.
Trajectories shard across ranks by global index (weak scaling, no collective on
the data path).  Beside the weak-scaling headline the line carries `strong_scaling` (the same
rollout with the GLOBAL batch fixed at 4096 and split over the ranks by parallel.shard_range,
SURVEY §8(d)) and `speedup_vs_1`: both figures divided by the one-GPU figure, which rank 0
measures alone inside the same job (the other ranks wait at a barrier), so the driver's 1->8
run reads a measured speed-up, not one true by construction.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "SDE trajectory-steps/sec (batch×horizon) at d=20; value-fn rel-L2 vs analytic"
B_PER_GPU, DIM, HORIZON, T_TOTAL = 4096, 20, 200, 0.2
B_STRONG = 4096  # strong scaling: the global batch, split over the ranks
N_SETS = 5  # rotating buffer sets: 5 x 138 MB (f32) > the 256 MiB Infinity Cache
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak
MFMA_F32_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (f32-in MFMA) dense peak
MFMA_F16_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 MFMA dense peak (~2.5 PF)
MFMA_F64_PEAK_TFS = 78.6  # AMD's MI355X spec: FP64 matrix dense peak (not in the guide)
MLP_FLOP_PER_ROW = 2 * (20 * 200 + 200 * 200 * 2 + 200 * 20)  # 176 000


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
    barrier+synchronize pairs (the wall clock: `value` and the headline roofline).  A HIP
    event pair on the launch stream (torch's current stream, which every launch here uses)
    brackets the same launches, its start recorded before the wall bracket opens (so the
    bracket holds nothing but the launches): per-launch time = event span / steps, kernel
    time plus the dispatch gaps (rocprofv3's per-kernel average excludes them)."""
    for i in range(warmup):
        launch(i)
    torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()  # before the wall bracket: the bracket holds only the K launches (and end's record)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        launch(i)
    end.record()
    torch.cuda.synchronize()
    barrier(world)
    wall = time.perf_counter() - t0
    per_launch_ms = start.elapsed_time(end) / steps
    return wall, per_launch_ms


def progress(msg):
    """One progress line on stderr (a long bench phase — the CPU baseline, the training
    variants — must not look hung to a watchdog that reads the output)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def max_over_ranks(v, world):
    if world == 1:
        return v
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class RolloutSets:
    """n buffer sets (x0, dw, x, dt, coef) of this rank's shard and a launcher of
    dpac_rollout_fwd over set i % n."""

    def __init__(self, lib, eqp, scheme, dtype, B, N, d, off, n):
        from deeppde_actorcritic_amd import _lib, ops
        self.lib, self.B, self.N = lib, B, N
        self.sets = []
        for i in range(n):
            x0, dw, _ = ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=1234 + i, traj_offset=off,
                                   dtype=dtype, device="cuda")
            x = torch.empty(N + 1, B, d, dtype=dtype, device="cuda")
            dt = torch.empty(B, N, dtype=dtype, device="cuda")
            coef = torch.empty(B, N, dtype=dtype, device="cuda")
            self.sets.append((x0, dw, x, dt, coef))
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        P = ctypes.c_void_p
        dt_id = _lib.F32 if dtype == torch.float32 else _lib.F64
        self.args = [(ctypes.byref(eqp), scheme, dt_id, B, N, T_TOTAL, P(x0.data_ptr()), P(dw.data_ptr()),
                      1234 + i, off, _lib.SAMPLE_NORMAL, P(x.data_ptr()), P(dt.data_ptr()),
                      P(coef.data_ptr()), None, _lib.COST_CRITIC, None, None, stream)
                     for i, (x0, dw, x, dt, coef) in enumerate(self.sets)]
        self.philox_args = [a[:7] + (None,) + a[8:] for a in self.args]
        self.err = _lib.DpacError

    def launcher(self, nsets, philox=False):
        fn, args = self.lib.dpac_rollout_fwd, (self.philox_args if philox else self.args)

        def launch(i):
            rc = fn(*args[i % nsets])
            if rc:
                raise self.err("dpac_rollout_fwd", rc, self.lib.dpac_last_error().decode())
        return launch


def training_variant(name, dtype, B, world=1, iters=6, warmup=3, par=None, total=None):
    """One BASELINE config's training iteration (critic step + actor step, solver.py:67-70,
    one sample pair per iteration; the solver's production path: device sampler, HIP
    graphs, split critic/actor steps on side streams, MFMA kernels, Adam kernel).
    B = this rank's batch, total = the global batch (data parallel) or None."""
    from deeppde_actorcritic_amd import equation as peq
    from deeppde_actorcritic_amd import solver as psol
    from deeppde_actorcritic_amd.config import baseline_config
    Bg = total or B
    progress(f"training variant {name}: batch {Bg} ({B} per rank)")
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    mem0 = torch.cuda.memory_allocated()
    cfg = baseline_config(iters, 10 ** 9, "float32" if dtype == torch.float32 else "float64", Bg, Bg, name=name)
    bsde = getattr(peq, cfg.eqn_config.eqn_name)(cfg.eqn_config)
    sp = psol.ActorCriticSolver(cfg, bsde, seed=1, sampler="device", parallel=par)
    N = cfg.eqn_config.num_time_interval_critic

    def iteration():  # solver.train's loop body on this rank's shards
        dc, da = sp.sample_iteration(Bg, N, N)
        sp.train_iteration(dc, da, Bg)
        sp.prefetch_samples(Bg, N, N)
    for _ in range(warmup):
        iteration()
    torch.cuda.synchronize()
    if par is not None:
        par.timings = []  # the gradient all-reduces of the timed iterations
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(iters):
        iteration()
    torch.cuda.synchronize()
    barrier(world)
    ms = max_over_ranks(time.perf_counter() - t0, world) / iters * 1e3
    coll = None
    if par is not None:
        tm, par.timings = par.timings, None
        ev_ms = sum(a.elapsed_time(b) for a, b, _ in tm) / iters
        coll = {"allreduces_per_iteration": len(tm) / iters,
                "allreduce_ms_per_iteration": max_over_ranks(ev_ms, world),
                "allreduce_host_ms_per_iteration": max_over_ranks(sum(h for _, _, h in tm) / iters * 1e3, world),
                "bytes_per_iteration": None if not tm else sum(
                    p.numel() * p.element_size() for p in sp.critic_variables() + sp.actor_variables()),
                "note": "HIP events on the calling stream around each dist.all_reduce of the timed "
                        "iterations (parallel.DataParallel.timings), summed per iteration, max over ranks; "
                        "host_ms: the Python call's wall time"}
    # MLP work per iteration, in forward-pass equivalents (176 kFLOP per row at d = 20) per
    # trajectory-step: EXECUTED by this build = 7 (actor forward in the critic's rollout, G
    # forward, G backward chain + G parameter gradients = 2, actor forward with saves,
    # BPTT chain, actor parameter gradients); the reference executes 11 (SURVEY §8(d),
    # with its duplicated NN_control evaluations, quirk 7).  An achieved rate, not a roofline.
    rate = Bg * N / (ms * 1e-3) * MLP_FLOP_PER_ROW / 1e12
    return {"config": name, "global_batch": Bg, "batch_per_gpu": Bg // max(world, 1), "horizon": N,
            "mlp": "20-200-200-200-%d" % cfg.eqn_config.control_dim, "ms_per_iteration": ms,
            "traj_steps_per_s": 2 * Bg * N / (ms * 1e-3),
            "mlp_executed_TFLOPs": 7 * rate, "mlp_reference_equiv_TFLOPs": 11 * rate,
            "mlp_math": ops_mlp_math(dtype), "collectives": coll, "graph_sets": psol.graph_sets(B),
            "peak_memory_GB": (torch.cuda.max_memory_allocated() - mem0) / 1e9,
            "peak_memory_note": "device memory this variant's solver, samples and HIP graph pools held at "
                                "their peak, above what was allocated before it (torch caching allocator)"}


def ops_mlp_math(dtype):
    """How this build's MLP kernels multiply (deeppde_actorcritic_amd.ops.MLP_MATH)."""
    from deeppde_actorcritic_amd import ops
    if dtype != torch.float32:
        return "f64 MFMA (v_mfma_f64_16x16x4_f64)"
    if ops.MLP_MATH == "x3":
        return ("f32 via split-fp16 MFMA (3 v_mfma_f32_16x16x32_f16 per product, f32 accumulate; "
                "f32-accurate, DESIGN.md 4.3) in the fused actor rollout / BPTT, the critic's row "
                "kernels and the parameter gradients")
    return "exact f32 MFMA (v_mfma_f32_16x16x4_f32)"


def cpu_info():
    model = platform.processor() or "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, os.cpu_count() or 1


def cpu_baseline(seconds=8.0):
    """The oracle (torch-CPU restatement; test infrastructure, timed here only) on the host
    cores: (i) the canonical rollout (equation.py:73-106, cheat=True) at the bench shape,
    fp64 and fp32; (ii) one full lqr_d20 training iteration (critic step + actor step,
    solver.py:67-70) at BASELINE's B = 4096, fp64 and fp32.  Threads = the box's CPU share
    for one GPU (16; `nproc` counts the whole host).  Bounded samples (about a minute in all)."""
    from oracle import equations as oeq
    from oracle import precision
    from oracle import solver as osol
    from deeppde_actorcritic_amd.config import baseline_config
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    model, nproc = cpu_info()
    entries = {}
    for dt in (torch.float64, torch.float32):
        precision.set_dtype(dt)
        tag = "f64" if dt == torch.float64 else "f32"
        eq = oeq.LQR(lqr_config())
        np.random.seed(1234)
        x0, dw, _ = eq.sample_normal(B_PER_GPU, HORIZON)
        x0t, dwt = torch.as_tensor(x0, dtype=dt), torch.as_tensor(dw, dtype=dt)
        reps, t0 = 0, time.perf_counter()
        while True:
            eq.propagate_adaptive(B_PER_GPU, x0t, dwt, None, False, T_TOTAL, HORIZON, True)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds or reps >= 50:
                break
        progress(f"cpu_baseline rollout {tag}: {reps} reps in {el:.1f} s")
        entries[f"rollout_{tag}"] = {
            "value": reps * B_PER_GPU * HORIZON / el, "unit": "traj-steps/s",
            "sample": f"{reps} x oracle propagate_adaptive(cheat=True), {tag}, B={B_PER_GPU}, d={DIM}, "
                      f"N={HORIZON} ({el:.1f} s)"}
        Bt = 4096
        cfg = baseline_config(1, 1, "float64" if dt == torch.float64 else "float32", Bt, Bt, "lqr_d20")
        eqi = oeq.make(cfg.eqn_config)
        gen = torch.Generator().manual_seed(1)
        params = {k: osol.init_params(osol.DeepNN(cfg, ac).sizes, gen)
                  for k, ac in (("critic", "critic"), ("critic_grad", "critic_grad"), ("actor", "actor"))}
        so = osol.ActorCriticSolver(cfg, eqi, params=params)
        np.random.seed(7)
        dc, da = so.sample(Bt, 100), so.sample(Bt, 100)
        t0 = time.perf_counter()
        so.train_step_critic(dc)
        so.train_step_actor(da)
        el = time.perf_counter() - t0
        progress(f"cpu_baseline iteration {tag}: {el:.1f} s")
        entries[f"iteration_lqr_d20_{tag}"] = {
            "value": 2 * Bt * 100 / el, "unit": "traj-steps/s", "ms_per_iteration": el * 1e3,
            "sample": f"1 oracle training iteration (critic + actor step) on lqr_d20, {tag}, B={Bt}, "
                      f"N=100, 3x200 MLPs ({el:.1f} s)"}
    # the same rollout on ALL of the host's cores (f64), a bounded sample — only where the job
    # may use them: a GPU box allots each job a CPU share (OMP_NUM_THREADS, 16 per GPU) of a
    # much larger host, and oversubscribing it stalls a single repetition for minutes
    allotted = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    try:
        allotted = min(allotted or nproc, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    if allotted and allotted < nproc:
        entries["rollout_f64_all_cores"] = {
            "value": None, "cores_visible": nproc, "cores_allotted": allotted,
            "note": f"not run: this job is allotted {allotted} of the host's {nproc} CPUs "
                    f"(OMP_NUM_THREADS); rollout_f64 above uses that share"}
        progress(f"cpu_baseline all-cores entry skipped: {allotted} of {nproc} CPUs allotted")
    else:
        precision.set_dtype(torch.float64)
        torch.set_num_threads(nproc)
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
        progress(f"cpu_baseline rollout f64 on {nproc} threads: {reps} reps in {el:.1f} s")
        entries["rollout_f64_all_cores"] = {
            "value": reps * B_PER_GPU * HORIZON / el, "unit": "traj-steps/s", "cores": nproc,
            "sample": f"{reps} x oracle propagate_adaptive(cheat=True), f64, B={B_PER_GPU}, d={DIM}, N={HORIZON}, "
                      f"torch threads = nproc = {nproc} ({el:.1f} s)"}
    torch.set_num_threads(threads)
    head = entries["rollout_f64"]
    return {"value": head["value"], "unit": "traj-steps/s", "cores": threads, "kind": "port",
            "sample": head["sample"] + "; the reference's precision (float64, main.py:35)",
            "cpu_model": model, "nproc": nproc, "entries": entries}


def pmc_traffic(key):
    """HBM bytes per launch measured by rocprofv3 PMC passes of this bench command
    (profiles/pmc_traffic.json, written by tools/collect_profiles.py), if present."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p)).get(key, {})
        return d.get("hbm_bytes_per_launch"), d.get("source")
    except Exception:
        return None, None


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`python bench.py --gpus N` (N > 1) run without a torch.distributed launcher: start one
    as a CHILD process — one rank per GPU, rendezvous on 127.0.0.1 — and relay its output.
    The parent has made no HIP call (importing torch does not initialise the GPU) and never
    re-execs itself; it forwards rank 0's JSON line to stdout, everything else to stderr, and
    returns the child's exit status."""
    import subprocess
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes", "1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    progress(f"launching {n} ranks: {' '.join(cmd[2:])}")
    proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, text=True)
    for line in proc.stdout:
        s = line.strip()
        if s.startswith("{") and '"metric"' in s:
            print(s, flush=True)
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    return proc.wait()


def strong_scaling(lib, eqp, scheme, dtype, rank, world, args, value, ms_per_step, esize, solo_value):
    """The headline rollout with the GLOBAL batch fixed at B_STRONG = 4096 trajectories, split
    over the ranks by parallel.shard_range (rank r rolls out global trajectories
    [offset_r, offset_r + count_r): trajectories are independent, equation.py:53-69), the same
    N_SETS cold buffer sets, barrier + synchronize wall clock, max over ranks.  frac is the
    algorithmic bytes over the wall time against the aggregate HBM peak of the world's GPUs.
    At N = 1 it is the headline itself (B_STRONG = B_PER_GPU)."""
    from deeppde_actorcritic_amd.parallel import shard_range
    N, d = HORIZON, DIM
    off, cnt = shard_range(B_STRONG, rank, world)
    per_gpu = [shard_range(B_STRONG, r, world)[1] for r in range(world)]
    if world == 1 and B_STRONG == B_PER_GPU:
        wall_ms = ms_per_step
    else:
        progress(f"strong scaling: global batch {B_STRONG}, {cnt} trajectories on rank {rank}")
        rs = RolloutSets(lib, eqp, scheme, dtype, cnt, N, d, off, N_SETS)
        wall, _ = time_launches(rs.launcher(N_SETS), args.steps, args.warmup, world)
        wall_ms = max_over_ranks(wall, world) / args.steps * 1e3
        del rs
    v = B_STRONG * N / (wall_ms * 1e-3)
    achieved = B_STRONG * N * (2 * d + 2) * esize / (wall_ms * 1e-3) / 1e9
    return {"value": v, "unit": "traj-steps/s", "ms_per_step": wall_ms, "scaling": "strong",
            "global_batch": B_STRONG, "batch_per_gpu": max(per_gpu), "batch_per_rank": per_gpu,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                         "frac": achieved / (HBM_PEAK_GBS * world),
                         "note": "algorithmic bytes (168 B per trajectory-step) of the whole 4096-trajectory "
                                 "batch / the max-over-ranks wall time per step, against the world's "
                                 "aggregate HBM peak"},
            "note": "each trajectory is a sequential 200-step chain on one 16-lane group, and at B = 4096 "
                    "one GPU already runs one wavefront per SIMD, so a rank's shard takes about the per-wave "
                    "chain latency whatever its size: strong scaling of THIS batch is latency-bound "
                    "(variants.strong_scaling_shard_proxy times the shards on one GPU)"}


def check_world(args, world):
    """Every rank: the launcher's world size is the --gpus asked for, and (RCCL) each rank has
    a GPU of its own.  DPAC_DIST_BACKEND=gloo is the rehearsal mode in which ranks may share
    a GPU (the one-GPU test box); it is reported as such in the line."""
    backend = os.environ.get("DPAC_DIST_BACKEND", "nccl") if world > 1 else None
    visible = torch.cuda.device_count()
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if backend == "nccl" and visible < local_world:
        raise SystemExit(f"bench.py: {local_world} ranks on this node need {local_world} GPUs, "
                         f"{visible} visible (DPAC_DIST_BACKEND=gloo rehearses ranks sharing a GPU)")
    if visible < 1:
        raise SystemExit("bench.py: no GPU visible")
    return backend, visible


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--scheme", choices=["adaptive", "naive"], default="adaptive")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--no-train", action="store_true", help="skip the training-iteration variants")
    ap.add_argument("--strong-proxy", action="store_true",
                    help="also time the strong-scaling shards (B = 4096 / 2, 4, 8) on this one GPU")
    ap.add_argument("--mall", action="store_true",
                    help="also time the MALL-resident one-set loop (same kernel as the headline)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    backend, visible = check_world(args, world)
    if world > 1:
        import torch.distributed as dist
        # one rank per GPU; DPAC_DIST_BACKEND=gloo lets ranks share a GPU (rehearsal only)
        torch.cuda.set_device(local_rank % visible)
        dist.init_process_group(backend)
        assert dist.get_world_size() == world
    else:
        torch.cuda.set_device(0)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    devices = min(visible, local_world)  # this node's GPUs in use
    # ranks share a GPU only when this node runs more ranks than it has GPUs (the gloo
    # rehearsal); a multi-node launch has world > the node's GPUs with one rank per GPU
    shared = world > 1 and local_world > visible

    from deeppde_actorcritic_amd import _lib, ops
    from deeppde_actorcritic_amd.equation import LQR
    lib = _lib.load()
    eqp = LQR(lqr_config()).params()
    dtype = torch.float32 if args.dtype == "f32" else torch.float64
    esize = 4 if dtype == torch.float32 else 8
    scheme = _lib.SCHEME_ADAPTIVE if args.scheme == "adaptive" else _lib.SCHEME_NAIVE
    B, N, d = B_PER_GPU, HORIZON, DIM
    off = rank * B  # this rank's global trajectories [rank*B, rank*B + B)
    rs = RolloutSets(lib, eqp, scheme, dtype, B, N, d, off, N_SETS)

    progress(f"headline: {args.warmup} + {args.steps} launches over {N_SETS} cold buffer sets")
    wall, per_launch_ms = time_launches(rs.launcher(N_SETS), args.steps, args.warmup, world)
    wall = max_over_ranks(wall, world)
    per_launch_ms = max_over_ranks(per_launch_ms, world)
    ms_per_step = wall / args.steps * 1e3
    value = world * B * N * args.steps / wall
    algo_bytes = B * N * (2 * d + 2) * esize
    # the one-GPU figure of the same job: rank 0 alone (the others wait at a barrier), the same
    # B = 4096 batch, launches and timer; at N = 1 it is the headline itself
    if world > 1:
        barrier(world)
        if rank == 0:
            progress("one-GPU reference: rank 0 alone")
            solo_wall, _ = time_launches(rs.launcher(N_SETS), args.steps, args.warmup, 1)
            solo_value = B * N * args.steps / solo_wall
        else:
            solo_value = 0.0
        barrier(world)
        solo_value = max_over_ranks(solo_value, world)
    else:
        solo_value = value
    strong = strong_scaling(lib, eqp, scheme, dtype, rank, world, args, value, ms_per_step, esize,
                            solo_value)
    # the same timer as `value`: the wall clock over the K launches (max over ranks) / K
    achieved = algo_bytes / (ms_per_step * 1e-3) / 1e9
    achieved_ev = algo_bytes / (per_launch_ms * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic(f"rollout_{args.scheme}_{args.dtype}_B{B}_N{N}_d{d}_cold{N_SETS}")
    out = {
        "metric": METRIC, "value": value, "unit": "traj-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic",
        "config": {"workload": f"canonical rollout, LQR d=20 synthetic: B={B}/GPU, horizon N={N}, "
                               f"T={T_TOTAL}, {args.scheme} scheme, analytic control, dw resident in HBM; "
                               f"launches rotate over {N_SETS} batches (not Infinity-Cache resident)",
                   "batch_per_gpu": B, "global_batch": B * world, "dim": d, "horizon": N,
                   "scheme": args.scheme, "parallelism": f"dp{world} (trajectory shards)"},
        "dist": {"world": world, "backend": backend, "devices_used": devices,
                 "gpus_visible_per_rank": visible,
                 "launcher": "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else (
                     "external" if world > 1 else None),
                 "note": ("ranks share a GPU: DPAC_DIST_BACKEND=gloo rehearsal, not a scaling figure"
                          if shared else "one rank per GPU")},
        "strong_scaling": strong,
        "speedup_vs_1": {"weak": value / solo_value, "strong": strong["value"] / solo_value,
                         "one_gpu_value": solo_value, "unit": "traj-steps/s",
                         "note": "one_gpu_value: B = 4096 on ONE GPU (rank 0 alone inside this job, the "
                                 "same launches and wall timer; at N = 1 the headline itself); weak = "
                                 "value / one_gpu_value (B = 4096 per GPU), strong = strong_scaling.value / "
                                 "one_gpu_value (B = 4096 in all)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": tsrc, "kernel": "dpac::k_rollout_staged",
                     "algorithmic_bytes_per_launch": algo_bytes, "ms_per_launch": ms_per_step,
                     "event_pair": {"avg_launch_ms": per_launch_ms, "achieved": achieved_ev,
                                    "frac": achieved_ev / HBM_PEAK_GBS},
                     "note": "achieved = algorithmic bytes (168 B per trajectory-step) / ms_per_step, the "
                             "wall clock that gives `value` (barrier + synchronize around the K launches, "
                             "max over ranks); event_pair: the HIP event pair over the same launches on the "
                             "launch stream.  Every launch of this kernel in a default run (N = 1) is an "
                             "HBM-cold one, so rocprofv3 --stats of the same command averages them "
                             "(tools/rocprof_headline.py -> profiles/r06_rocprof_headline.json)"},
    }
    if not args.no_variants:
        progress("variants: in-kernel Philox, float64, TD1, fused NN rollout" + (", MALL-resident" if args.mall else ""))
        variants = {}
        k2 = max(20, args.steps // 4)
        if args.mall:
            # the same launch on ONE buffer set: inputs and outputs stay in the Infinity Cache
            w1, pl1 = time_launches(rs.launcher(1), k2, 5, world)
            variants["rollout_mall_resident"] = {
                "traj_steps_per_s": world * B * N * k2 / max_over_ranks(w1, world), "avg_launch_ms": pl1,
                "GBps_algorithmic": algo_bytes / (pl1 * 1e-3) / 1e9,
                "frac_of_hbm_peak": algo_bytes / (pl1 * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "note": "one 138 MB buffer set re-used every launch (Infinity-Cache resident)"}
        # in-kernel Philox increments (dw not read): 4*(d+2) B per traj-step
        w2, pl2 = time_launches(rs.launcher(N_SETS, philox=True), k2, 5, world)
        variants["rollout_inkernel_philox"] = {
            "traj_steps_per_s": world * B * N * k2 / max_over_ranks(w2, world),
            "avg_launch_ms": pl2, "hbm_GBps_algorithmic": B * N * (d + 2) * esize / (pl2 * 1e-3) / 1e9}
        # the device sampler (k_sample_dw, equation.py:13-23's draws) at the bench shape, writing
        # x0, dw [N, B, d] and x_bdry: (N + 2)·B·d elements per call
        sbufs = [tuple(torch.empty(t.shape, dtype=dtype, device=t.device) for t in (st[0], st[1], st[0]))
                 for st in rs.sets]

        def sample_launch(i):
            x0s, dws, xbs = sbufs[i % N_SETS]
            ops.sample(eqp, _lib.SAMPLE_NORMAL, B, N, seed=99 + i, traj_offset=off, dtype=dtype,
                       device=x0s.device, out=(x0s, dws, xbs))
        w6, pl6 = time_launches(sample_launch, k2, 5, world)
        sbytes = (N + 2) * B * d * esize
        variants["sample_normal_device"] = {
            "kernel": "dpac::k_sample_dw (+ the x0 / x_bdry launch)", "traj_steps_per_s":
            world * B * N * k2 / max_over_ranks(w6, world), "avg_call_ms": pl6,
            "roofline": {"bound": "hbm", "achieved": sbytes / (pl6 * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": sbytes / (pl6 * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_call": sbytes},
            "note": "ops.sample into the bench's cold buffer sets (Philox4x32-10 normals, every generated "
                    "normal used): the bytes written over the HIP event pair per call"}
        del sbufs
        if args.strong_proxy and world == 1:
            # what a rank of the strong-scaling run computes, timed on this one GPU: the
            # 4096-trajectory batch's shard for 2, 4 and 8 ranks
            from deeppde_actorcritic_amd.parallel import shard_range
            prox = {}
            for g in (2, 4, 8):
                cnt = shard_range(B_STRONG, 0, g)[1]
                rsg = RolloutSets(lib, eqp, scheme, dtype, cnt, N, d, 0, N_SETS)
                wg, _ = time_launches(rsg.launcher(N_SETS), args.steps, args.warmup, 1)
                del rsg
                msg = wg / args.steps * 1e3
                prox[f"gpus_{g}"] = {"batch_per_gpu": cnt, "ms_per_step": msg,
                                     "predicted_strong_speedup": ms_per_step / msg}
            variants["strong_scaling_shard_proxy"] = {
                "shards": prox, "note": "one rank's shard of the 4096-trajectory batch timed alone on one "
                                        "GPU (no collective exists on this path, so a rank's time is its "
                                        "shard's); predicted speed-up = the headline's ms_per_step / the shard's"}
        # the reference's own precision (float64, main.py:35): 336 B per traj-step
        if dtype == torch.float32:
            rs64 = RolloutSets(lib, eqp, scheme, torch.float64, B, N, d, off, N_SETS)
            w5, pl5 = time_launches(rs64.launcher(N_SETS), k2, 5, world)
            w5 = max_over_ranks(w5, world)
            ms5 = w5 / k2 * 1e3
            b64 = B * N * (2 * d + 2) * 8
            variants["rollout_f64"] = {
                "traj_steps_per_s": world * B * N * k2 / w5, "ms_per_launch": ms5,
                "roofline": {"bound": "hbm", "achieved": b64 / (ms5 * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": b64 / (ms5 * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "algorithmic_bytes_per_launch": b64,
                             "event_pair": {"avg_launch_ms": pl5, "achieved": b64 / (pl5 * 1e-3) / 1e9,
                                            "frac": b64 / (pl5 * 1e-3) / 1e9 / HBM_PEAK_GBS}},
                "note": f"float64 (the reference's dtype), {N_SETS} rotating sets of 276 MB; achieved from "
                        "the same wall clock as `value` (barrier + synchronize around the launches), the "
                        "HIP event pair beside it"}
            del rs64
        # TD1 target assembly over one rolled-out batch: reads x,u,dw,G,dt,coef
        x0, dw, x, dtb, coef = rs.sets[0]
        u = torch.zeros(N, B, d, dtype=dtype, device="cuda")
        G = torch.randn(N, B, d, dtype=dtype, device="cuda")
        y = torch.empty(B, dtype=dtype, device="cuda")
        disc = torch.empty(B, dtype=dtype, device="cuda")
        P = ctypes.c_void_p
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        tfn = lib.dpac_td_assemble_fwd
        targs = (ctypes.byref(eqp), _lib.TD1, _lib.COST_CRITIC, _lib.F32 if dtype == torch.float32 else _lib.F64,
                 B, N, P(x.data_ptr()), P(u.data_ptr()), P(dw.data_ptr()), 0, 0, 0, P(dtb.data_ptr()),
                 P(coef.data_ptr()), P(G.data_ptr()), P(y.data_ptr()), P(disc.data_ptr()), stream)

        def td_launch(i):
            rc = tfn(*targs)
            if rc:
                raise _lib.DpacError("dpac_td_assemble_fwd", rc, lib.dpac_last_error().decode())
        w3, pl3 = time_launches(td_launch, k2, 5, world)
        variants["td1_assembly"] = {
            "traj_steps_per_s": world * B * N * k2 / max_over_ranks(w3, world), "avg_launch_ms": pl3,
            "hbm_GBps_algorithmic": B * N * (3 * d + d + 2) * esize / (pl3 * 1e-3) / 1e9}
        # fused NN-control rollout: actor MLP d-200-200-200-d on MFMA inside the time loop
        from deeppde_actorcritic_amd import solver as psol
        from deeppde_actorcritic_amd.config import baseline_config
        cfg_nn = baseline_config(1, 1, "float32" if dtype == torch.float32 else "float64", B, B)
        net = psol.DeepNN(cfg_nn, "actor", torch.Generator().manual_seed(0), dtype, "cuda")
        view = net.mlp_view()
        nn_out = {}

        def nn_launch(i):
            nn_out["r"] = ops.rollout_nn(eqp, scheme, x0, dw, T_TOTAL, N, view, want_u=False)
        k4 = max(5, args.steps // 20)
        w4, pl4 = time_launches(nn_launch, k4, 2, world)
        flops = MLP_FLOP_PER_ROW * B * N
        tfs = flops / (pl4 * 1e-3) / 1e12
        x3 = dtype == torch.float32 and ops.MLP_MATH == "x3"
        peak_nn = MFMA_F16_PEAK_TFS / 3 if x3 else (MFMA_F32_PEAK_TFS if dtype == torch.float32
                                                     else MFMA_F64_PEAK_TFS)
        variants["rollout_nn_fused"] = {
            "traj_steps_per_s": world * B * N * k4 / max_over_ranks(w4, world), "avg_launch_ms": pl4,
            "mlp": "20-200-200-200-20", "mlp_math": ops_mlp_math(dtype),
            # the primary peak is the ceiling of the instruction the kernel runs: split-fp16 products
            # (3 fp16 MFMAs per f32 product) -> the fp16 dense peak / 3 in f32-equivalent
            # flops; the exact-f32 kernels -> the f32-input MFMA peak
            "roofline": {"bound": "mfma", "achieved": tfs, "peak": peak_nn, "unit": "TFLOP/s",
                         "frac": tfs / peak_nn,
                         "kernel": "dpac::k_rollout_nn_x3" if x3 else "dpac::k_rollout_nn",
                         "frac_of_f32_mfma_peak": tfs / MFMA_F32_PEAK_TFS,
                         "note": "achieved in f32-equivalent flops (176 kFLOP per trajectory-step)"
                                 + (f"; peak = the fp16 dense MFMA peak / 3 = {peak_nn:.0f} TFLOP/s "
                                    "f32-equivalent, the ceiling of the split-fp16 products this kernel "
                                    "executes; frac_of_f32_mfma_peak compares with the f32-input MFMA "
                                    "(157.3 TFLOP/s), which it does not execute" if x3 else
                                    "; peak = the f32-input MFMA peak")}}
        del rs, nn_out
        torch.cuda.empty_cache()
        if not args.no_train:
            progress("training-iteration variants")
            if world == 1:
                # BASELINE configs[1], [2] (B = 4096 on one GPU), configs[4]'s per-GPU shard of
                # 65536 over 8 GPUs, and the reference's shipped batch (configs/*.json: 2048)
                variants["training_lqr_d20"] = training_variant("lqr_d20", dtype, 2048, iters=30, warmup=5)
                variants["training_lqr_d20_b4096"] = training_variant("lqr_d20", dtype, 4096, iters=20, warmup=5)
                variants["training_ekn_d20_b4096"] = training_variant("ekn_d20", dtype, 4096)
                variants["training_vdp_d20_b8192"] = training_variant("vdp_d20", dtype, 8192, iters=4)
            # BASELINE configs[3]: lqr_var_d20, global batch 16384 split over the ranks, one
            # gradient all-reduce per optimiser step (strong scaling)
            from deeppde_actorcritic_amd.parallel import DataParallel
            par = DataParallel() if world > 1 else None
            v = training_variant("lqr_var_d20", dtype, 16384 // world, world, iters=4, par=par, total=16384)
            v["scaling"] = "strong"
            v["world"] = world
            v["backend"] = torch.distributed.get_backend() if world > 1 else None
            v["process_group_size"] = torch.distributed.get_world_size() if world > 1 else 1
            v["collective"] = ((f"two gradient all-reduces per iteration ({v['backend']}; nccl = RCCL "
                                "over xGMI): V's, then the actor's and G's in one flattened exchange")
                               if world > 1 else None)
            if world > 1:  # the same global batch on ONE GPU: rank 0 alone, inside this job
                del par
                torch.cuda.empty_cache()
                barrier(world)
                one = training_variant("lqr_var_d20", dtype, 16384, 1, iters=4) if rank == 0 else None
                barrier(world)
                one_ms = max_over_ranks(one["ms_per_iteration"] if one else 0.0, world)
            else:
                one_ms = v["ms_per_iteration"]
            v["ms_per_iteration_1gpu"] = one_ms
            v["speedup_vs_1"] = one_ms / v["ms_per_iteration"]
            variants["training_dp_lqr_var_d20"] = v
        out["variants"] = variants
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("cpu_baseline (oracle on the host cores, bounded samples)")
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
