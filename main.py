"""Drop-in replacement for the reference's main.py (main.py:1-70).

    python main.py --config_path=configs/lqr_d5.json [--exp_name=NAME]

Same flags, same ./logs outputs: {exp}_config.json, {exp}_{sample}_{scheme}_{TD}_{train}.csv
(history, 9 columns) and ..._hist.csv (x, y_NN, y_true, Z_NN, z_true).  Extra
optional flags: --seed, --sampler {device,host}, --dtype {float32,float64}.
Multi-GPU: launch with torch.distributed.run; every rank trains its shard of
each batch and gradients are all-reduced (RCCL).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys

import numpy as np


def parse_args(argv):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--config_path", default="configs/lqr_d5.json", help="The path to load json file.")
    p.add_argument("--exp_name", default=None,
                   help="The name of numerical experiments, prefix for logging")
    p.add_argument("--log_dir", default="./logs")
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--sampler", choices=["device", "host"], default=None)
    p.add_argument("--dtype", choices=["float32", "float64"], default=None,
                   help="override net_config.dtype")
    p.add_argument("--num_iterations", type=int, default=None, help="override net_config.num_iterations")
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(sys.argv[1:] if argv is None else argv)
    import torch
    import deeppde_actorcritic_amd as dpac
    from deeppde_actorcritic_amd import equation as eqn
    from deeppde_actorcritic_amd.parallel import DataParallel

    exp_name = args.exp_name or os.path.splitext(os.path.basename(args.config_path))[0]
    config = dpac.load_config(args.config_path)
    if args.dtype:
        config.net_config.dtype = args.dtype
    if args.num_iterations is not None:
        config.net_config.num_iterations = args.num_iterations

    par = None
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
        par = DataParallel()
    rank = par.rank if par else 0

    bsde = getattr(eqn, config.eqn_config.eqn_name)(config.eqn_config)  # main.py:34
    dpac.set_floatx(config.net_config.dtype)                              # main.py:35
    dim, control_dim = config.eqn_config.dim, config.eqn_config.control_dim
    tc = config.train_config
    path_prefix = os.path.join(args.log_dir, exp_name)
    if rank == 0:
        os.makedirs(args.log_dir, exist_ok=True)
        with open(f"{path_prefix}_config.json", "w") as outfile:  # main.py:46-49
            json.dump(dpac.config.unmunchify(config), outfile, indent=2)
    logging.basicConfig(format="%(levelname)-6s %(message)s", level=logging.INFO)
    logging.info("Begin to solve %s " % config.eqn_config.eqn_name)
    solver = dpac.ActorCriticSolver(config, bsde, seed=args.seed, sampler=args.sampler, parallel=par)
    training_history, x, y, true_y, z, true_z, grad_y = solver.train()
    if rank == 0:  # main.py:58-68
        char = tc.sample_type + "_" + tc.scheme + "_" + tc.TD_type + "_" + tc.train
        np.savetxt(f"{path_prefix}_{char}.csv", training_history,
                   fmt=["%d", "%.5e", "%.5e", "%.5e", "%.5e", "%.5e", "%.5e", "%.5e", "%d"],
                   delimiter=",",
                   header="step, loss_critic, loss_actor, err_value, error_value_infty, err_control, "
                          "err_value_grad,error_cost2, elapsed_time",
                   comments="")
        figure_data = np.concatenate([x, y, true_y, z, true_z], axis=1)
        head = ("x,") * dim + "y_NN,y_true," + ("Z_NN,") * control_dim + "z_true" + (",z_true") * (control_dim - 1)
        np.savetxt(f"{path_prefix}_{char}_hist.csv", figure_data, delimiter=",", header=head, comments="")
    if par is not None:
        import torch.distributed as dist
        dist.destroy_process_group()
    return training_history


if __name__ == "__main__":
    main()
