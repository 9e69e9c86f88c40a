#!/usr/bin/env bash
# Seed spread of the north-star accuracy bar: full 50 000-iteration
# lqr_d20 runs (configs/lqr_d20.json: B = 2048, N = 100, 3x200 MLPs, TD1, adaptive) on the
# production path, one process per (dtype, seed), run concurrently on the one GPU.
#   bash tools/seed_spread.sh "gpu32:101 gpu32:202 gpu32:303 gpu64:101"
# -> gpurun_out/seed_<run>_<seed>.json (tests/train_check.py format); the device sampler draws
# the increments in float64 for both dtypes, so a (seed) pair sees the same noise.
set -u
mkdir -p gpurun_out
pids=()
for spec in $1; do
  run=${spec%%:*}; seed=${spec##*:}
  timeout -k 10 1150 python -u tests/train_check.py --iters 50000 --log-freq 100 --runs "$run" \
    --sampler device --seed "$seed" --data-seed "$seed" \
    --out "gpurun_out/seed_${run}_${seed}.json" > "gpurun_out/seed_${run}_${seed}.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
tail -n 2 gpurun_out/seed_*.log
exit $rc
