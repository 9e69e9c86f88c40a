# Round-2 call 9: the full 50 000-iteration lqr_d20 run in float64 (the reference's
# precision), same seeds and increments as the fp32 run of call 7.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
mkdir -p gpurun_out/r02c9
run 1120 full_fp64 python -u tests/train_check.py --iters 50000 --log-freq 100 --batch 2048 --valid 2048 --runs gpu64 --sampler device --out gpurun_out/r02c9/full_lqr_d20_fp64.json
