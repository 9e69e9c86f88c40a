# Round-2 call 28: the strong-scaling BASELINE configs on one GPU, at their global batch and
# at their 8-GPU per-rank shard (lqr_var_d20: 16384 / 2048; vdp_d20: 65536 / 8192).
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 200 lqrvar_2048 python -u tools/train_bench.py --config lqr_var_d20 --iters 20 --batch 2048
run 300 lqrvar_16384 python -u tools/train_bench.py --config lqr_var_d20 --iters 10 --batch 16384
run 200 vdp_8192 python -u tools/train_bench.py --config vdp_d20 --iters 10 --batch 8192
run 400 vdp_65536 python -u tools/train_bench.py --config vdp_d20 --iters 5 --warmup 2 --batch 65536
