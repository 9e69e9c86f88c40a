# bench.py at N=1 (with the DP variant) and a 2-rank rehearsal of the N>1 path on one GPU (gloo).
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 300 bench1 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline
DPAC_DIST_BACKEND=gloo run 300 bench2_gloo python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3
