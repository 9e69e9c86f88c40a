# round 4 call 21: host submission time of one training iteration
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 300 tb python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_4096 python -u tools/train_bench.py --iters 20 --warmup 3 --batch 4096
