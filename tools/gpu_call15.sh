# round 4 call 15: V's parameter gradients (3B rows): chunking and the one-launch f32 path
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 300 tb_base python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_small env DPAC_PG_SMALL=16384 python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_small64 env DPAC_PG_SMALL=16384 DPAC_PG_MIN_ROWS=64 python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_small32 env DPAC_PG_SMALL=16384 DPAC_PG_MIN_ROWS=32 python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_min64 env DPAC_PG_MIN_ROWS=64 python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_base2 python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_small_4096 env DPAC_PG_SMALL=16384 python -u tools/train_bench.py --iters 20 --warmup 3 --batch 4096
run 300 tb_base_4096 python -u tools/train_bench.py --iters 20 --warmup 3 --batch 4096
