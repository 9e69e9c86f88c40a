# round 4 call 20: the split-fp16 row backward over 32-row workgroups (no spills), the forward at 64
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 x3_tests python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_td_fused.py tests/test_gpu_x3_guard.py tests/test_gpu_fp32_production.py -q -p no:cacheprovider --timeout 300 --timeout-method thread -x
run 300 rows python -u tools/probe_x3.py 204800 x3
run 300 tb python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_4096 python -u tools/train_bench.py --iters 20 --warmup 3 --batch 4096
run 300 tb2 python -u tools/train_bench.py --iters 30 --warmup 5
