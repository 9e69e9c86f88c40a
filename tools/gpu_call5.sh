source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 guard python -u -m pytest tests/test_gpu_x3_guard.py -q -p no:cacheprovider --timeout 300 --timeout-method thread -rA
run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --maxfail 20 -rA
run 300 rows python -u tools/probe_x3.py
run 300 tb_guard python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_noguard env DPAC_X3_GUARD=0 python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_4096 python -u tools/train_bench.py --iters 20 --warmup 3 --batch 4096
