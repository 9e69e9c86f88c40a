# round 4 call 10: the three-stage ring PG kernel (k_param_grads_x3p)
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_pg
run 300 pg_tests python -u -m pytest tests/test_gpu_mlp.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -rA -x
run 300 pg_p python -u tools/probe_x3.py 204800 x3 --pg
run 300 pg_w env DPAC_PGX_W=1 python -u tools/probe_x3.py 204800 x3 --pg
run 300 prof_pg rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_pg -o run --output-format csv -- python tools/probe_x3.py 204800 x3 --pg
run 300 tb_p python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_w env DPAC_PGX_W=1 python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_p4096 python -u tools/train_bench.py --iters 20 --warmup 3 --batch 4096
run 300 tb_early env DPAC_GBACK=early python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_noguard env DPAC_X3_GUARD=0 python -u tools/train_bench.py --iters 30 --warmup 5
run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --maxfail 20 -rA
