# round 4 call 12: the merged-group kernel for the input and narrow output layers too
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_pg
run 300 pg_tests python -u -m pytest tests/test_gpu_mlp.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -rA -x
run 300 pg_w python -u tools/probe_x3.py 204800 x3 --pg
run 300 prof_pg rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_pg -o run --output-format csv -- python tools/probe_x3.py 204800 x3 --pg
run 300 tb_w python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_w4096 python -u tools/train_bench.py --iters 20 --warmup 3 --batch 4096
run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --maxfail 20 -rA
