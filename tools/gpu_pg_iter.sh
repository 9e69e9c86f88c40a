source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_pg*
run 300 pytest_mlp python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_models.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 prof_pg_new rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_pg_new -o run --output-format csv -- python -u tools/probe_pg.py
run 300 train_bench32 python -u tools/train_bench.py --iters 20 --dtype float32
