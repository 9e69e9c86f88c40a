# Model-level GPU tests, the lqr_d20 training iteration, and its kernel trace.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_train
run 400 pytest_models python -u -m pytest ${TESTS:-tests/test_gpu_models.py} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 train_bench32 python -u tools/train_bench.py --iters 20 --dtype float32
run 300 prof_train rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run --output-format csv -- python tools/train_bench.py --iters 3 --warmup 1 --dtype float32
