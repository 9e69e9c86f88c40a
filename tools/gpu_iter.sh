# Iteration helper on the GPU box: tests given in $TESTS (default: all gpu), then train_bench.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 600 pytest_gpu python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 train_bench32 python -u tools/train_bench.py --iters 20 --dtype float32
