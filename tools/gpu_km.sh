# k-major weight images: full GPU suite, probe and training A/B.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 600 pytest_gpu python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 probe_nn python -u tools/probe_nn.py --B 2048,16384 --N 100 --reps 5
DPAC_WEIGHT_KM=off run 200 probe_nn_off python -u tools/probe_nn.py --B 2048,16384 --N 100 --reps 5
run 300 train_bench32 python -u tools/train_bench.py --iters 20 --dtype float32
DPAC_WEIGHT_KM=off run 300 train_bench32_off python -u tools/train_bench.py --iters 20 --dtype float32
