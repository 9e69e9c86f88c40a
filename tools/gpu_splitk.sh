# Split-K narrow layers: NN rollout tests, probe A/B, training iteration.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 400 nn_tests python -u -m pytest tests/test_gpu_rollout_nn.py tests/test_gpu_models.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 probe_nn python -u tools/probe_nn.py --B 2048,4096 --N 100
DPAC_LIB=$PWD/tools/variants/libdpac_nosplit.so run 200 probe_nn_nosplit python -u tools/probe_nn.py --B 2048,4096 --N 100
run 300 train_bench32 python -u tools/train_bench.py --iters 20 --dtype float32
DPAC_LIB=$PWD/tools/variants/libdpac_nosplit.so run 300 train_bench32_nosplit python -u tools/train_bench.py --iters 20 --dtype float32
