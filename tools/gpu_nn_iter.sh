# NN rollout / model tests, the fused-rollout probe and the training iteration.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 400 nn_tests python -u -m pytest tests/test_gpu_rollout_nn.py tests/test_gpu_models.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 probe_nn python -u tools/probe_nn.py --B 2048,16384 --N 100 --reps 5
run 300 train_bench32 python -u tools/train_bench.py --iters 30 --dtype float32
