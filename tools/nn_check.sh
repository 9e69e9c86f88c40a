source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 nn_tests python -m pytest tests/test_gpu_rollout_nn.py -x -q
run 900 gputests python -m pytest tests -m gpu -x -q
run 300 train_bench32 python tools/train_bench.py --iters 20 --dtype float32
