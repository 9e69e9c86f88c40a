source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 nn_tests python -m pytest tests/test_gpu_rollout_nn.py tests/test_gpu_models.py tests/test_main.py -x -q
run 300 train_bench32 python tools/train_bench.py --iters 20 --dtype float32
run 300 train_bench64 python tools/train_bench.py --iters 10 --dtype float64
