source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 nn_tests python -m pytest tests/test_gpu_rollout_nn.py -x -q
