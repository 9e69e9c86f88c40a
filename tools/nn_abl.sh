source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 200 nn_base python tools/probe_nn.py --B 256,2048,8192
DPAC_LIB=$PWD/tools/variants/libdpac_nnabl1.so run 200 nn_abl1 python tools/probe_nn.py --B 256,2048,8192
run 200 nn_f64 python tools/probe_nn.py --B 2048 --dtype f64 --reps 5
run 600 nn_tests python -m pytest tests/test_gpu_rollout_nn.py tests/test_gpu_models.py -x -q
run 300 train_bench32 python tools/train_bench.py --iters 20 --dtype float32
