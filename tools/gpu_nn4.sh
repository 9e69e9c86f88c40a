source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 300 nn_tests python -u -m pytest tests/test_gpu_rollout_nn.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 probe_nn python -u tools/probe_nn.py --B 512,1024,2048,4096 --N 100
DPAC_NN_TILE=16 run 200 probe_nn16 python -u tools/probe_nn.py --B 2048,4096 --N 100
