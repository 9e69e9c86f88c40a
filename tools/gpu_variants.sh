source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 200 probe_nn python -u tools/probe_nn.py --B 2048,4096 --N 100
DPAC_LIB=$PWD/tools/variants/libdpac_w8.so run 200 probe_nn_w8 python -u tools/probe_nn.py --B 2048,4096 --N 100
run 200 probe_rows python -u tools/probe_rows.py
DPAC_LIB=$PWD/tools/variants/libdpac_rt1.so run 200 probe_rows_rt1 python -u tools/probe_rows.py
DPAC_LIB=$PWD/tools/variants/libdpac_w8.so run 300 nn_tests_w8 python -u -m pytest tests/test_gpu_rollout_nn.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
