source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 200 probe_r python -u tools/probe_rollout.py --B 2048,4096,8192 --N 200
DPAC_LIB=$PWD/tools/variants/libdpac_sp2.so run 200 probe_r_sp2 python -u tools/probe_rollout.py --B 2048,4096,8192 --N 200
DPAC_LIB=$PWD/tools/variants/libdpac_sp2.so run 300 kt_sp2 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
