source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 120 lanes_base python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100
DPAC_LIB=$PWD/tools/variants/libdpac_cap8.so run 120 lanes_cap8 python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100
DPAC_LIB=$PWD/tools/variants/libdpac_cap4.so run 120 lanes_cap4 python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100
DPAC_LIB=$PWD/tools/variants/libdpac_cap8.so run 300 lanes_cap8_tests python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
