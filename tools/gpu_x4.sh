source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 200 probe_nn_base python -u tools/probe_nn.py --B 2048,16384 --N 100 --reps 5
DPAC_LIB=$PWD/tools/variants/libdpac_x4.so run 200 probe_nn_x4 python -u tools/probe_nn.py --B 2048,16384 --N 100 --reps 5
