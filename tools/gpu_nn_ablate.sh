source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
DPAC_NN_TILE=16 run 200 probe_nn16 python -u tools/probe_nn.py --B 2048 --N 100
DPAC_NN_TILE=16 DPAC_LIB=$PWD/tools/variants/libdpac_abl1.so run 200 probe_abl1 python -u tools/probe_nn.py --B 2048 --N 100
DPAC_NN_TILE=16 DPAC_LIB=$PWD/tools/variants/libdpac_abl2.so run 200 probe_abl2 python -u tools/probe_nn.py --B 2048 --N 100
