source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 200 probe_nn python -u tools/probe_nn.py --B 2048,4096 --N 100
for v in abl1 abl2; do
  DPAC_LIB=$PWD/tools/variants/libdpac_$v.so run 200 probe_nn_$v python -u tools/probe_nn.py --B 2048,4096 --N 100
done
