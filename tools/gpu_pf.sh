source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 200 probe_nn_pf8 python -u tools/probe_nn.py --B 2048,16384 --N 100 --reps 5
for v in pf4 pf12 pf16; do
  DPAC_LIB=$PWD/tools/variants/libdpac_$v.so run 200 probe_nn_$v python -u tools/probe_nn.py --B 2048,16384 --N 100 --reps 5
done
