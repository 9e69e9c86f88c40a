source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
for v in kb4 kb8 kb12 kb16; do
  DPAC_LIB=$PWD/tools/variants/libdpac_$v.so run 200 var_$v python tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100
done
