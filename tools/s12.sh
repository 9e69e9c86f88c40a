source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
for v in base abl1 abl2 abl5 p32 p32abl1 p32abl5; do
  DPAC_LIB=$PWD/tools/variants/libdpac_$v.so run 200 var_$v python tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100
done
