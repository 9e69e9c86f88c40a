source tools/gpu_steps.sh
for v in xcd xcd_nostore; do
  DPAC_LIB=$PWD/tools/variants/libdpac_$v.so run 200 var_$v python tools/probe_rollout.py --B 2048,4096,8192,16384 --N 200 --reps 100
done
