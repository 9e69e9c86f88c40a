source tools/gpu_steps.sh
run 200 copybw python tools/copy_bw.py
for v in base nostore nodtc nox; do
  DPAC_LIB=$PWD/tools/variants/libdpac_$v.so run 200 var_$v python tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100
done
