# Round-2 call 17: what bounds the step-major rollout in the cold-cache regime: ablations
# (1 no stores, 2 no dw loads, 3 no dt/coef stores, 4 no x stores), 5 rotating sets.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 120 roll_base python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100 --sets 5
for v in abl1 abl2 abl3 abl4; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 120 roll_$v python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100 --sets 5
done
