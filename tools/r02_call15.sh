# Round-2 call 15: the reference-layout rollout (dpac_rollout_fwd_bdn): bitwise test
# against the step-major kernel, kernel tests, timings cold/MALL, bench.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 300 kernel_tests python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for L in bdn step; do
  run 120 roll_${L}_cold python -u tools/probe_rollout.py --layout $L --B 4096,16384 --N 200 --reps 100 --sets 5
  run 120 roll_${L}_mall python -u tools/probe_rollout.py --layout $L --B 4096,16384 --N 200 --reps 100 --sets 1
done
run 120 roll_bdn_f64 python -u tools/probe_rollout.py --layout bdn --dtype f64 --B 4096 --N 200 --reps 50 --sets 5
run 400 bench python bench.py --no-cpu-baseline --no-train
