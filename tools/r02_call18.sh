# Round-2 call 18: the LDS-staged analytic rollout (k_rollout_staged): bitwise test against
# k_rollout, all kernel tests, timings cold / MALL-resident, staged vs direct.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 300 kernel_tests python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 120 roll_staged_cold python -u tools/probe_rollout.py --B 4096,8192,16384 --N 200 --reps 100 --sets 5
run 120 roll_staged_mall python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100 --sets 1
DPAC_ROLLOUT_STAGED=0 run 120 roll_direct_cold python -u tools/probe_rollout.py --B 4096,8192,16384 --N 200 --reps 100 --sets 5
run 120 roll_staged_f64 python -u tools/probe_rollout.py --dtype f64 --B 4096 --N 200 --reps 50 --sets 5
