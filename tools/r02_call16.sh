# Round-2 call 16: why the reference-layout rollout is slow (ablations, cache counters) and
# where it differs from the step-major kernel (LQR_var d=10, N=101).
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 120 debug_bdn python -u tools/debug_bdn.py
run 120 roll_bdn python -u tools/probe_rollout.py --layout bdn --B 4096 --N 200 --reps 50 --sets 5
for v in abl2 abl4; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 120 roll_bdn_$v python -u tools/probe_rollout.py --layout bdn --B 4096 --N 200 --reps 50 --sets 5
done
run 120 pmc_tcp timeout -s KILL 100 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum -d $R/gpurun_out/pmc_tcp -o run --output-format csv -- python tools/probe_rollout.py --layout bdn --B 4096 --N 200 --reps 3 --sets 1
run 120 pmc_tcp_step timeout -s KILL 100 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum -d $R/gpurun_out/pmc_tcp_step -o run --output-format csv -- python tools/probe_rollout.py --layout step --B 4096 --N 200 --reps 3 --sets 1
