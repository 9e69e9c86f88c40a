# Round-2 call 7: the rollout's prefetch ring depth and cache-policy variants in the
# cold-cache regime (5 rotating buffer sets, as bench.py times it); the MLP weight-stream
# ablation; the long lqr_d20 accuracy runs (fp32 vs fp64 over 5000 iterations at B=4096,
# and the full 50 000-iteration fp32 run at the reference's batch).
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
mkdir -p gpurun_out/r02c7
run 120 roll_base python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100 --sets 5
for v in ring64 ring128 ntdw ntx r128nt; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 120 roll_$v python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100 --sets 5
done
DPAC_LIB=$R/tools/variants/libdpac_nnw.so run 200 probe_nnw python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only fwd,bwd
run 900 long_b4096 python -u tests/train_check.py --iters 5000 --log-freq 100 --batch 4096 --valid 4096 --runs gpu32,gpu64 --sampler device --out gpurun_out/r02c7/long_lqr_d20_b4096.json
run 900 full_fp32 python -u tests/train_check.py --iters 50000 --log-freq 100 --batch 2048 --valid 2048 --runs gpu32 --sampler device --out gpurun_out/r02c7/full_lqr_d20_fp32.json
