# Round-2 call 3: the stager/writer BPTT kernel (k_rollout_nn_bwd2): its bitwise test and the
# model tests, timings against k_rollout_nn_bwd, the training iteration; the cold-cache
# rollout variants (ring depth, non-temporal hints).
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 300 nn_tests python -u -m pytest tests/test_gpu_rollout_nn.py tests/test_gpu_models.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 probe_bptt2 python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only bwd
DPAC_BPTT=1 run 200 probe_bptt1 python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only bwd
run 200 train_bench python -u tools/train_bench.py --iters 20 --dtype float32
run 120 roll_base python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100 --sets 5
for v in ring64 ring128 ntdw ntx ntboth; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 120 roll_$v python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100 --sets 5
done
