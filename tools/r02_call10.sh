# Round-2 call 10: the actor-shape fast path (resident narrow layers, wide-layer weight
# prefetch): bitwise tests, timings against the generic path, phase trace, iteration.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 300 nn_tests python -u -m pytest tests/test_gpu_rollout_nn.py tests/test_gpu_models.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 probe_fast python -u tools/probe_bptt.py --B 2048,4096 --N 100
DPAC_NN_FAST=0 run 200 probe_generic python -u tools/probe_bptt.py --B 2048 --N 100 --only fwd,bwd
DPAC_LIB=$R/tools/variants/libdpac_trace.so run 200 trace python -u tools/probe_trace.py --B 2048 --N 100
run 200 train_bench python -u tools/train_bench.py --iters 20 --dtype float32
run 200 train_bench4096 python -u tools/train_bench.py --iters 20 --dtype float32 --batch 4096
