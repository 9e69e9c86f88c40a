# Round-2 call 6 (fresh container, rebuilt tree): the BPTT kernels timed (bwd2 default vs
# k_rollout_nn_bwd), the training iteration, then the round's evidence (profile_round.sh).
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 300 nn_tests python -u -m pytest tests/test_gpu_rollout_nn.py tests/test_gpu_models.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 probe_def python -u tools/probe_bptt.py --B 2048,4096 --N 100
DPAC_BPTT=1 run 200 probe_bwd1 python -u tools/probe_bptt.py --B 2048 --N 100 --only bwd
run 200 train_bench python -u tools/train_bench.py --iters 20 --dtype float32
run 200 train_bench4096 python -u tools/train_bench.py --iters 20 --dtype float32 --batch 4096
bash tools/profile_round.sh
