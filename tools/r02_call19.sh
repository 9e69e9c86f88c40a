# Round-2 call 19: the tile-contiguous sign-bit mask ([N][B/16][mh][16]): NN tests, BPTT
# timing with the mask on/off, and the training iteration.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 400 nn_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rollout_nn.py
run 120 bptt_mask python -u tools/probe_bptt.py --B 2048,4096 --N 100 --reps 10
DPAC_MASK_BPTT=0 run 120 bptt_nomask python -u tools/probe_bptt.py --B 2048,4096 --N 100 --reps 10
run 200 train_mask python -u tools/train_bench.py --iters 20 --batch 2048
DPAC_MASK_BPTT=0 run 200 train_nomask python -u tools/train_bench.py --iters 20 --batch 2048
