# Round-2 call 21: wide layers balanced over the SIMDs (tile 12's K chained over waves 4..7)
# and the next layer's weight prefetch before the epilogue: NN tests, then forward/BPTT
# timing of the default and the three knob variants, then the training iteration.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 300 nn_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rollout_nn.py
run 120 bptt_default python -u tools/probe_bptt.py --B 2048,4096 --N 100 --reps 10
for v in bal0 bal0pre bal1late; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 120 bptt_$v python -u tools/probe_bptt.py --B 2048,4096 --N 100 --reps 10
done
run 200 train_default python -u tools/train_bench.py --iters 20 --batch 2048
DPAC_LIB=$R/tools/variants/libdpac_bal0.so run 200 train_bal0 python -u tools/train_bench.py --iters 20 --batch 2048
