# Round-2 call 24: fused TD1 G forward with sigma*dw prefetched at kernel start:
# bitwise tests, split-vs-fused kernel probe, training iteration both modes.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 300 td_fused_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_td_fused.py tests/test_gpu_models.py
run 200 probe_td_fused python -u tools/probe_td_fused.py 2048 4096
for b in 2048 4096; do
  DPAC_CRITIC_TD1=split run 200 train_split_$b python -u tools/train_bench.py --iters 30 --batch $b
  DPAC_CRITIC_TD1=fused run 200 train_fused_$b python -u tools/train_bench.py --iters 30 --batch $b
done
DPAC_CRITIC_TD1=split run 200 train_split_2048b python -u tools/train_bench.py --iters 30 --batch 2048
DPAC_CRITIC_TD1=fused run 200 train_fused_2048b python -u tools/train_bench.py --iters 30 --batch 2048
