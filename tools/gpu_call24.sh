# round 4 call 24: 8-trajectory workgroups for the split-fp16 NN rollout and BPTT (DPAC_NX_ROWS)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 nx_tests python -u -m pytest tests/test_gpu_nn_x3.py tests/test_gpu_rollout_nn.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
for r in 16 8 16 8; do
  run 200 bptt_$r env DPAC_NX_ROWS=$r python -u tools/probe_bptt.py --B 1024,2048,4096 --only fwd,bwd --reps 10
done
for r in 16 8 16 8; do
  run 300 tb_$r env DPAC_NX_ROWS=$r python -u tools/train_bench.py --iters 30 --warmup 5
done
for r in 16 8; do
  run 300 tb4k_$r env DPAC_NX_ROWS=$r python -u tools/train_bench.py --iters 20 --warmup 5 --batch 4096
done
