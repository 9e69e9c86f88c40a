# Round-2 call 23: the critic's G network with the TD1 dot fused.
# New bitwise tests, then the whole GPU suite and smoke on the final library, then the
# lqr_d20 training iteration with the fused and the split critic front (B = 2048, 4096),
# and a kernel trace of the fused iteration.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
rm -rf gpurun_out/prof_train_fused
run 300 td_fused_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_td_fused.py tests/test_abi.py
run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
for b in 2048 4096; do
  DPAC_CRITIC_TD1=split run 200 train_split_$b python -u tools/train_bench.py --iters 20 --batch $b
  DPAC_CRITIC_TD1=fused run 200 train_fused_$b python -u tools/train_bench.py --iters 20 --batch $b
done
run 300 prof_train_fused rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train_fused -o run --output-format csv -- python tools/train_bench.py --iters 3 --warmup 1 --dtype float32
