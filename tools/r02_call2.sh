# Round-2 call 2: the new GPU tests (sharding, d=20 training, B=4096 vectors, 2-rank DP),
# the 2-rank DP equality script as a top-level torchrun, the lane-split builds' tests
# (flush invariant fixed) and timings, the MLP-kernel timing variants, the new bench.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
mkdir -p gpurun_out/r02c2
run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf
run 200 dp_equality python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tests/dp_equality.py --out gpurun_out/r02c2/dp_equality.json
for v in cap8 cap4; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 300 lanes_${v}_tests python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
done
run 120 lanes_base python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100
for v in cap8 cap4; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 120 lanes_$v python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100
done
run 200 probe_bptt python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only fwd,bwd
for v in pg3 pg4 w12 w16; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 probe_bptt_$v python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only fwd,bwd
done
run 600 bench python bench.py
