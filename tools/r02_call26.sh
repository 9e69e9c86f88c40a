# Round-2 call 26: staged rollout with 16-byte-aligned slots and deeper rings (4/5/6 chunks of
# 16 steps; default: 4 chunks of 1 KB-aligned slots): bitwise check against k_rollout, then
# the bench's headline (HBM-cold rotation) for each build, default first and last.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 200 bench_default python bench.py --steps 400 --warmup 20 --no-train --no-cpu-baseline
for v in tight4 tight5 tight6; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 test_$v python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "staged and float32"
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 bench_$v python bench.py --steps 400 --warmup 20 --no-train --no-cpu-baseline
done
run 200 bench_default2 python bench.py --steps 400 --warmup 20 --no-train --no-cpu-baseline
