# Round-2 call 25: float64 rollout on the LDS-staged kernel (3-chunk ring of 16-byte-aligned
# slots): the kernel tests (staged == k_rollout bitwise, both dtypes), smoke, the bench line
# (its rollout_f64 variant), and a kernel trace of the bench.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
rm -rf gpurun_out/prof_kt25
run 300 kernel_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py
run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
run 300 bench python bench.py --steps 200 --warmup 20 --no-train
DPAC_ROLLOUT_STAGED=0 run 300 bench_unstaged python bench.py --steps 200 --warmup 20 --no-train --no-cpu-baseline
run 300 prof_kt25 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt25 -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-train
