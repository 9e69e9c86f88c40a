# Round-2 call 27: closing pass on the final library: the whole GPU suite, smoke, the bench
# line (with the float64 rollout on the staged kernel), and its kernel trace.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
rm -rf gpurun_out/prof_kt
run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
run 300 bench python bench.py --steps 200 --warmup 20
run 300 prof_kt rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-train
