# Round-2 call 31: closing pass on the final library (row-MLP LDS stride 264): the whole GPU
# suite, smoke, the bench line, the training iteration.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
run 300 bench python bench.py --steps 200 --warmup 20
run 200 rows python -u tools/probe_rows.py 204800
