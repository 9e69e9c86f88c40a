# round 4 call 17: final validation on the round's tree: GPU suite, smoke, the driver's bench command
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --maxfail 20 -rA
run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
run 600 bench python -u bench.py --gpus 1 --steps 20 --warmup 5
