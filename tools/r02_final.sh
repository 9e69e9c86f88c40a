# Round-2 final evidence (part 1): GPU tests, smoke, bench line, the actor-step kernel
# probe, the training iteration, rocprofv3 kernel traces of the bench and of the iteration,
# and the two HBM counter passes over the bench's headline rollout.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
rm -rf gpurun_out/prof_kt gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/prof_train
run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
run 300 bench python bench.py --steps 200 --warmup 20
run 200 probe_bptt python -u tools/probe_bptt.py --B 2048,4096 --N 100
run 300 train2k python -u tools/train_bench.py --iters 20 --batch 2048
run 300 train4k python -u tools/train_bench.py --iters 20 --batch 4096
run 200 probe_td_fused python -u tools/probe_td_fused.py 2048 4096
run 300 prof_kt rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-train
run 300 prof_train rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run --output-format csv -- python tools/train_bench.py --iters 3 --warmup 1 --dtype float32
run 300 pmc_fetch rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-variants
run 300 pmc_write rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-variants
