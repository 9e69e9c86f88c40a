#!/usr/bin/env bash
# One round's GPU evidence: GPU tests, smoke(), bench line, rocprofv3 kernel trace of the
# bench (-> the headline's cold / MALL-resident launch split, tools/rocprof_headline.py) and
# of the lqr_d20 training iteration, the two HBM counter passes (FETCH_SIZE, WRITE_SIZE in
# separate runs, as MI355X_MICROARCH.md §HBM prescribes), and the MLP kernels' counters
# (tools/pmc_mlp.sh).  On the GPU box:
#   gpurun -- 'bash tools/profile_round.sh'   then   python tools/collect_profiles.py rNN
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
rm -rf gpurun_out/prof_kt gpurun_out/prof_mall gpurun_out/pmc_it_fetch gpurun_out/pmc_it_write gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/prof_train
if false; then
  run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
  run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
fi
# (bench: tools/gpu_call17.sh)
# the driver's exact command under the profiler (its --stats AverageNs of the headline kernel is
# the mean over exactly the W + K headline launches: the MALL variant runs only with --mall)
run 400 prof_kt rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5
run 60 headline python tools/rocprof_headline.py gpurun_out/prof_kt/run_kernel_trace.csv gpurun_out/prof_kt.log --steps 20 --warmup 5 --stats gpurun_out/prof_kt/run_kernel_stats.csv
# the MALL-resident (one buffer set) variant on its own, for the cold / resident comparison
run 300 prof_mall rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mall -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --mall --no-cpu-baseline --no-train
run 60 headline_mall python tools/rocprof_headline.py gpurun_out/prof_mall/run_kernel_trace.csv gpurun_out/prof_mall.log --steps 20 --warmup 5 --mall
run 300 prof_train rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run --output-format csv -- python tools/train_bench.py --iters 3 --warmup 1 --dtype float32
run 300 pmc_fetch rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-variants
run 300 pmc_write rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-variants
run 900 pmc_mlp bash tools/pmc_mlp.sh
# HBM bytes of one lqr_d20 training iteration (FETCH_SIZE and WRITE_SIZE in separate passes)
run 300 pmc_it_fetch rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_it_fetch -o run --output-format csv -- python tools/train_bench.py --iters 3 --warmup 1 --dtype float32
run 300 pmc_it_write rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_it_write -o run --output-format csv -- python tools/train_bench.py --iters 3 --warmup 1 --dtype float32
run 60 pmc_iteration python tools/pmc_iteration.py gpurun_out/pmc_it_fetch/run_counter_collection.csv gpurun_out/pmc_it_write/run_counter_collection.csv
