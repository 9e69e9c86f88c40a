# round 4 call 9: timeline after the merged-group PG kernel; per-layer PG kernel times
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_train gpurun_out/prof_pg
run 300 prof_train rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run --output-format csv -- python tools/train_bench.py --iters 3 --warmup 1 --dtype float32
run 60 timeline python tools/iter_timeline.py gpurun_out/prof_train/run_kernel_trace.csv
run 300 prof_pg rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_pg -o run --output-format csv -- python tools/probe_x3.py 204800 x3 --pg
