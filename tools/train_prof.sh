source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_train
run 600 train_check python tests/train_check.py --iters 100 --log-freq 25 --runs gpu32,gpu64 --oracle-from profiles/r01_train_check_lqr_d20.json
run 300 train_bench32 python tools/train_bench.py --iters 20 --dtype float32
run 300 train_bench64 python tools/train_bench.py --iters 10 --dtype float64
run 300 prof_train rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run --output-format csv -- python tools/train_bench.py --iters 5 --warmup 1 --dtype float32
