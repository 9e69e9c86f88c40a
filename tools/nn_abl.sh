source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_train
run 900 gputests python -m pytest tests -m gpu -x -q
run 600 train_check python tools/train_check.py --iters 100 --log-freq 25 --runs gpu32,gpu64 --oracle-from profiles/r01_train_check_lqr_d20.json
run 300 prof_train rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run --output-format csv -- python tools/train_bench.py --iters 10 --warmup 2 --dtype float32
