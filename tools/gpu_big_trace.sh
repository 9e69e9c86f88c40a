# lqr_d20 shape at a large batch (B=16384): wall time and a kernel trace.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_train
run 300 train_bench_big python -u tools/train_bench.py --iters 5 --warmup 2 --dtype float32 --batch 16384
run 300 prof_train rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run --output-format csv -- python tools/train_bench.py --iters 2 --warmup 1 --dtype float32 --batch 16384
