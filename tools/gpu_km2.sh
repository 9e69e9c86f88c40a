source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_train
run 600 pytest_gpu python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 probe_rows python -u tools/probe_rows.py
DPAC_WEIGHT_KM=off run 200 probe_rows_off python -u tools/probe_rows.py
run 300 train_bench32 python -u tools/train_bench.py --iters 20 --dtype float32
run 300 prof_train rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_train -o run --output-format csv -- python tools/train_bench.py --iters 3 --warmup 1 --dtype float32
