source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 300 pytest_mlp python -u -m pytest tests/test_gpu_mlp.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 probe_pg python -u tools/probe_pg.py
run 200 probe_rows python -u tools/probe_rows.py
DPAC_LIB=$PWD/tools/variants/libdpac_rt2.so run 200 probe_rows_rt2 python -u tools/probe_rows.py
run 300 train_bench32 python -u tools/train_bench.py --iters 20 --dtype float32
