# round 4 call 22: the row backward's z loads issued before the K loop (DPAC_X3_ZPRE=1 variant)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 zpre_tests env DPAC_LIB=tools/variants/libdpac_zpre.so python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_td_fused.py tests/test_gpu_x3_guard.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
run 300 rows_base python -u tools/probe_x3.py 204800 x3
run 300 rows_zpre env DPAC_LIB=tools/variants/libdpac_zpre.so python -u tools/probe_x3.py 204800 x3
run 300 tb_base python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_zpre env DPAC_LIB=tools/variants/libdpac_zpre.so python -u tools/train_bench.py --iters 30 --warmup 5
