# round 4 call 16: row kernels with adjacent feature tiles per wave (DPAC_X3_ADJ=1 variant)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 adj_tests env DPAC_LIB=tools/variants/libdpac_x3adj.so python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_td_fused.py tests/test_gpu_x3_guard.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
run 300 rows_base python -u tools/probe_x3.py 204800 x3
run 300 rows_adj env DPAC_LIB=tools/variants/libdpac_x3adj.so python -u tools/probe_x3.py 204800 x3
run 300 tb_base python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_adj env DPAC_LIB=tools/variants/libdpac_x3adj.so python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_base2 python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_adj2 env DPAC_LIB=tools/variants/libdpac_x3adj.so python -u tools/train_bench.py --iters 30 --warmup 5
