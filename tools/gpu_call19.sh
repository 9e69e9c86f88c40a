# round 4 call 19: split-fp16 row kernels over 32-row workgroups (DPAC_X3_RT=2: no register spills)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 rt2_tests env DPAC_LIB=tools/variants/libdpac_rt2.so python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_td_fused.py tests/test_gpu_x3_guard.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
run 300 rows_base python -u tools/probe_x3.py 204800 x3
run 300 rows_rt2 env DPAC_LIB=tools/variants/libdpac_rt2.so python -u tools/probe_x3.py 204800 x3
run 300 tb_base python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_rt2 env DPAC_LIB=tools/variants/libdpac_rt2.so python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_base_4096 python -u tools/train_bench.py --iters 20 --warmup 3 --batch 4096
run 300 tb_rt2_4096 env DPAC_LIB=tools/variants/libdpac_rt2.so python -u tools/train_bench.py --iters 20 --warmup 3 --batch 4096
