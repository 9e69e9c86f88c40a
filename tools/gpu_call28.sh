# round 4 call 28: the split-fp16 row forward at 48-row workgroups (DPAC_X3_RT=3: 230 VGPRs, no spill; 4 = 64 rows spills 76 B)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 rt3_tests env DPAC_LIB=tools/variants/libdpac_rt3.so python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_td_fused.py tests/test_gpu_x3_guard.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
for v in base rt3 base rt3; do
  if [ $v = base ]; then L=""; else L="DPAC_LIB=tools/variants/libdpac_$v.so"; fi
  run 300 rows_$v env $L python -u tools/probe_x3.py 204800 x3
done
for v in base rt3 base rt3; do
  if [ $v = base ]; then L=""; else L="DPAC_LIB=tools/variants/libdpac_$v.so"; fi
  run 300 tb_$v env $L python -u tools/train_bench.py --iters 30 --warmup 5
done
