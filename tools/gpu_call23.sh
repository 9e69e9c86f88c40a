# round 4 call 23: the staged rollout's dw read PD steps ahead of use (DPAC_ST_PD variants)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 300 pd2_tests env DPAC_LIB=tools/variants/libdpac_pd2.so python -u -m pytest tests/test_gpu_kernels.py -k "staged or rollout" -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
run 300 pd4_tests env DPAC_LIB=tools/variants/libdpac_pd4.so python -u -m pytest tests/test_gpu_kernels.py -k "staged or rollout" -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
for v in pd1 pd2 pd4 pd1 pd2 pd4; do
  run 200 probe_$v env DPAC_LIB=tools/variants/libdpac_$v.so python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 200 --sets 5
  run 200 probem_$v env DPAC_LIB=tools/variants/libdpac_$v.so python -u tools/probe_rollout.py --B 4096 --N 200 --reps 200 --sets 1
done
