# round 4 call 30: parameter-gradient row chunks per launch (DPAC_PG_CHUNKS 128 / 512 vs the shipped 256)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 ch128_tests env DPAC_LIB=tools/variants/libdpac_ch128.so python -u -m pytest tests/test_gpu_mlp.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -x -k "param_grads"
for v in base ch128 ch512 base ch128 ch512; do
  if [ $v = base ]; then L=""; else L="DPAC_LIB=tools/variants/libdpac_$v.so"; fi
  run 300 tb_$v env $L python -u tools/train_bench.py --iters 30 --warmup 5
done
for v in base ch128 ch512; do
  if [ $v = base ]; then L=""; else L="DPAC_LIB=tools/variants/libdpac_$v.so"; fi
  run 300 tb4k_$v env $L python -u tools/train_bench.py --iters 20 --warmup 5 --batch 4096
done
