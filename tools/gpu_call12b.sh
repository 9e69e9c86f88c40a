# round 4 call 12b: attribution of the fp32 LQR critic gradient error (x3 vs exact-f32 MLP products)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 300 attr_x3 python -u tools/grad_attribution.py LQR
run 300 attr_f32 env DPAC_MLP_MATH=f32 python -u tools/grad_attribution.py LQR
