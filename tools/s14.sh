source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 200 diag_new python tools/diag_fp32.py VDP 20 naive cost
run 200 diag_new4 python tools/diag_fp32.py VDP 10 naive cost
