source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
run 300 probe python tools/probe_rollout.py --B 1024,2048,4096,8192,16384,32768 --N 200
run 300 probe_n python tools/probe_rollout.py --B 4096 --N 50,100,200,400
run 300 probe_f64 python tools/probe_rollout.py --B 4096,16384 --N 200 --dtype f64
run 300 pmc_sq rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d $R/gpurun_out/pmc_sq -o run --output-format csv -- python tools/probe_rollout.py --B 4096 --N 200 --reps 5
run 300 pmc_sq2 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR -d $R/gpurun_out/pmc_sq2 -o run --output-format csv -- python tools/probe_rollout.py --B 4096 --N 200 --reps 5
