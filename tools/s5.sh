source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
run 300 pmc_sq rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $R/gpurun_out/pmc_sq -o run --output-format csv -- python tools/probe_rollout.py --B 4096 --N 200 --reps 5
run 300 pmc_sq2 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU -d $R/gpurun_out/pmc_sq2 -o run --output-format csv -- python tools/probe_rollout.py --B 4096 --N 200 --reps 5
