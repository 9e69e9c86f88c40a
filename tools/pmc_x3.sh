#!/usr/bin/env bash
# PMC passes (one counter set per run) over the split-fp16 row kernels (tools/probe_x3.py x3).
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_*
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 100 rocprofv3 --pmc $set -d gpurun_out/pmc_x3_$i -o run --output-format csv -- python tools/probe_x3.py 204800 x3 > gpurun_out/pmc_x3_$i.log 2>&1 || exit 1
done
python tools/pmc_summary.py gpurun_out gpurun_out/pmcx3_summary.json --kernels k_mlp_rows_fwd_x3,k_mlp_rows_bwd_x3 || true
