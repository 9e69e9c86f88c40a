#!/usr/bin/env bash
# PMC passes (one counter set per run, MI355X_MICROARCH.md §rocprofv3 PMC slots) over the
# split-fp16 MLP kernels at lqr_d20's shape: the actor's fused forward / BPTT / parameter
# gradients (tools/probe_bptt.py, B = 2048, N = 100) and the critic's row kernels over
# 204 800 rows (tools/probe_x3.py; the row backward with the forward's sign bits is
# k_mlp_rows_bwd_x3<true>, the z-reading one <false>), then tools/pmc_summary.py.
#   gpurun -- 'bash tools/pmc_mlp.sh'  ->  gpurun_out/pmc_mlp/summary.json
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_mlp
rm -rf gpurun_out/pmc_mlp/pmc_*
sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
      "FETCH_SIZE"
      "WRITE_SIZE")
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmc_mlp/pmc_nn_$i -o run --output-format csv -- \
    python tools/probe_bptt.py --B 2048 --reps 3 > gpurun_out/pmc_mlp/pmc_nn_$i.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmc_mlp/pmc_rows_$i -o run --output-format csv -- \
    python tools/probe_x3.py 204800 x3 > gpurun_out/pmc_mlp/pmc_rows_$i.log 2>&1 || exit 1
done
python tools/pmc_summary.py gpurun_out/pmc_mlp gpurun_out/pmc_mlp/summary.json \
  --kernels "k_rollout_nn_x3<,k_rollout_nn_bwd_x3<,k_param_grads_x3w<13,k_param_grads_x3w<2,k_mlp_rows_fwd_x3,k_mlp_rows_bwd_x3<true,k_mlp_rows_bwd_x3<false" \
  --note "lqr_d20 fp32 split-fp16 kernels: actor B=2048 N=100 (probe_bptt), critic rows 204800 (probe_x3)"
