# Round-2 call 29: PMC passes (one counter set per run) over the final MLP kernels: the actor's
# fused forward, BPTT and parameter gradients (tools/probe_bptt.py, B=2048) and the critic's
# G network with the TD1 dot fused (tools/probe_td_fused.py, B=2048).
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
rm -rf gpurun_out/r02c29
mkdir -p gpurun_out/r02c29/bptt gpurun_out/r02c29/td
rocprofv3 -L > gpurun_out/r02c29/counters.txt 2>&1 || true
have() { grep -q "\b$1\b" gpurun_out/r02c29/counters.txt; }
pass=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  ok=""
  for c in $set; do base=${c%_sum}; if have $base || have $c; then ok="$ok $c"; fi; done
  pass=$((pass+1))
  [ -z "$ok" ] && continue
  run 120 pmc_bptt_$pass timeout -s KILL 100 rocprofv3 --pmc $ok -d $R/gpurun_out/r02c29/bptt/pmc_$pass -o run --output-format csv -- python tools/probe_bptt.py --B 2048 --N 100 --reps 2
  run 120 pmc_td_$pass timeout -s KILL 100 rocprofv3 --pmc $ok -d $R/gpurun_out/r02c29/td/pmc_$pass -o run --output-format csv -- python tools/probe_td_fused.py 2048
done
