# Round-2 first GPU call: GPU tests + smoke + bench on the rebuilt tree, the actor-step
# kernels timed one by one (tools/probe_bptt.py), BPTT ablation builds, a kernel trace and
# PMC passes (one counter set per run) over the BPTT / forward / parameter-gradient kernels.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
rm -rf gpurun_out/r02c1
mkdir -p gpurun_out/r02c1
rocprofv3 -L > gpurun_out/r02c1/counters.txt 2>&1 || true
run 600 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
run 300 bench python bench.py --steps 200 --warmup 20
run 200 probe_bptt python -u tools/probe_bptt.py --B 2048,4096,8192 --N 100
for v in z g s m zgs; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 probe_bptt_$v python -u tools/probe_bptt.py --B 2048 --N 100 --only bwd
done
run 200 prof_bptt rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r02c1/kt -o run --output-format csv -- python tools/probe_bptt.py --B 2048 --N 100 --reps 5
have() { grep -q "\b$1\b" gpurun_out/r02c1/counters.txt; }
pass=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  ok=""
  for c in $set; do base=${c%_sum}; if have $base || have $c; then ok="$ok $c"; fi; done
  pass=$((pass+1))
  echo "pass $pass:$ok" >> gpurun_out/r02c1/passes.txt
  [ -z "$ok" ] && continue
  run 120 pmc_$pass timeout -s KILL 100 rocprofv3 --pmc $ok -d $R/gpurun_out/r02c1/pmc_$pass -o run --output-format csv -- python tools/probe_bptt.py --B 2048 --N 100 --reps 2
done
