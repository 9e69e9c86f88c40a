# Round-2 call 11: B-ring depth (PG 3, 4) now that the ring is pinned; z staged through
# the stager's VGPRs instead of LDS-DMA.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 200 probe_base python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only fwd,bwd
for v in pg3 pg4 zreg zregpg3; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 probe_$v python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only fwd,bwd
done
rocprofv3 -L > gpurun_out/counters_r02.txt 2>&1 || true
ic=""
for c in SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES; do grep -q "\b$c\b" gpurun_out/counters_r02.txt && ic="$ic $c"; done
echo "icache pass:$ic" >> gpurun_out/steps.log
[ -n "$ic" ] && run 120 pmc_icache timeout -s KILL 100 rocprofv3 --pmc $ic -d $R/gpurun_out/pmc_icache -o run --output-format csv -- python tools/probe_bptt.py --B 2048 --N 100 --reps 2 --only fwd,bwd
