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
