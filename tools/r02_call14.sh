# Round-2 call 14: non-temporal cache policy for the BPTT's G stores (writer wave), the
# stager's LDS-DMA, and the forward's z saves; the training iteration with each.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 200 probe_base python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only fwd,bwd
for v in wnt snt fnt allnt; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 probe_$v python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only fwd,bwd
done
run 200 train_base python -u tools/train_bench.py --iters 20 --dtype float32
DPAC_LIB=$R/tools/variants/libdpac_allnt.so run 200 train_allnt python -u tools/train_bench.py --iters 20 --dtype float32
