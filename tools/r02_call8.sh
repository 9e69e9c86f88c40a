# Round-2 call 8: rollout (nt x stores now default) cold/MALL, the 32-lane split; BPTT
# ablations (stager off, writer off, both, no weight loads); clock trace of the NN kernels;
# the training iteration with the BPTT claiming its CUs' whole LDS.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 120 roll_cold python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100 --sets 5
run 120 roll_mall python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100 --sets 1
DPAC_LIB=$R/tools/variants/libdpac_lanes32.so run 120 roll_lanes32 python -u tools/probe_rollout.py --B 4096,16384 --N 200 --reps 100 --sets 5
run 200 probe_def python -u tools/probe_bptt.py --B 2048 --N 100 --only fwd,bwd
for v in nost nowr nohelp nnw; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 probe_$v python -u tools/probe_bptt.py --B 2048 --N 100 --only fwd,bwd
done
DPAC_LIB=$R/tools/variants/libdpac_trace.so run 200 trace python -u tools/probe_trace.py --B 2048 --N 100
run 200 train_def python -u tools/train_bench.py --iters 20 --dtype float32
DPAC_BPTT_LDS=max run 200 train_ldsmax python -u tools/train_bench.py --iters 20 --dtype float32
