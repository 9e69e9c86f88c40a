# Round-2 call 4: k_rollout_nn_bwd2 with the faster writer / spread stager; helper ablations.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 300 nn_tests python -u -m pytest tests/test_gpu_rollout_nn.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bitwise or bptt"
run 200 probe_bptt2 python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only bwd
DPAC_BPTT=1 run 200 probe_bptt1 python -u tools/probe_bptt.py --B 2048 --N 100 --only bwd
for v in nost nowr nohelp; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 probe_bptt_$v python -u tools/probe_bptt.py --B 2048 --N 100 --only bwd
done
