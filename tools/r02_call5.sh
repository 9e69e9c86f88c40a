# Round-2 call 5: static-K MFMA layers (mfma_rows16_kms) in the fused forward and BPTT,
# forced inlining (no scratch), the bwd2 kernel; variants for ring depth and ablations.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 300 nn_tests python -u -m pytest tests/test_gpu_rollout_nn.py tests/test_gpu_models.py tests/test_gpu_mlp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 probe_def python -u tools/probe_bptt.py --B 2048,4096 --N 100 --only fwd,bwd
DPAC_BPTT=1 run 200 probe_bwd1 python -u tools/probe_bptt.py --B 2048 --N 100 --only bwd
for v in kms0 kmspg2 kmspg4; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 probe_$v python -u tools/probe_bptt.py --B 2048 --N 100 --only fwd,bwd
done
for v in nohelp nowr; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 probe_$v python -u tools/probe_bptt.py --B 2048 --N 100 --only bwd
done
run 200 train_bench python -u tools/train_bench.py --iters 20 --dtype float32
