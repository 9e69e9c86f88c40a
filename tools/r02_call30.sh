# Round-2 call 30: LDS row stride +8 instead of +4 elements (gfx950 ds_read_b128 lane groups:
# stride = 8 mod 64 dwords makes the A-operand reads conflict-free) in the row-parallel MLP
# kernels (pad8), the NN rollout / BPTT (nnpad8), both (both8): tests, then timings.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
DPAC_LIB=$R/tools/variants/libdpac_both8.so run 300 tests_both8 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlp.py tests/test_gpu_td_fused.py tests/test_gpu_rollout_nn.py tests/test_gpu_models.py
run 200 rows_default python -u tools/probe_rows.py 204800
DPAC_LIB=$R/tools/variants/libdpac_pad8.so run 200 rows_pad8 python -u tools/probe_rows.py 204800
run 200 bptt_default python -u tools/probe_bptt.py --B 2048,4096 --N 100 --reps 10
DPAC_LIB=$R/tools/variants/libdpac_nnpad8.so run 200 bptt_nnpad8 python -u tools/probe_bptt.py --B 2048,4096 --N 100 --reps 10
run 200 train_default python -u tools/train_bench.py --iters 20 --batch 2048
DPAC_LIB=$R/tools/variants/libdpac_both8.so run 200 train_both8 python -u tools/train_bench.py --iters 20 --batch 2048
run 200 train_default2 python -u tools/train_bench.py --iters 20 --batch 2048
DPAC_LIB=$R/tools/variants/libdpac_both8.so run 200 train_both8b python -u tools/train_bench.py --iters 20 --batch 2048
