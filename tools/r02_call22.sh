# Round-2 call 22 (rebuilt container): smoke on the rebuilt library, then the row-parallel
# MLP kernels (critic G network, R = N*B = 204 800 rows) with and without the per-workgroup
# rotation of the waves' column-tile sets (DPAC_MR_ROT), the narrow parameter-gradient
# layers forked onto a side stream (DPAC_PG_FORK), then the training iteration.
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
DPAC_LIB=$R/tools/variants/libdpac_rot1fork.so run 400 tests_rot1fork python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlp.py tests/test_gpu_models.py
run 200 rows_default python -u tools/probe_rows.py 204800
for v in rot1 rot2; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 rows_$v python -u tools/probe_rows.py 204800
done
run 200 train_default python -u tools/train_bench.py --iters 20 --batch 2048
for v in rot1 rot2 fork rot1fork; do
  DPAC_LIB=$R/tools/variants/libdpac_$v.so run 200 train_$v python -u tools/train_bench.py --iters 20 --batch 2048
done
run 200 train_default_again python -u tools/train_bench.py --iters 20 --batch 2048
