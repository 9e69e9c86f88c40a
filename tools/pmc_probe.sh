# PMC passes (one counter set per run) over the MLP kernels' probes.
source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log; rm -rf gpurun_out/pmc_*
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
run 200 probe_rows python -u tools/probe_rows.py
run 200 probe_nn python -u tools/probe_nn.py --B 2048 --N 100
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"; do
  tag=$(echo $set | md5sum | cut -c1-6)
  run 120 pmc_nn_$tag timeout -s KILL 100 rocprofv3 --pmc $set -d gpurun_out/pmc_nn_$tag -o run --output-format csv -- python tools/probe_nn.py --B 2048 --N 100 --reps 2
  run 120 pmc_rows_$tag timeout -s KILL 100 rocprofv3 --pmc $set -d gpurun_out/pmc_rows_$tag -o run --output-format csv -- python tools/probe_rows.py 204800
done
