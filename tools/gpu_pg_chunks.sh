source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_pg*
run 200 prof_pg_base rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_pg_base -o run --output-format csv -- python -u tools/probe_pg.py
for v in ch256 ch512; do
  DPAC_LIB=$PWD/tools/variants/libdpac_$v.so run 200 prof_pg_$v rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_pg_$v -o run --output-format csv -- python -u tools/probe_pg.py
done
DPAC_LIB=$PWD/tools/variants/libdpac_ch256.so run 300 train_bench32_ch256 python -u tools/train_bench.py --iters 20 --dtype float32
DPAC_LIB=$PWD/tools/variants/libdpac_ch512.so run 300 train_bench32_ch512 python -u tools/train_bench.py --iters 20 --dtype float32
