source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_pg_*
run 200 probe_rows python -u tools/probe_rows.py
DPAC_LIB=$PWD/tools/variants/libdpac_rt2.so run 200 probe_rows_rt2 python -u tools/probe_rows.py
run 200 prof_pg_base rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_pg_base -o run --output-format csv -- python -u tools/probe_pg.py
for v in sr32 sr8; do
  DPAC_LIB=$PWD/tools/variants/libdpac_$v.so run 200 prof_pg_$v rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_pg_$v -o run --output-format csv -- python -u tools/probe_pg.py
done
