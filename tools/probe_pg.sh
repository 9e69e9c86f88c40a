source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_pg
run 200 probe_pg python -u tools/probe_pg.py
run 200 prof_pg rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pg -o run --output-format csv -- python -u tools/probe_pg.py
