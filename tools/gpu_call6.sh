# round 4 call 6: the training iteration's timeline, parameter-gradient variants
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log; rm -rf gpurun_out/prof_train
run 300 prof_train rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run --output-format csv -- python tools/train_bench.py --iters 3 --warmup 1 --dtype float32
run 60 timeline python tools/iter_timeline.py gpurun_out/prof_train/run_kernel_trace.csv
run 300 pg_base python -u tools/probe_x3.py 204800 x3 --pg
run 300 pg_rowdesc env DPAC_LIB=tools/variants/libdpac_pgrowdesc.so python -u tools/probe_x3.py 204800 x3 --pg
run 300 pg_nw16 env DPAC_PGX_NW=16 python -u tools/probe_x3.py 204800 x3 --pg
run 300 pg_rowdesc_nw16 env DPAC_PGX_NW=16 DPAC_LIB=tools/variants/libdpac_pgrowdesc.so python -u tools/probe_x3.py 204800 x3 --pg
run 300 tb_base python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_rowdesc env DPAC_LIB=tools/variants/libdpac_pgrowdesc.so python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_nw16 env DPAC_PGX_NW=16 python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_min64 env DPAC_LIB=tools/variants/libdpac_minrows64.so python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_min32 env DPAC_LIB=tools/variants/libdpac_minrows32.so python -u tools/train_bench.py --iters 30 --warmup 5
