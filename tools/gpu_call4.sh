source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 guard python -u -m pytest tests/test_gpu_x3_guard.py -q -p no:cacheprovider --timeout 300 --timeout-method thread -rA
run 900 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --maxfail 20
run 300 tb_guard python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_noguard env DPAC_X3_GUARD=0 python -u tools/train_bench.py --iters 30 --warmup 5
run 300 tb_guard2 python -u tools/train_bench.py --iters 30 --warmup 5
for v in ring7 ring5 ring2; do
  run 300 bptt_$v env DPAC_LIB=tools/variants/libdpac_$v.so python -u tools/probe_bptt.py --B 2048,4096 --only fwd,bwd
done
run 300 bptt_base python -u tools/probe_bptt.py --B 2048,4096
run 300 rows python -u tools/probe_x3.py
rm -rf gpurun_out/prof_kt
run 400 prof_kt rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_kt -o run --output-format csv -- python bench.py --steps 20 --warmup 5
run 60 headline python tools/rocprof_headline.py gpurun_out/prof_kt/run_kernel_trace.csv gpurun_out/prof_kt.log --steps 20 --warmup 5 --stats gpurun_out/prof_kt/run_kernel_stats.csv
