#!/usr/bin/env bash
# A round's GPU check on the current tree: the GPU test suite, smoke(), the driver's bench
# command, and a rocprofv3 kernel trace of that same command (-> the headline's launches and
# the bench line side by side, tools/rocprof_headline.py).  On the GPU box:
#   gpurun -- 'bash tools/gpu_check.sh'        (SKIP_TESTS=1 / SKIP_PROF=1 to leave parts out)
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log
if [ -z "${SKIP_TESTS:-}" ]; then
  run 1000 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --maxfail 20 -rA
  run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
fi
run 400 bench python -u bench.py --steps 20 --warmup 5
if [ -z "${SKIP_PROF:-}" ]; then
  rm -rf gpurun_out/prof_kt
  run 400 prof_kt rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt -o run --output-format csv -- python bench.py --steps 20 --warmup 5
  run 60 headline python tools/rocprof_headline.py gpurun_out/prof_kt/run_kernel_trace.csv gpurun_out/prof_kt.log --steps 20 --warmup 5 --stats gpurun_out/prof_kt/run_kernel_stats.csv
fi
