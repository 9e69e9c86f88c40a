#!/usr/bin/env bash
# Named GPU recipes, one gpurun call each (they replace rounds 2-4's one-off tools/gpu_call*.sh):
#
#   bash tools/gpu_recipes.sh check      GPU test suite, smoke(), the driver's bench command, and a
#                                        rocprofv3 kernel trace of that command beside its line
#                                        (SKIP_TESTS=1 / SKIP_PROF=1 leave parts out)
#   bash tools/gpu_recipes.sh profile    the round's profiles/ evidence (tools/profile_round.sh)
#   bash tools/gpu_recipes.sh dp         bench.py --gpus 2 on one GPU (gloo rehearsal) and N = 1
#   bash tools/gpu_recipes.sh seeds "gpu32:101 gpu64:101"     full lqr_d20 runs (tools/seed_spread.sh)
#   bash tools/gpu_recipes.sh ab "<pytest files>" "<probe cmd>" SPEC...
#        A/B of timing variants: SPEC is `base`, `lib:<name>` (tools/variants/libdpac_<name>.so,
#        built by tools/build_variants.sh) or `env:KEY=VAL`.  Every non-base variant first runs
#        the given tests; then each SPEC runs the probe command twice, in alternation.
#        e.g. bash tools/gpu_recipes.sh ab tests/test_gpu_mlp.py \
#               "python -u tools/train_bench.py --iters 30 --warmup 5" base lib:rt3 env:DPAC_NX_ROWS=8
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$PWD
rm -f gpurun_out/steps.log

spec_env() {  # SPEC -> the `env` arguments that select it
  case "$1" in
    base) echo "" ;;
    lib:*) echo "DPAC_LIB=tools/variants/libdpac_${1#lib:}.so" ;;
    env:*) echo "${1#env:}" ;;
  esac
}

case "${1:-check}" in
  check)
    if [ -z "${SKIP_TESTS:-}" ]; then
      run 1000 pytest_gpu python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --maxfail 20 -rA
      run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
    fi
    run 400 bench python -u bench.py --gpus 1 --steps 20 --warmup 5
    if [ -z "${SKIP_PROF:-}" ]; then
      rm -rf gpurun_out/prof_kt
      run 400 prof_kt rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5
      run 60 headline python tools/rocprof_headline.py gpurun_out/prof_kt/run_kernel_trace.csv gpurun_out/prof_kt.log --steps 20 --warmup 5 --stats gpurun_out/prof_kt/run_kernel_stats.csv
    fi
    ;;
  profile)
    bash tools/profile_round.sh
    ;;
  dp)
    run 300 bench1 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline
    DPAC_DIST_BACKEND=gloo run 300 bench2_gloo python -u bench.py --gpus 2 --steps 20 --warmup 3
    ;;
  seeds)
    bash tools/seed_spread.sh "$2"
    ;;
  ab)
    tests=$2; probe=$3; shift 3
    for s in "$@"; do
      [ "$s" = base ] && continue
      run 600 "tests_${s//[:=\/]/_}" env $(spec_env "$s") python -u -m pytest $tests -q -p no:cacheprovider --timeout 120 --timeout-method thread -x
    done
    for rep in 1 2; do
      for s in "$@"; do
        run 300 "probe_${s//[:=\/]/_}_$rep" env $(spec_env "$s") $probe
      done
    done
    ;;
  *)
    echo "unknown recipe $1" >&2; exit 2 ;;
esac
