#!/usr/bin/env bash
# Run GPU steps in order; each step: "<timeout_s> <logname> <command...>".
# Continues past ordinary failures (exit 1/2/4/5) but stops at anything that
# looks like a fault, abort, segfault or timeout (124, 134, 137, 139, >128), and at a step
# whose log reports a GPU memory fault (a Python process exits 1 on one).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tmo=$1 log=$2; shift 2
  echo "=== [$log] $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$log.log" 2>&1
  local rc=$?
  echo "=== [$log] exit $rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$log.log"
  if grep -q "illegal memory access\|hipErrorIllegalAddress\|Memory access fault\|HSA_STATUS_ERROR" "gpurun_out/$log.log"; then
    echo "GPU fault in step $log: stopping" | tee -a gpurun_out/steps.log
    exit 99
  fi
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "fatal exit $rc in step $log: stopping" | tee -a gpurun_out/steps.log
    exit $rc
  fi
  return 0
}
