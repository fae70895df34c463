#!/bin/bash
# GPU test runner for gpurun: each step time-limited; stop on crash/timeout, continue on test failures.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 25 "gpurun_out/$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name exited $rc"; exit $rc; fi
  return 0
}
