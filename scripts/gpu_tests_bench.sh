#!/bin/bash
# GPU tests (optionally a subset: TESTS="tests/x.py ...") then bench runs given as "B:T" pairs in
# BENCH ("1:0 8:0 64:256" = batch 1; batch 8; 256 tiles in micro-batches of 64).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
if [ -n "${TESTS-}" ]; then
  step pytest 900 python -u -m pytest ${TESTS} ${K:+-k "$K"} -x -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider || exit 1
fi
for bt in ${BENCH-}; do
  b=${bt%%:*}; t=${bt##*:}
  extra=""; [ "$t" != "0" ] && extra="--tiles $t --stitch"
  step bench_b${b}_t${t} 900 python -u bench.py --steps ${STEPS:-2} --warmup 1 --batch $b $extra ${BENCH_FLAGS-} || exit 1
done
