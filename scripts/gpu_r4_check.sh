#!/bin/bash
# Round-4 GPU check: (optional) build the library from source on the box and time it, then the given
# tests, then the default bench.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
if [ "${SRC_BUILD-0}" = "1" ]; then
  mkdir -p /tmp/tair_prebuilt && mv tair_amd/libtair_cldm.so /tmp/tair_prebuilt/ && rm -rf build/obj
  step build_from_source 900 bash -c 'time python -m tair_amd.build --jobs 16' || exit 1
fi
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
if [ -n "${TESTS-}" ]; then
  step pytest 1100 python -u -m pytest ${TESTS} ${K:+-k "$K"} $([ -n "${NOX-}" ] && echo --maxfail=50 || echo -x) -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider || exit 1
fi
if [ -n "${BENCH-}" ]; then
  step bench 600 python -u bench.py ${BENCH} || exit 1
  grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench.json
fi
