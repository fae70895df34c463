#!/bin/bash
# Round-5: 8-wave tiles for the B >= 64 short-K linears (TAIR_SK_WIDE) vs the 2-stage 64x64 plan
# (libtair_cldm_skw0.so): GEMM kernel tests, forward / golden tests, configs[2] paired.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step ktests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" || exit 1
step ftests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_golden_gpu.py tests/test_cldm_gpu.py || exit 1
step cfg2_wide 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=skw0 step cfg2_narrow 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
