#!/bin/bash
# Round-5 A/B: epilogue items loop compiled per feature set (product) vs the generic loop only (nosets),
# B=1 and B=16 bench, then the kernel + network GPU tests on the product library.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step bench_sets1 300 $B || exit 1
TAIR_LIB_VARIANT=nosets step bench_nosets1 300 $B || exit 1
step bench_sets2 300 $B || exit 1
TAIR_LIB_VARIANT=nosets step bench_nosets2 300 $B || exit 1
step bench16_sets 300 $B --batch 16 || exit 1
TAIR_LIB_VARIANT=nosets step bench16_nosets 300 $B --batch 16 || exit 1
step tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_cldm_gpu.py || exit 1
step golden 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_golden_gpu.py || exit 1
