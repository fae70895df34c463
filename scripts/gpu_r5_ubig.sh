#!/bin/bash
# Round-5 A/B: (1) two epilogue items in flight per thread on the 8-wave 256x128 / 128x256 tiles (ubig2
# variant); (2) attention key splits merged in-kernel (product) vs the merge kernel (TAIR_ATTN_INK=0).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c90-150; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step ktests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step b1_ink 300 $B || exit 1
TAIR_ATTN_INK=0 step b1_noink 300 $B || exit 1
step b1_ink2 300 $B || exit 1
TAIR_ATTN_INK=0 step b1_noink2 300 $B || exit 1
step b16_u1 300 $B --batch 16 || exit 1
TAIR_LIB_VARIANT=ubig2 step b16_u2 300 $B --batch 16 || exit 1
step cfg2_u1 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=ubig2 step cfg2_u2 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
step ctests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cldm_gpu.py || exit 1
