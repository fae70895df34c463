#!/bin/bash
# Round-5: attention keys split only from 32 key tiles (TAIR_ATTN_SPLIT_MIN) vs always (libtair_cldm_sm0.so):
# attention tests, B=1 bench paired x2.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step atests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
for r in 1 2; do
  step b1_sm32_$r 300 $B || exit 1
  TAIR_LIB_VARIANT=sm0 step b1_sm0_$r 300 $B || exit 1
done
