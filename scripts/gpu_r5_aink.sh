#!/bin/bash
# Round-5 A/B: attention key splits merged in-kernel (batched sc1 loads) vs the merge kernel (TAIR_ATTN_INK=0).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c90-150; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step ktests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
step attn1_ink 300 python -u tools/attn_bench.py --batch 1 || exit 1
TAIR_ATTN_INK=0 step attn1_noink 300 python -u tools/attn_bench.py --batch 1 || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step b1_ink 300 $B || exit 1
TAIR_ATTN_INK=0 step b1_noink 300 $B || exit 1
step b1_ink2 300 $B || exit 1
TAIR_ATTN_INK=0 step b1_noink2 300 $B || exit 1
