#!/bin/bash
# Round-5: 64 queries per wave (QSETS 4) in the attention kernel: tests, plan sweep at B=64 and B=1.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-150; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step atests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
step attn64_q4 400 python -u tools/attn_bench.py --batch 64 --reps 5 || exit 1
step attn1_q4 300 python -u tools/attn_bench.py --batch 1 || exit 1
