#!/bin/bash
# Round-5: XCD-aware attention block order (product) vs round 4's order (noremap variant): attention sweeps at
# B=64 and B=1, attention tests, configs[2] with each.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-200; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step atests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
step attn64_remap 300 python -u tools/attn_bench.py --batch 64 --reps 5 || exit 1
TAIR_LIB_VARIANT=noremap step attn64_noremap 300 python -u tools/attn_bench.py --batch 64 --reps 5 || exit 1
step attn1_remap 300 python -u tools/attn_bench.py --batch 1 || exit 1
step cfg2_remap 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=noremap step cfg2_noremap 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
