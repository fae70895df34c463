#!/bin/bash
# Round-5: attention K/V prefetch depth (ATTN_PD 3 product vs variants pd1 = round 4, pd2): attention sweeps
# at B=1 and B=64, B=1 bench with each, attention tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-200; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step atests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
step attn_pd3 300 python -u tools/attn_bench.py --batch 1 || exit 1
TAIR_LIB_VARIANT=pd1 step attn_pd1 300 python -u tools/attn_bench.py --batch 1 || exit 1
TAIR_LIB_VARIANT=pd2 step attn_pd2 300 python -u tools/attn_bench.py --batch 1 || exit 1
step attn64_pd3 300 python -u tools/attn_bench.py --batch 64 --reps 5 || exit 1
TAIR_LIB_VARIANT=pd1 step attn64_pd1 300 python -u tools/attn_bench.py --batch 64 --reps 5 || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step bench_pd3 300 $B || exit 1
TAIR_LIB_VARIANT=pd1 step bench_pd1 300 $B || exit 1
TAIR_LIB_VARIANT=pd2 step bench_pd2 300 $B || exit 1
