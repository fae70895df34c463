#!/bin/bash
# Round-5 A/B: attention with the Q-fragment loads completed before the loop (product) vs round-5 earlier
# (attnold variant): attention timing, tests, B=1 bench and configs[2].
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c90-150; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step atests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
step abl_new 200 python -u tools/attn_ablate.py --tag new || exit 1
TAIR_LIB_VARIANT=attnold step abl_old 200 python -u tools/attn_ablate.py --tag old || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step b1_new 300 $B || exit 1
TAIR_LIB_VARIANT=attnold step b1_old 300 $B || exit 1
step cfg2_new 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=attnold step cfg2_old 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
