#!/bin/bash
# Round-5: cross-attention plan (16 queries per wave) -- attention tests, B=1 bench x2, configs[2].
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c90-150; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step atests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step b1_x1 300 $B || exit 1
step b1_x2 300 $B || exit 1
step cfg2_x 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
