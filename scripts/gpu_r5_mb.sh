#!/bin/bash
# Round-5: configs[2] (256 tiles, stitch) at micro-batches of 128 and 256 against 64.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c90-160; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
C="python -u bench.py --tiles 256 --stitch --no-cpu-baseline --no-stage3-probe --no-profile"
step mb128 600 $C --batch 128 || exit 1
step mb64 600 $C --batch 64 || exit 1
step mb256 600 $C --batch 256 || exit 1
