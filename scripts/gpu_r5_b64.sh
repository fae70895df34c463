#!/bin/bash
# Round-5 batched evidence: configs[2] bench (B=64 micro-batches + stitch), then the B=64 rocprof + PMC profile
# with per-key algorithmic bytes.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step cfg2 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe || exit 1
B=64 TAG=r05b64 timeout -k 10 1000 bash scripts/gpu_profile.sh || exit 1
