#!/bin/bash
# Round-5 evidence on the final attention code: B=1 and B=64 rocprof + PMC profiles, configs[2] and configs[3].
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c90-200; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
B=1 TAG=r05fb1 timeout -k 10 900 bash scripts/gpu_profile.sh || exit 1
B=64 TAG=r05fb64 timeout -k 10 900 bash scripts/gpu_profile.sh || exit 1
step cfg2_final 600 python -u bench.py --config 2 --no-stage3-probe || exit 1
step cfg3_final 600 python -u bench.py --config 3 --no-cpu-baseline --no-stage3-probe || exit 1
