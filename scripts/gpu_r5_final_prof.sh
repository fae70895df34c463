#!/bin/bash
# Round-5 evidence on the current code: B=1 and B=64 rocprof + PMC profiles (per-class algorithmic bytes),
# configs[3] and configs[4] benches, the fp8 B=1 profile for configs[4]'s traffic field.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c90-200; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
B=1 TAG=r05b1 timeout -k 10 900 bash scripts/gpu_profile.sh || exit 1
B=64 TAG=r05b64 timeout -k 10 900 bash scripts/gpu_profile.sh || exit 1
B=1 FP8=1 TAG=r05b1_fp8 timeout -k 10 900 bash scripts/gpu_profile.sh || exit 1
step cfg3 600 python -u bench.py --config 3 --no-cpu-baseline --no-stage3-probe || exit 1
step cfg4 600 python -u bench.py --config 4 --no-cpu-baseline || exit 1
