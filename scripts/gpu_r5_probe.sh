#!/bin/bash
# Round-5 B=1 anatomy: per-launch HIP-event table of one eager B=1 denoise step (tags = GEMM shapes and
# plans), the graph-replayed launch floor, and a short default bench for the baseline on this box.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
TAIR_PROFILE_CSV=gpurun_out/r05_launches_b1.csv step prof_b1 300 python -u bench.py --profile-only --sampling-steps 2 --batch 1 || exit 1
step floor 120 python -u tools/launch_floor.py || exit 1
step bench_b1 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe || exit 1
step sweep_b1 600 python -u tools/gemm_sweep.py --batch 1 --sweep || exit 1
