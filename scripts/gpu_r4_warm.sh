#!/bin/bash
# B=1 GEMMs: in-network per-launch shapes, then each shape timed warm (weights L2/MALL-resident, repeated launches).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
TAIR_PROFILE_CSV=gpurun_out/r4_b1_launch.csv timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-stage3-probe > gpurun_out/r4_b1_launch.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/gemm_bench.py gpurun_out/r4_b1_launch.csv --reps 15 > gpurun_out/r4_b1_warm.log 2>&1 || exit 1
tail -1 gpurun_out/r4_b1_warm.log
