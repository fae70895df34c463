#!/bin/bash
# Per-launch event tables of one eager B=64 denoise step, halo tiles on and off.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
B="--batch 64 --tiles 64 --steps 1 --warmup 1 --no-cpu-baseline --no-stage3-probe"
TAIR_PROFILE_CSV=gpurun_out/r4_b64_launch_halo.csv timeout -k 10 300 python -u bench.py $B > gpurun_out/r4_b64_csv_halo.log 2>&1 || exit 1
#TAIR_HALO=0 TAIR_PROFILE_CSV=gpurun_out/r4_b64_launch_tile.csv timeout -k 10 300 python -u bench.py $B > gpurun_out/r4_b64_csv_tile.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --batch 16 --tiles 16 --steps 2 --warmup 1 --no-cpu-baseline --no-stage3-probe > gpurun_out/r4_b16_halo3.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --batch 64 --tiles 64 --steps 1 --warmup 1 --no-cpu-baseline --no-stage3-probe > gpurun_out/r4_b64_halo3.log 2>&1 || exit 1
