#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
TAIR_NO_FORK=1 run bench_nofork 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile
TAIR_PROFILE_CSV=gpurun_out/prof_b1.csv run prof1 300 python bench.py --profile-only --batch 1
run gemmsweep 900 python tools/gemm_bench.py gpurun_out/prof_b1.csv --sweep --reps 10 --out gpurun_out/gemm_b1_v4.json
