#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
TAIR_PROFILE_CSV=gpurun_out/prof_b1.csv run prof1 300 python bench.py --profile-only --batch 1
TAIR_PROFILE_CSV=gpurun_out/prof_b8.csv run prof8 300 python bench.py --profile-only --batch 8
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof -o r01 -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile
ls -R gpurun_out/rocprof | head -20
